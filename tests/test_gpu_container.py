"""GPU parity of the RCB1 container: compress() on the GPU against the
oracle's container bytes (oracle/container.py over oracle/cpu.py streams), byte for byte, and
decompress() round trips, including ragged last chunks, the adaptive model, empty input and
malformed containers."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402
from oracle import container as OC  # noqa: E402
from oracle import cpu  # noqa: E402
from oracle import model_build as O  # noqa: E402
from gpu_helpers import dev  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


def zipf_data(n, seed):
    c, _, _ = synth.zipf_table()
    rng = np.random.default_rng(seed)
    return rng.choice(256, n, p=np.asarray(c, float) / np.sum(c)).astype(np.uint8)


@pytest.mark.parametrize("n,chunk", [(16, 16), (10000, 3000), (65536 * 3 + 5, 65536),
                                     (50000, 4096), (1, 65536)])
def test_static_container_bytes_match_oracle(ctx, n, chunk):
    c, cum, total = synth.zipf_table()
    data = zipf_data(n, n)
    m = rc.StaticModel(c, cum, total)
    blob = rc.compress(dev(data), chunk_size=chunk, model=m)
    want = OC.compress_static(c, cum, total, data, chunk)
    assert bytes(blob.cpu().numpy()) == want
    assert torch.equal(rc.decompress(blob), dev(data))


def test_sample_container(ctx):
    data = np.array([2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5], np.uint8)
    m = rc.StaticModel([1, 5, 2, 0, 2, 2, 1, 1, 1, 1])
    blob = rc.compress(dev(data), chunk_size=16, model=m)
    assert bytes(blob.cpu().numpy()) == OC.compress_static(
        [1, 5, 2, 0, 2, 2, 1, 1, 1, 1], [0, 1, 6, 8, 8, 10, 12, 13, 14, 15], 16, data, 16)
    assert list(rc.decompress(blob).cpu().numpy()) == list(data)


@pytest.mark.parametrize("T", [1 << 16, 4096, 1 << 20])
def test_auto_model_container(ctx, T):
    data = zipf_data(300000, T)
    blob = rc.compress(dev(data), chunk_size=65536, target_total=T)
    c, cum, total = O.quantize_counts(np.bincount(data, minlength=256), T, O.Q_ALL_SYMBOLS)
    assert bytes(blob.cpu().numpy()) == OC.compress_static(c, cum, total, data, 65536)
    assert torch.equal(rc.decompress(blob), dev(data))


def test_adaptive_container(ctx):
    data = zipf_data(70000, 5)
    m = rc.AdaptiveModel(256, **rc.ADAPTIVE_DEFAULTS)
    blob = rc.compress(dev(data), chunk_size=16384, model=m)
    chunks = [bytes(data[i:i + 16384]) for i in range(0, len(data), 16384)]
    codes = []
    for ch in chunks:
        f, b, _ = cpu.encode_adaptive(256, 32, 57343, 256, ch)
        assert f == 0
        codes.append(b)
    assert bytes(blob.cpu().numpy()) == OC.build(1, 256, chunks, codes, adaptive=(32, 57343, 256))
    assert torch.equal(rc.decompress(blob), dev(data))


def test_empty_input(ctx):
    m = rc.StaticModel(*synth.uniform_table())
    blob = rc.compress(torch.empty(0, dtype=torch.uint8, device="cuda"), model=m)
    inf = rc.container.info(blob)
    assert inf.n_chunks == 0 and inf.n_syms == 0 and blob.numel() == inf.container_bytes
    assert rc.decompress(blob).numel() == 0


def test_large_round_trip(ctx):
    n, L = 4096, 65536
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    c, _, _ = synth.zipf_table()
    synth.fill(ctx, 11, synth.inverse_cdf(c), syms, L, n)
    blob = rc.compress(syms)
    assert blob.numel() < 0.7 * syms.numel()
    assert torch.equal(rc.decompress(blob), syms)


def test_malformed_containers(ctx):
    data = zipf_data(20000, 3)
    m = rc.StaticModel(*synth.zipf_table())
    blob = rc.compress(dev(data), chunk_size=4096, model=m)
    inf = rc.container.info(blob)
    with pytest.raises(rc.ContainerError):  # truncated
        rc.decompress(blob[:-16].clone())
    bad = blob.clone()  # a code length that no longer adds up to the payload
    bad[inf.index_off + 8] = (int(bad[inf.index_off + 8]) + 16) & 255
    with pytest.raises(rc.ContainerError):
        rc.decompress(bad)
    bad = blob.clone()  # symbol count changed
    bad[inf.index_off] = (int(bad[inf.index_off]) + 1) & 255
    with pytest.raises(rc.ContainerError):
        rc.decompress(bad)
    bad = blob.clone()  # table no longer sums to total
    bad[inf.table_off] = (int(bad[inf.table_off]) + 1) & 255
    with pytest.raises(rc.ContainerError):
        rc.decompress(bad)
    bad = blob.clone()  # corrupt payload byte: decodes (no framing error) to different symbols
    bad[inf.payload_off + 20] ^= 0x55
    out = None
    try:
        out = rc.decompress(bad)
    except rc.RangeCoderError:
        pass
    assert out is None or not torch.equal(out, dev(data))
