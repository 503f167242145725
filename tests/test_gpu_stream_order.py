"""Stream ordering of the batch entry points (include/range_coder.h: rc_ctx_set_stream,
rc_ctx_reset_stream, rc_ctx_synchronize).

The Python mirror launches on torch's current stream (Context.bind_stream before every batch
call), so a torch producer and the coder on a side stream need no synchronisation between them;
a C-ABI caller that reset the context to its own stream orders work by rc_ctx_synchronize.  Each
case keeps the side stream busy with a long matmul chain in front of the producer, so a launch
that escaped the stream order would read the input before it was written.  Bytes are checked
against the C oracle (encoder.rs:24-46 per chunk) and the decode against the input
(decoder.rs:38-54)."""
import ctypes

import numpy as np
import pytest
import torch

import range_coder_rust_amd as rc
from range_coder_rust_amd import _native as N
from range_coder_rust_amd import synth

pytestmark = pytest.mark.gpu

N_CH, L = 256, 16384


def _busy(side):
    """Queue ~tens of ms of matmuls on `side` (the producer below waits behind them)."""
    with torch.cuda.stream(side):
        a = torch.randn(4096, 4096, device="cuda")
        for _ in range(24):
            a = (a @ a).clamp_(-1, 1)
    return a


def _oracle_chunks(c, cum, total, host_syms, ks):
    from oracle import cpu
    out = {}
    for k in ks:
        f, b, _ = cpu.encode(c, cum, total, host_syms[k * L:(k + 1) * L])
        assert f == 0
        out[k] = b
    return out


def test_batch_calls_follow_the_torch_stream():
    ctx = rc.Context(0)
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total, ctx=ctx)
    cap = rc.slot_capacity(L, 12.0)  # (chunk 0 is uniform data under the Zipf model: ~10 bits)
    side = torch.cuda.Stream()
    keep = _busy(side)
    with torch.cuda.stream(side):
        syms = torch.empty(N_CH * L, dtype=torch.uint8, device="cuda")
        # the producer: synth.fill (a kernel of the library) then a torch op rewriting chunk 0
        synth.fill(ctx, 0x5EED0777, synth.inverse_cdf(c), syms, L, N_CH)
        syms[:L] = torch.arange(L, device="cuda").remainder(256).to(torch.uint8)
        so = torch.arange(N_CH + 1, dtype=torch.int64, device="cuda") * L
        oo = torch.arange(N_CH + 1, dtype=torch.int64, device="cuda") * cap
        out = torch.empty(N_CH * cap, dtype=torch.uint8, device="cuda")
        ol, fe = rc.encode_batch(m, syms, so, out, oo)
        dec = torch.empty_like(syms)
        fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
        same = torch.equal(dec, syms)  # (on the side stream too)
    side.synchronize()
    del keep
    assert not fe.any() and not fd.any()
    assert same
    h = syms.cpu().numpy()
    want = _oracle_chunks(c, cum, total, h, [0, 1, N_CH - 1])
    hb, hl = out.cpu().numpy(), ol.cpu().numpy()
    for k, b in want.items():
        assert bytes(hb[k * cap:k * cap + int(hl[k])]) == b, f"chunk {k}"


def test_reset_stream_then_synchronize_through_the_c_abi():
    ctx = rc.Context(0)
    lib = N.load()
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total, ctx=ctx)
    cap = rc.slot_capacity(L, 8.0)
    syms = torch.empty(N_CH * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x5EED0778, synth.inverse_cdf(c), syms, L, N_CH)
    so = torch.arange(N_CH + 1, dtype=torch.int64, device="cuda") * L
    oo = torch.arange(N_CH + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.zeros(N_CH * cap, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(N_CH, dtype=torch.int64, device="cuda")
    fe = torch.full((N_CH,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    # back to the context's own stream, then raw C-ABI launches ordered by rc_ctx_synchronize
    assert lib.rc_ctx_reset_stream(ctx.handle) == N.RC_OK
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib.rc_encode_batch(ctx.handle, m.handle, P(syms), P(so), N_CH, P(out), P(oo), P(ol),
                               P(fe)) == N.RC_OK
    dec = torch.zeros_like(syms)
    fd = torch.full((N_CH,), -1, dtype=torch.int32, device="cuda")
    co = oo[:-1].contiguous()
    torch.cuda.synchronize()  # (co's copy kernel, on torch's stream)
    assert lib.rc_decode_batch(ctx.handle, m.handle, P(out), P(co), P(ol), P(dec), P(so), N_CH,
                               P(fd)) == N.RC_OK
    assert lib.rc_ctx_synchronize(ctx.handle) == N.RC_OK
    assert not fe.any() and not fd.any()
    assert torch.equal(dec, syms)
    h = syms.cpu().numpy()
    want = _oracle_chunks(c, cum, total, h, [0, N_CH // 2, N_CH - 1])
    hb, hl = out.cpu().numpy(), ol.cpu().numpy()
    for k, b in want.items():
        assert bytes(hb[k * cap:k * cap + int(hl[k])]) == b, f"chunk {k}"
    # the stream pointer stays valid: a later Python call binds torch's stream again
    fd2 = rc.decode_batch(m, out, co, ol, dec, so)
    torch.cuda.synchronize()
    assert not fd2.any()


def test_batch_round_trips_from_concurrent_host_threads():
    """One context per host thread (include/range_coder.h), each on its own torch stream with
    its own model (uniform, Zipf, a random table with a non-power-of-two total): concurrent
    model creation, encode and decode; every thread's bytes against the oracle and its decode
    against its input.  The reference's coders are independent Send state machines
    (encoder.rs:7-20, decoder.rs:6-23): parallelism is independent instances."""
    import threading

    n_threads, n_ch, ln, reps = 4, 64, 16384, 3
    rng = np.random.default_rng(11)
    tables = [synth.uniform_table(), synth.zipf_table()]
    while len(tables) < n_threads:
        c = rng.integers(1, 400, 256).astype(np.uint32)
        tables.append((c, np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint32),
                       int(c.sum())))
    results, errors = [None] * n_threads, []
    start = threading.Barrier(n_threads)

    def work(t):
        try:
            c, cum, total = tables[t]
            ctx = rc.Context(0)
            s = torch.cuda.Stream()
            start.wait()
            with torch.cuda.stream(s):
                m = rc.StaticModel(c, cum, total, ctx=ctx)
                cap = rc.slot_capacity(ln, 12.0)
                syms = torch.empty(n_ch * ln, dtype=torch.uint8, device="cuda")
                synth.fill(ctx, 0x5EED0900 + t, synth.inverse_cdf(c), syms, ln, n_ch)
                so = torch.arange(n_ch + 1, dtype=torch.int64, device="cuda") * ln
                oo = torch.arange(n_ch + 1, dtype=torch.int64, device="cuda") * cap
                out = torch.empty(n_ch * cap, dtype=torch.uint8, device="cuda")
                dec = torch.empty_like(syms)
                ok = True
                for _ in range(reps):
                    ol, fe = rc.encode_batch(m, syms, so, out, oo)
                    fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
                    ok = ok and bool(torch.equal(dec, syms)) and not fe.any() and not fd.any()
                s.synchronize()
                results[t] = (ok, syms.cpu().numpy(), out.cpu().numpy(), ol.cpu().numpy(), cap)
            m.close()
            ctx.close()
        except Exception as exc:  # noqa: BLE001 (reported below)
            errors.append((t, repr(exc)))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(n_threads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    from oracle import cpu
    for t, (ok, h, hb, hl, cap) in enumerate(results):
        assert ok, f"thread {t}: round trip"
        c, cum, total = tables[t]
        for k in (0, n_ch - 1):
            f, b, _ = cpu.encode(c, cum, total, h[k * ln:(k + 1) * ln])
            assert f == 0 and bytes(hb[k * cap:k * cap + int(hl[k])]) == b, f"thread {t} chunk {k}"
