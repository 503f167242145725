"""Chunk sharding across ranks: contiguous shards, per-rank synthetic inputs equal
to the global stream's slices, global code offsets by exclusive scan, max-over-ranks timing.
The multi-process case runs world_size 2 on gloo (CPU) with the C oracle as the per-rank coder,
and checks that the ranks' concatenated code equals a single-process encode of all chunks."""
import multiprocessing as mp
import os

import numpy as np
import pytest

from oracle import cpu
from range_coder_rust_amd import shard, synth

SEED = 0x5EED0001
L = 1024
N_CHUNKS = 37  # not a multiple of the world size


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (37, 2), (37, 8), (1 << 20, 8), (5, 8)])
def test_shard_range_partitions(n, world):
    ranges = [shard.shard_range(n, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a, b), (c, d) in zip(ranges, ranges[1:]):
        assert b == c
    sizes = [b - a for a, b in ranges]
    assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_args():
    for args in ((10, 0, 0), (10, 2, 2), (-1, 1, 0)):
        with pytest.raises(ValueError):
            shard.shard_range(*args)


def test_synth_seed_slices_the_global_stream():
    inv = synth.inverse_cdf(synth.zipf_table()[0])
    for base in (0, 1, 12345, (1 << 20) - 3):
        s = shard.synth_seed(SEED, base)
        for j in (0, 2):
            assert np.array_equal(synth.host_chunk(s, inv, j, 257),
                                  synth.host_chunk(SEED, inv, base + j, 257))


def test_exclusive_scan():
    off, total = shard.exclusive_scan([5, 0, 7, 1])
    assert off.tolist() == [0, 5, 5, 12] and total == 13
    off, total = shard.exclusive_scan([])
    assert off.size == 0 and total == 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_headline_is_one_workload_at_every_n(world):
    """bench.py's headline is configs[4] at every N: the same stream, only the shard count in
    the workload string changes, and the shards cover the global chunks exactly once."""
    import bench
    one = bench.plan(1, 0)
    assert one["n"] == one["n_all"] == 1 << 20 and one["scaling"] == "strong"
    assert "Zipf(1.2)" in one["workload"] and "configs[4]" in one["workload"]
    plans = [bench.plan(world, r) for r in range(world)]
    for p in plans:
        assert p["workload"] == one["workload"].replace("over 1 GPU(s)", f"over {world} GPU(s)")
        assert p["n_all"] == one["n_all"] and p["scaling"] == "strong"
        # the uniform configs[1] extra keeps 2^20 chunks per GPU (weak)
        assert p["weak_n"] == 1 << 20
    assert sum(p["n"] for p in plans) == 1 << 20
    assert [p["lo"] for p in plans] == [shard.shard_range(1 << 20, world, r)[0]
                                         for r in range(world)]


def test_sum_over_ranks_single_process():
    assert shard.sum_over_ranks(7) == 7


def _table():
    c, cum, total = synth.zipf_table()
    return c, cum, total, synth.inverse_cdf(c)


def _encode_range(lo, hi):
    """Oracle-encode global chunks [lo, hi) generated from per-rank seeds; compact code."""
    c, cum, total, inv = _table()
    seed = shard.synth_seed(SEED, lo)
    syms = np.concatenate([synth.host_chunk(seed, inv, j, L) for j in range(hi - lo)]
                          or [np.zeros(0, np.uint8)])
    n = hi - lo
    so = (np.arange(n + 1) * L).astype(np.uint64)
    cap = 16 + 2 * L
    oo = (np.arange(n + 1) * cap).astype(np.uint64)
    out, ol, fl = cpu.encode_batch(c, cum, total, syms, so, oo, 1)
    assert (fl == 0).all()
    return b"".join(bytes(out[k * cap: k * cap + int(ol[k])]) for k in range(n)), ol


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.shard_range(N_CHUNKS, world, rank)
        code, lens = _encode_range(lo, hi)
        base, total = shard.global_code_offset(len(code), dist)
        t = shard.max_over_ranks(0.25 * (rank + 1), dist)
        # (bench.py's aggregate roofline: every rank's bytes summed)
        assert shard.sum_over_ranks(len(code), dist) == total
        q.put((rank, lo, hi, base, total, t, code))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_shards_equal_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = shard.free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole, _ = _encode_range(0, N_CHUNKS)
    arena = bytearray(res[0][4])
    for rank, lo, hi, base, total, t, code in res:
        assert total == len(whole)
        assert t == pytest.approx(0.25 * world)  # the slowest rank's time
        arena[base: base + len(code)] = code
    assert bytes(arena) == whole
    assert [r[1:3] for r in res] == [shard.shard_range(N_CHUNKS, world, r) for r in range(world)]
