"""Chunk sharding across GPUs: one process per GPU, contiguous chunk ranges.

Every chunk is an independent stream (a fresh reference Encoder per chunk, encoder.rs:14-16),
so a batch splits across ranks with no data-path collective.  The only cross-rank
bookkeeping is control data: where each rank's code lands in a global arena (an exclusive
scan of per-rank byte counts, one int64 per rank) and the max-over-ranks step time.
"""
import numpy as np

from .synth import GOLDEN

M64 = (1 << 64) - 1


def shard_range(n_chunks, world, rank):
    """[lo, hi) of the global chunks owned by `rank`: contiguous, sizes differ by at most one
    (the first n_chunks % world ranks take one more)."""
    if world < 1 or not 0 <= rank < world or n_chunks < 0:
        raise ValueError(f"bad shard: n_chunks={n_chunks} world={world} rank={rank}")
    q, r = divmod(n_chunks, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def synth_seed(seed, first_chunk):
    """Seed under which rc_synth_fill's chunk 0 is global chunk `first_chunk` of `seed`.

    Symbol i of chunk k is drawn from mix64(seed + GOLDEN * ((k << 32) + i/4 + 1)), so shifting
    k by `first_chunk` is adding GOLDEN * (first_chunk << 32) to the seed (mod 2^64): every
    rank then generates exactly its slice of one global stream, whatever the world size."""
    return (seed + GOLDEN * ((first_chunk << 32) & M64)) & M64


def exclusive_scan(counts):
    """Exclusive prefix sum (u64) of per-chunk or per-rank byte counts, plus the total."""
    c = np.asarray(counts, dtype=np.uint64)
    off = np.zeros(c.size + 1, dtype=np.uint64)
    np.cumsum(c, out=off[1:])
    return off[:-1], int(off[-1])


def global_code_offset(local_bytes, dist=None, device=None):
    """(base, total): where this rank's code starts in the concatenation of all ranks' code,
    in rank order, and the global code size.  Single process: (0, local_bytes)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return 0, int(local_bytes)
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.tensor([int(local_bytes)], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    per_rank = [int(x.item()) for x in out]
    off, total = exclusive_scan(per_rank)
    return int(off[rank]), total


def max_over_ranks(value, dist=None, device=None):
    """The slowest rank's value (bench timing: the job ends when the last rank ends)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, dist=None, device=None):
    """The sum of an integer count over the ranks (bench: every rank's algorithmic bytes)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return int(value)
    import torch
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def all_ranks_true(flag, dist=None, device=None):
    """True when `flag` holds on every rank (an all-reduce MIN of one int)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(flag)
    import torch
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def free_port():
    """A free TCP port on 127.0.0.1 for the rendezvous."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(script, argv, nprocs, port=None, env=None):
    """Run `script argv` as `nprocs` rank processes of one node (one per GPU) under
    torch.distributed.run with a 127.0.0.1 rendezvous, and return its exit code.

    The caller must not have initialised the GPU (no HIP call, no torch.cuda.is_available()):
    the ranks are fresh child processes, never an exec of this one.  Each rank reads RANK,
    LOCAL_RANK and WORLD_SIZE from its environment."""
    import subprocess
    import sys
    if nprocs < 1:
        raise ValueError(f"nprocs must be >= 1, got {nprocs}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={int(nprocs)}", "--master-addr", "127.0.0.1",
           "--master-port", str(port or free_port()), script] + list(argv)
    return subprocess.run(cmd, env=env).returncode
