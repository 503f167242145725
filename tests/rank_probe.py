"""Rank process for tests/test_launcher.py (not a test module): one rank of a CPU (gloo) job
started by range_coder_rust_amd.shard.launch_ranks — the launcher bench.py --gpus N uses.  Each
rank oracle-encodes its contiguous shard of a small synthetic stream; rank 0 writes what every
rank reported to the JSON file named by argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import cpu  # noqa: E402
from range_coder_rust_amd import shard, synth  # noqa: E402


def main():
    out_path, n_chunks, L = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo")
    c, cum, total = synth.zipf_table()
    inv = synth.inverse_cdf(c)
    lo, hi = shard.shard_range(n_chunks, world, rank)
    seed = shard.synth_seed(0x5EED0001, lo)
    n = hi - lo
    syms = np.concatenate([synth.host_chunk(seed, inv, j, L) for j in range(n)]
                          or [np.zeros(0, np.uint8)])
    so = (np.arange(n + 1) * L).astype(np.uint64)
    cap = 16 + 2 * L
    oo = (np.arange(n + 1) * cap).astype(np.uint64)
    out, ol, fl = cpu.encode_batch(c, cum, total, syms, so, oo, 1)
    code_bytes = int(ol.sum())
    rep = torch.tensor([rank, lo, hi, code_bytes, int((fl == 0).all())], dtype=torch.int64)
    got = [torch.zeros_like(rep) for _ in range(world)]
    dist.all_gather(got, rep)
    ok = shard.all_ranks_true(bool((fl == 0).all()), dist)
    base, tot = shard.global_code_offset(code_bytes, dist)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(dict(world=world, ranks=[g.tolist() for g in got], ok=ok, total=tot), f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
