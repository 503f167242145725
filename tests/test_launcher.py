"""The multi-rank launcher of bench.py --gpus N (range_coder_rust_amd.shard.launch_ranks), run on
the CPU: world_size 2 over gloo with the C oracle as each rank's coder; and bench.py's
refusals (more GPUs than visible, --gpus disagreeing with WORLD_SIZE) on a box without GPUs."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import cpu
from range_coder_rust_amd import shard, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_launch_ranks_every_rank_reports(tmp_path, world):
    n_chunks, L = 7, 512
    out = tmp_path / "ranks.json"
    rc = shard.launch_ranks(os.path.join(ROOT, "tests", "rank_probe.py"),
                            [str(out), str(n_chunks), str(L)], world,
                            env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert rc == 0
    rep = json.loads(out.read_text())
    assert rep["world"] == world and rep["ok"]
    ranks = sorted(rep["ranks"])
    assert [r[0] for r in ranks] == list(range(world))
    assert [tuple(r[1:3]) for r in ranks] == [shard.shard_range(n_chunks, world, r)
                                              for r in range(world)]
    # the shards' code adds up to a single-process encode of the whole stream
    c, cum, total = synth.zipf_table()
    inv = synth.inverse_cdf(c)
    syms = np.concatenate([synth.host_chunk(0x5EED0001, inv, j, L) for j in range(n_chunks)])
    so = (np.arange(n_chunks + 1) * L).astype(np.uint64)
    oo = (np.arange(n_chunks + 1) * (16 + 2 * L)).astype(np.uint64)
    _, ol, fl = cpu.encode_batch(c, cum, total, syms, so, oo, 1)
    assert (fl == 0).all() and rep["total"] == int(ol.sum()) == sum(r[3] for r in ranks)


def _bench(args, env=None):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=120,
                          env=dict(os.environ, **(env or {})))


def test_bench_refuses_more_gpus_than_visible():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible")
    r = _bench(["--gpus", "2"])
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr


def test_bench_refuses_gpus_world_size_mismatch():
    r = _bench(["--gpus", "2"], env=dict(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "disagrees with WORLD_SIZE=3" in r.stderr
