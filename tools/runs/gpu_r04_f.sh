# Round 4, call F: the GPU suite on the 16-B-entry LUT 4 build, its same-box A/B against the
# LUT 0 build (r4base), then the shard-shape scratch A/Bs (gpu_r04_d.sh).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab_bench.sh $O/ab 3 default r4base
bash tools/runs/gpu_r04_d.sh r04f/shard
