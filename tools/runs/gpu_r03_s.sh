set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03ab
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -1 $O/gpu.log
bash tools/strong_sweep.sh $O/strong
bash tools/profile.sh r03
