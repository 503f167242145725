set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_container.py tests/test_gpu_limits.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -2 $O/gpu.log
bash tools/traffic_ab.sh r03b default ld8
