set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03o
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -1 $O/gpu.log
bash tools/ab_bench.sh $O/ab 3 default prev
