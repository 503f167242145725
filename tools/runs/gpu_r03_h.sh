set -e
# Histogram kernel A/B (round-2 workgroup kernel, lane-private ds_add, lane-private RMW) and the
# model-build parity tests of the default (rmw) build.
O=$GRAFT_REPO_ROOT/gpurun_out/r03h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_model_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/mb.log 2>&1 || { tail -40 $O/mb.log; exit 1; }
tail -1 $O/mb.log
timeout -k 10 300 python -u tools/hist_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
