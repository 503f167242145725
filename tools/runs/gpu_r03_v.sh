set -e
# Re-entry check of a rebuilt tree (lane-private histogram): model-build tests first, then every
# GPU test, smoke, the default bench line.
O=$GRAFT_REPO_ROOT/gpurun_out/r03v
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_model_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/mb.log 2>&1 || { tail -40 $O/mb.log; exit 1; }
tail -1 $O/mb.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -1 $O/gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
