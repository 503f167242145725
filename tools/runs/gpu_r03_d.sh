# round 3: GPU tests on the default build, per-call mirror costs, and the VALU-slack experiment
# (RC_FILL: n extra 2-cycle VALU per symbol step) at 2^20 and at 2^17 chunks
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -2 $O/gpu.log
timeout -k 10 300 python tools/percall_bench.py > $O/percall.json 2> $O/percall.err || { tail $O/percall.err; exit 1; }
cat $O/percall.json
for v in default fill2 fill4; do
  L=""; [ $v != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$v.so
  RC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream > $O/fill_$v.json 2> $O/fill_$v.err
  RC_LIB_PATH=$L timeout -k 10 300 python bench.py --config zipf --global-chunks 131072 --steps 5 --warmup 1 --no-cpu-baseline > $O/fill17_$v.json 2> $O/fill17_$v.err
  echo "$v done"
done
