# pair-bucket decoder (LUT 3): parity, then 2^17 / 2^20 Zipf with and without it
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for p in auto 0 1024; do
  E=""; [ $p != auto ] && E=$p
  for n in 131072 262144 1048576; do
    RC_DEC_PAIR=$E timeout -k 10 300 python bench.py --config zipf --global-chunks $n --steps 5 --warmup 1 --no-cpu-baseline > $O/z_${p}_$n.json 2> $O/z_${p}_$n.err
  done
  echo "$p done"
done
