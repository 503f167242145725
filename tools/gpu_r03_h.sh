set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -2 $O/gpu.log
B="--steps 5 --warmup 1 --no-cpu-baseline"
for n in 131072 262144 524288; do
  timeout -k 10 300 python bench.py --config zipf --global-chunks $n $B > $O/z$n.json 2> $O/z$n.err
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo done
