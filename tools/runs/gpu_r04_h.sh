# Round 4, call H: the GPU suite with the split encoder, then its A/B at the configs[4] shard
# shapes (Zipf; 2^17 chunks = the N = 8 shard, 2^18 = N = 4), forced on / off by RC_ENC_SPLIT.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04h}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for sp in 0 1; do
    for n in 131072 262144; do
      RC_ENC_SPLIT=$sp timeout -k 10 300 python3 bench.py --config zipf --global-chunks $n $ONE --steps 5 --warmup 1 > $O/split${sp}_${n}_$r.json 2> $O/split${sp}_${n}_$r.err || { tail -5 $O/split${sp}_${n}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/split${sp}_${n}_$r.json "split=$sp $n $r"
    done
  done
done
