# Round 4, call J: the deferred-output encoder (ENC_DEFER=1, default) against the build without
# it (variants/librc_amd_nodefer.so), same box, uniform + Zipf at 2^20 and the 2^17 / 2^18 shard
# shapes; then the GPU suite.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for lib in default nodefer; do
    L=""; [ "$lib" != default ] && L="$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so"
    RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py $ONE --steps 5 --warmup 1 > $O/${lib}_full_$r.json 2> $O/${lib}_full_$r.err || { tail -5 $O/${lib}_full_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); z=d['extras']['zipf1.2']; print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], z['encode_gsym_s'], z['decode_gsym_s'])" $O/${lib}_full_$r.json "$lib full $r"
    for n in 131072 262144; do
      RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks $n $ONE --no-zipf --steps 5 --warmup 1 > $O/${lib}_${n}_$r.json 2> $O/${lib}_${n}_$r.err || { tail -5 $O/${lib}_${n}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/${lib}_${n}_$r.json "$lib $n $r"
    done
  done
done
