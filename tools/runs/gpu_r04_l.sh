# Round 4, call L: the decoupled-FIFO split encoder (variants/librc_amd_split2.so, -DRC_ENC_SPLIT2):
# the encoder battery and the parity suite on it, then its A/B against the default build at the
# configs[4] shard shapes (Zipf 2^17, 2^18; RC_ENC_SPLIT=1 forces the split kernel at 2^18).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04l
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$GRAFT_REPO_ROOT/variants/librc_amd_split2.so
RC_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parity.py tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread > $O/pytest_split2.log 2>&1 || { tail -40 $O/pytest_split2.log; exit 1; }
tail -1 $O/pytest_split2.log
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for lib in default split2; do
    L=""; [ "$lib" != default ] && L=$V
    for n in 131072 262144; do
      RC_ENC_SPLIT=$([ "$lib" = split2 ] && echo 1 || echo 0) RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks $n $ONE --steps 5 --warmup 1 > $O/${lib}_${n}_$r.json 2> $O/${lib}_${n}_$r.err || { tail -5 $O/${lib}_${n}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/${lib}_${n}_$r.json "$lib $n $r"
    done
  done
done
