# Round 4, call AA: the pair decoder with its table entry AND its ring pair read one symbol ahead
# (variants/librc_amd_xspec2.so, -DDEC_XSPEC=1): parity and ring suites forced to the 512-lane
# pair decoder, then Zipf at 2^17 chunks: LUT 4 (default), the pair decoder, and the read-ahead
# pair decoder, 3 interleaved rounds, one box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04aa
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$GRAFT_REPO_ROOT/variants/librc_amd_xspec2.so
RC_DEC_PAIR=512 RC_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread > $O/pytest512.log 2>&1 || { tail -40 $O/pytest512.log; exit 1; }
tail -1 $O/pytest512.log
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
run() {  # tag lib pair
  RC_DEC_PAIR=$3 RC_LIB_PATH=$2 timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/$1.json "$1"
}
for r in 1 2 3; do
  run lut4_$r "" ""
  run pair_$r "" 512
  run xspec2_$r $V 512
done
