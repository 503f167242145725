# Round 4, call T: the build with 2^12-bucket LUT 4 in 512-lane workgroups as the default: the
# whole GPU suite, then at 2^17 chunks LUT 4 (RC_DEC_PAIR=0) against the pair decoder (default),
# 3 rounds.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04t
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
run() {  # tag pair n
  RC_DEC_PAIR=$2 timeout -k 10 300 python3 bench.py --config zipf --global-chunks $3 $ONE --steps 5 --warmup 1 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/$1.json "$1"
}
for r in 1 2 3; do
  run pair_131072_$r "" 131072
  run lut4_131072_$r 0 131072
done
