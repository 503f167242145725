#!/bin/bash
# Same-box A/B of library builds: bench.py legs (uniform + Zipf, no CPU baseline / adaptive /
# model-build / container / host-stream), ROUNDS rounds interleaved.
#   gpurun -- 'bash tools/ab_bench.sh OUTDIR ROUNDS lib1 lib2 ...'   ("default" = in-tree)
set -euo pipefail
O=$1; R=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$O"
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
# an argument may carry environment settings after a colon: default:RC_PRIO=off
for r in $(seq 1 "$R"); do
  for arg in "$@"; do
    lib=${arg%%:*}; envs=""; [ "$arg" != "$lib" ] && envs=${arg#*:}
    L=""; [ "$lib" != default ] && L="$ROOT/variants/librc_amd_$lib.so"
    lib=${arg//[:=]/_}
    env $envs RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py $ONE --steps 5 --warmup 1 > "$O/${lib}_$r.json" 2> "$O/${lib}_$r.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); z=d['extras'].get('zipf1.2',{}); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], z.get('encode_gsym_s'), z.get('decode_gsym_s'), 'exact' if d['bit_exact_round_trip'] and z.get('bit_exact_round_trip', True) else 'MISMATCH')" "$O/${lib}_$r.json" "$lib.$r"
  done
done
