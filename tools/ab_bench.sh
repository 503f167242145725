#!/bin/bash
# Same-box A/B of library builds: tools/kbench.py on the uniform and Zipf(1.2) configurations
# (2^20 x 64 KiB), ROUNDS rounds interleaved.
#   gpurun -- 'bash tools/ab_bench.sh OUTDIR ROUNDS lib1 lib2 ...'   ("default" = in-tree)
# An argument may carry environment settings after a colon (default:RC_PRIO=off); the library
# reads them when kbench.py creates its context.
set -euo pipefail
O=$1; R=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$O"
for r in $(seq 1 "$R"); do
  for arg in "$@"; do
    lib=${arg%%:*}; envs=""; [ "$arg" != "$lib" ] && envs=${arg#*:}
    L=""; [ "$lib" != default ] && L="$ROOT/variants/librc_amd_$lib.so"
    tag=${arg//[:=]/_}
    for cfg in uniform zipf; do
      env $envs RC_LIB_PATH=$L timeout -k 10 300 python3 "$ROOT/tools/kbench.py" --config $cfg \
        --steps 5 --warmup 1 > "$O/${tag}_${cfg}_$r.json" 2> "$O/${tag}_${cfg}_$r.err"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" "$O/${tag}_${cfg}_$r.json" "$tag.$cfg.$r"
    done
  done
done
