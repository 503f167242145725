#!/bin/bash
# Waves per SIMD against decode throughput, same code (round 6): the 256-lane decoders (LUT 2 on
# the uniform model, LUT 4 on a Zipf(0.8) table of total 2^13, whose 2^10 buckets keep the
# workgroup at 30 KiB) in scratch builds whose only difference is extra LDS per workgroup
# (-DRC_DEC_LDS_PAD), which sets how many workgroups share a CU: 5 (VGPR-bound at 96), 4, 3, 2;
# plus an 80-VGPR build (-DRC_DEC_WAVES=6: the uniform decoder at 6 waves).  3,932,160 chunks
# of 4 KiB are whole rounds at every one of those occupancies.
#   local:  bash tools/occupancy_sweep.sh build
#   box:    bash tools/occupancy_sweep.sh run OUTDIR
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS="occ5:0 occ4:4096 occ3:16384 occ2:32768"
if [ "$1" = build ]; then
  for v in $VARIANTS; do
    RC_REV_FLAGS="-DRC_DEC_LDS_PAD=${v#*:}" bash "$ROOT/tools/build_rev.sh" HEAD "${v%%:*}"
  done
  RC_REV_FLAGS="-DRC_DEC_WAVES=6" bash "$ROOT/tools/build_rev.sh" HEAD occ6
  exit 0
fi
O=$2
mkdir -p "$O"
N=3932160
for r in 1 2; do
  for tag in occ5 occ4 occ3 occ2 occ6; do
    for cfg in uniform zipf; do
      RC_LIB_PATH="$ROOT/variants/librc_amd_$tag.so" timeout -k 10 300 python3 "$ROOT/tools/kbench.py" \
        --config $cfg --zipf-s 0.8 --zipf-total 8192 --chunks $N --chunk-bytes 4096 --steps 3 \
        --warmup 1 > "$O/${tag}_${cfg}_$r.json" 2> "$O/${tag}_${cfg}_$r.err"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" "$O/${tag}_${cfg}_$r.json" "$tag.$cfg.$r"
    done
  done
done
# the pair-bucket decoder (one LDS round trip per symbol, 1024-lane workgroups) against LUT 4
# on the headline shape, in-tree library
for r in 1 2; do
  for pw in 0 1024; do
    RC_DEC_PAIR=$pw timeout -k 10 300 python3 "$ROOT/tools/kbench.py" --config zipf --steps 3 \
      --warmup 1 > "$O/pair${pw}_zipf_$r.json" 2> "$O/pair${pw}_zipf_$r.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" "$O/pair${pw}_zipf_$r.json" "pair$pw.$r"
  done
done
