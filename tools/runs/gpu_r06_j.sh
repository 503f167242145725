#!/bin/bash
# Round 6: the direct-table (uniform) decoder at 4 waves per SIMD (LDS pad, occ3 build: 2^20
# chunks = 4 whole rounds) against 5 (in-tree: 3.2 rounds), headline shape, 3 rounds interleaved
set -euo pipefail
O=gpurun_out/r06j; mkdir -p $O
for r in 1 2 3; do
  for lib in default occ3; do
    L=""; [ $lib != default ] && L=variants/librc_amd_$lib.so
    RC_LIB_PATH=$L timeout -k 10 300 python3 tools/kbench.py --config uniform --steps 5 --warmup 1 \
      > $O/${lib}_uniform_$r.json 2> $O/${lib}_uniform_$r.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['decode_frac'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" $O/${lib}_uniform_$r.json $lib.$r
  done
done
