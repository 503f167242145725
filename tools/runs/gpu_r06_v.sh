#!/bin/bash
# Round 6: the flat-model coders (k_decode_static LUT 5, k_encode_static SM 3: no table reads
# for 256 symbols of c = 1) in variants/librc_amd_flat.so: the whole GPU suite on it, then a
# same-box A/B against the in-tree final build, 3 rounds alternating
set -euo pipefail
O=gpurun_out/r06v; mkdir -p $O
RC_LIB_PATH=$PWD/variants/librc_amd_flat.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  if [ $((r % 2)) = 0 ]; then order="flat default"; else order="default flat"; fi
  for lib in $order; do
    for cfg in uniform zipf; do
      L=""; [ $lib != default ] && L=$PWD/variants/librc_amd_$lib.so
      RC_LIB_PATH=$L timeout -k 10 300 python3 tools/kbench.py --config $cfg --steps 5 --warmup 1 \
        > $O/${lib}_${cfg}_$r.json 2> $O/${lib}_${cfg}_$r.err
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['decode_frac'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" $O/${lib}_${cfg}_$r.json $lib.$cfg.$r
    done
  done
done
