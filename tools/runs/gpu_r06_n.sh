#!/bin/bash
# Round 6: the rank-table records fpos | lane (flushd) against the in-tree ranked flush, 4 rounds with
# the order alternating (flushd first in even rounds)
set -euo pipefail
O=gpurun_out/r06n; mkdir -p $O
RC_LIB_PATH=$PWD/variants/librc_amd_flushd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encode.py tests/test_gpu_parity.py tests/test_gpu_container.py tests/test_gpu_stream_order.py > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for r in 1 2 3 4; do
  if [ $((r % 2)) = 0 ]; then order="flushd default"; else order="default flushd"; fi
  for lib in $order; do
    L=""; [ $lib != default ] && L=$PWD/variants/librc_amd_$lib.so
    for cfg in uniform zipf; do
      RC_LIB_PATH=$L timeout -k 10 300 python3 tools/kbench.py --config $cfg --steps 5 --warmup 1 \
        > $O/${lib}_${cfg}_$r.json 2> $O/${lib}_${cfg}_$r.err
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" $O/${lib}_${cfg}_$r.json $lib.$cfg.$r
    done
  done
done
