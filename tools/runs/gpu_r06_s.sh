#!/bin/bash
# Round 6: the encoder's slow flush path rolled, its symbol quarters fully unrolled for small models (roll), against
# the in-tree final build, same box, 4 rounds alternating; the coder GPU tests on roll first
set -euo pipefail
O=gpurun_out/r06s; mkdir -p $O
RC_LIB_PATH=$PWD/variants/librc_amd_roll.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encode.py tests/test_gpu_parity.py tests/test_gpu_container.py tests/test_gpu_stream_order.py tests/test_gpu_host_stream.py tests/test_gpu_limits.py > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for r in 1 2 3 4; do
  if [ $((r % 2)) = 0 ]; then order="roll default"; else order="default roll"; fi
  for lib in $order; do
    for cfg in uniform zipf; do
      L=""; [ $lib != default ] && L=$PWD/variants/librc_amd_$lib.so
      RC_LIB_PATH=$L timeout -k 10 300 python3 tools/kbench.py --config $cfg --steps 5 --warmup 1 \
        > $O/${lib}_${cfg}_$r.json 2> $O/${lib}_${cfg}_$r.err
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" $O/${lib}_${cfg}_$r.json $lib.$cfg.$r
    done
  done
done
