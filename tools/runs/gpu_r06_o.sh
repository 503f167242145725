#!/bin/bash
# Round 6: coder variants, same box, 4 rounds, order rotating: in-tree (ranked flush rounds),
# flushe (+ rank records fpos | lane, one round per trigger), dec1 (flushe + decoder load
# bursts clamped once per segment); the coder GPU tests on dec1 first
set -euo pipefail
O=gpurun_out/r06o; mkdir -p $O
RC_LIB_PATH=$PWD/variants/librc_amd_dec1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encode.py tests/test_gpu_parity.py tests/test_gpu_ring.py tests/test_gpu_container.py tests/test_gpu_stream_order.py tests/test_gpu_host_stream.py tests/test_gpu_limits.py > $O/pytest.log 2>&1
tail -1 $O/pytest.log
libs=(default flushe dec1)
for r in 1 2 3 4; do
  for i in 0 1 2; do
    lib=${libs[$(( (i + r) % 3 ))]}
    L=""; [ $lib != default ] && L=$PWD/variants/librc_amd_$lib.so
    for cfg in uniform zipf; do
      RC_LIB_PATH=$L timeout -k 10 300 python3 tools/kbench.py --config $cfg --steps 5 --warmup 1 \
        > $O/${lib}_${cfg}_$r.json 2> $O/${lib}_${cfg}_$r.err
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" $O/${lib}_${cfg}_$r.json $lib.$cfg.$r
    done
  done
done
