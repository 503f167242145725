#!/bin/bash
# Round 6: the flat encoder's range written as r (no 24-bit mask and copy): the GPU suite on the
# in-tree build, a same-box A/B against the previous build (variants/librc_amd_e441.so), then
# the evidence call Q for the in-tree build
set -euo pipefail
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  if [ $((r % 2)) = 0 ]; then order="default e441"; else order="e441 default"; fi
  for lib in $order; do
    L=""; [ $lib != default ] && L=$PWD/variants/librc_amd_$lib.so
    RC_LIB_PATH=$L timeout -k 10 300 python3 tools/kbench.py --config uniform --steps 5 --warmup 1 \
      > $O/${lib}_uniform_$r.json 2> $O/${lib}_uniform_$r.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], 'exact' if d['bit_exact_round_trip'] else 'MISMATCH')" $O/${lib}_uniform_$r.json $lib.$r
  done
done
bash tools/runs/gpu_r06_q.sh
