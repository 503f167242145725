#!/bin/bash
# Round 6: encoder flush rounds over ranked ready chunks (variants/librc_amd_flushc.so): the
# encoder's GPU tests on the variant, then a same-box A/B against the in-tree library
set -euo pipefail
O=gpurun_out/r06l; mkdir -p $O
RC_LIB_PATH=$PWD/variants/librc_amd_flushc.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_encode.py tests/test_gpu_parity.py tests/test_gpu_container.py \
  tests/test_gpu_stream_order.py > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/ab_bench.sh $O 3 default flushc
