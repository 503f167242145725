#!/bin/bash
# SQ counter passes over one adaptive (C4) encode + decode of 2^16 x 16 KiB chunks.
# Usage on the GPU box:  bash tools/pmc_adapt.sh TAG   -> gpurun_out/ad_<TAG>/
set -euo pipefail
TAG=${1:?usage: pmc_adapt.sh TAG}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O="$ROOT/gpurun_out/ad_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
RUN=(python3 tools/adapt_bench.py 65536 1)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  -d "$O/p1" -o run --output-format csv -- "${RUN[@]}" > "$O/p1.log" 2>&1
echo "pass 1 done"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_WAVES \
  -d "$O/p2" -o run --output-format csv -- "${RUN[@]}" > "$O/p2.log" 2>&1
echo "pass 2 done"
