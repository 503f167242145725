#!/bin/bash
# Two SQ counter passes over one encode+decode of 2^18 chunks (stall attribution for the static
# kernels).  Usage on the GPU box:  bash tools/pmc_sq.sh TAG   -> gpurun_out/sq_<TAG>/
set -euo pipefail
TAG=${1:?usage: pmc_sq.sh TAG}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O="$ROOT/gpurun_out/sq_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
RUN=(python3 bench.py --chunks 262144 --no-cpu-baseline --no-zipf --no-adaptive --steps 1 --warmup 0)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  -d "$O/p1" -o run --output-format csv -- "${RUN[@]}" > "$O/p1.log" 2>&1
echo "pass 1 done"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA \
  -d "$O/p2" -o run --output-format csv -- "${RUN[@]}" > "$O/p2.log" 2>&1
echo "pass 2 done"
