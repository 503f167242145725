#!/bin/bash
# What binds the static kernels: per configuration (uniform: direct-table
# decoder; zipf: bucket decoder) one kernel-trace pass (durations, VGPR counts) and two SQ counter
# passes with the GRBM clock counters, over one launch of each kernel at 2^20 x 64 KiB; "shard":
# the configs[4] N = 8 shard (2^17 Zipf chunks: the LUT 4 bucket decoder in 512-lane workgroups).
# Usage on the GPU box:  [CONFIGS="shard"] bash tools/pmc_bound.sh TAG   -> gpurun_out/bound_<TAG>/
# then locally: python3 tools/pmc_bound.py gpurun_out/bound_<TAG>
set -euo pipefail
TAG=${1:?usage: pmc_bound.sh TAG}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O="$ROOT/gpurun_out/bound_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
for cfg in ${CONFIGS:-uniform zipf}; do
  if [ "$cfg" = shard ]; then
    RUN=(python3 tools/kbench.py --config zipf --chunks 131072 --steps 1 --warmup 0)
  else
    RUN=(python3 tools/kbench.py --config $cfg --steps 1 --warmup 0)
  fi
  mkdir -p "$O/$cfg"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$cfg/trace" -o run --output-format csv \
    -- "${RUN[@]}" > "$O/$cfg/trace.log" 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    GRBM_GUI_ACTIVE GRBM_COUNT -d "$O/$cfg/p1" -o run --output-format csv -- "${RUN[@]}" \
    > "$O/$cfg/p1.log" 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH \
    SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$O/$cfg/p2" -o run --output-format csv \
    -- "${RUN[@]}" > "$O/$cfg/p2.log" 2>&1
  echo "$cfg done"
done
