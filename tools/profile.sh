#!/bin/bash
# Profile the default bench on the GPU box; everything lands under gpurun_out/prof_<tag>/.
#   gpurun -- 'bash tools/profile.sh r01'
# then, locally: python tools/pmc_traffic.py gpurun_out/prof_r01 --tag r01
# (writes profiles/traffic.json and profiles/r01/*, which bench.py and DESIGN.md cite).
# Each pass is its own rocprofv3 run: kernel trace + stats of the exact default bench command,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (they do not fit one pass, and
# counters are never combined with trace domains), then SQ instruction/wait counters.
set -euo pipefail
TAG=${1:?usage: profile.sh TAG}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
# the PMC passes replay the headline workload once (no Zipf leg, no CPU sample): one launch each
PMC=(python3 bench.py --no-cpu-baseline --no-zipf --steps 1 --warmup 0)

timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
  -- python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "trace pass done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv \
  -- "${PMC[@]}" > "$O/fetch.log" 2>&1
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv \
  -- "${PMC[@]}" > "$O/write.log" 2>&1
echo "write pass done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$O/sq" -o run \
  --output-format csv -- "${PMC[@]}" > "$O/sq.log" 2>&1
echo "sq pass done"
