#!/bin/bash
# Profile the default bench on the GPU box; everything lands under gpurun_out/prof_<tag>/.
#   gpurun -- 'bash tools/profile.sh r02'
# then, locally: python tools/pmc_traffic.py gpurun_out/prof_r02 --tag r02 --config zipf
# (writes profiles/traffic.json and profiles/r02/*, which bench.py and DESIGN.md cite).
# Each pass is its own rocprofv3 run: kernel trace + stats of the exact default bench command,
# then counter passes (counters are never combined with trace domains; at most 4 TCC counters
# per pass): FETCH_SIZE and WRITE_SIZE as MI355X_MICROARCH.md prescribes, the raw TCC->EA
# request counters by size (which FETCH_SIZE's gfx950 expression folds wrongly: 128-B reads
# count as 64 B) and the DRAM-bound ones, then SQ instruction counters.  The same counter passes
# run over tools/pmc_calib (known byte counts in the coders' access shapes and the guide's
# coalesced anchor shape), so every factor is calibrated on this box, in this run.
set -euo pipefail
TAG=${1:?usage: profile.sh TAG}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
sha256sum range_coder_rust_amd/librc_amd.so > "$O/lib.sha256"  # (pmc_traffic.py keys traffic.json to it)
# the PMC passes replay one configuration's encode and decode once (CONFIG: zipf, the headline,
# or uniform): one launch of each kernel
PMC=(python3 tools/kbench.py --config "${CONFIG:-zipf}" --steps 1 --warmup 0)
CAL=("$ROOT/tools/pmc_calib")
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
        "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum")

if [ -z "${SKIP_TRACE:-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
  echo "trace pass done"
fi
# the counter passes' workload once without a profiler: its algorithmic bytes per launch
timeout -k 10 300 "${PMC[@]}" > "$O/kbench.json" 2> "$O/kbench.err"
i=0
for p in "${PASSES[@]}"; do
  # shellcheck disable=SC2086
  timeout -s KILL 300 rocprofv3 --pmc $p -d "$O/pmc$i" -o run --output-format csv \
    -- "${PMC[@]}" > "$O/pmc$i.log" 2>&1
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $p -d "$O/cal$i" -o run --output-format csv \
    -- "${CAL[@]}" > "$O/cal$i.log" 2>&1
  echo "counter pass $i done ($p)"
  i=$((i + 1))
done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$O/sq" -o run \
  --output-format csv -- "${PMC[@]}" > "$O/sq.log" 2>&1
echo "sq pass done"
