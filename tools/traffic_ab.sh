#!/bin/bash
# Read traffic of the static coders per library build (the half-line refetch):
# for each build a plain timed bench run (uniform + Zipf legs) and one counter pass of the
# TCC->EA read requests by size over one launch of each kernel.
# Usage on the GPU box:  bash tools/traffic_ab.sh TAG lib1 [lib2 ...]   ("default" = in-tree)
# -> gpurun_out/traffic_<TAG>/<lib>/ ; summarise with python3 tools/traffic_ab.py
set -euo pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
ONE=(--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream)
for lib in "$@"; do
  O="$ROOT/gpurun_out/traffic_$TAG/$lib"
  mkdir -p "$O"
  L=""; [ "$lib" != default ] && L="$ROOT/variants/librc_amd_$lib.so"
  RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py "${ONE[@]}" --steps 5 --warmup 1 > "$O/bench.json" 2> "$O/bench.err"
  RC_LIB_PATH=$L timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
    TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d "$O/rd" -o run --output-format csv \
    -- python3 bench.py "${ONE[@]}" --steps 1 --warmup 0 > "$O/rd.log" 2>&1
  echo "$lib done"
done
