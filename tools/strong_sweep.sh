#!/bin/bash
# Per-GPU rate of the configs[4] shard sizes on one GPU: the chunk count one rank codes at
# N = 8, 4, 2, 1 (2^17 .. 2^20 chunks of 64 KiB, Zipf(1.2), rank 0's slice of the bench
# stream).  rate x N over rate(2^20) predicts the strong-scaling efficiency an 8-GPU run can
# reach (the ranks share nothing).
#   gpurun -- 'bash tools/strong_sweep.sh [outdir]'   -> <outdir>/strong_<chunks>.json
# RC_LIB_PATH selects a scratch library build.
set -e
out=${1:-gpurun_out}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
for n in 131072 262144 524288 1048576; do
  timeout -k 10 300 python3 "$ROOT/tools/kbench.py" --config zipf --chunks $n --steps 5 \
    --warmup 2 > "$out/strong_$n.json" 2> "$out/strong_$n.err"
  echo "$n done"
done
