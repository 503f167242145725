#!/bin/bash
# Round 6: instruction-cache counters of the coders (the encoder's hot loop inlines its flush
# rounds: ~53k instructions in the kernel), one launch of each kernel at 2^20 x 64 KiB
set -euo pipefail
O=gpurun_out/r06k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in zipf uniform; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE \
    -d $O/$cfg -o run --output-format csv -- python3 tools/kbench.py --config $cfg --steps 1 --warmup 0 > $O/$cfg.log 2>&1
  echo "$cfg done"
done
