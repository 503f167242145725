# Round 6, call C: why the two-chain Zipf decoder is slower: SQ counters of k_decode_ilp and
# k_decode_static LUT 4 (RC_DEC_ILP=0) over one 2^20-chunk launch each, and the available
# instruction-cache counters.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r06c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -i "icache\|SQC_" $O/avail.txt | head -60 > $O/avail_sqc.txt || true
RUN=(python3 tools/kbench.py --config zipf --chunks 1048576 --steps 1 --warmup 0)
for mode in 1 0; do
  export RC_DEC_ILP=$mode
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$mode -o run --output-format csv -- "${RUN[@]}" > $O/t$mode.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/p1_$mode -o run --output-format csv -- "${RUN[@]}" > $O/p1_$mode.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $O/p2_$mode -o run --output-format csv -- "${RUN[@]}" > $O/p2_$mode.log 2>&1
  echo "mode $mode done"
done
