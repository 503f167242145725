# Round 4, call G: adaptive (C4) SQ counters at 2^21 x 16 KiB (the bench shape halved: the
# script checks the round trip with a full-size temporary) for the ceiling derivation (§5.1).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/ad_r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RUN=(python3 tools/adapt_bench.py 2097152 1)
timeout -k 10 300 "${RUN[@]}" > $O/plain.log 2>&1
cat $O/plain.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- "${RUN[@]}" > $O/trace.log 2>&1
echo trace done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  -d $O/p1 -o run --output-format csv -- "${RUN[@]}" > $O/p1.log 2>&1
echo pass 1 done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/p2 -o run --output-format csv -- "${RUN[@]}" > $O/p2.log 2>&1
echo pass 2 done
