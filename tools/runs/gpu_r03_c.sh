set -e
bash tools/pmc_bound.sh r03
O=$GRAFT_REPO_ROOT/gpurun_out/bound_r03/dec80
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_dec80.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream --steps 3 --warmup 1 > $O/trace.log 2>&1
echo dec80 done
