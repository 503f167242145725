# decoder occupancy: the shipped 96-VGPR (5 waves/SIMD) build against the 80-VGPR (6 waves) one
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03
mkdir -p $O
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_96.json 2> $O/bench_96.err
RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_dec80.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_80.json 2> $O/bench_80.err
bash tools/strong_sweep.sh $O/sweep96
RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_dec80.so bash tools/strong_sweep.sh $O/sweep80
