# decoder variants after the speculative step: LUT0 (RC_DEC_PAIR=0), pair 512 / 1024, and the
# DEC_SPEC=1 build (speculative step in every SM decoder), Zipf 2^17 / 2^18 / 2^20, uniform 2^20
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03g
mkdir -p $O
B="--steps 5 --warmup 1 --no-cpu-baseline"
run() { timeout -k 10 300 python bench.py "$@" > $O/$TAG.json 2> $O/$TAG.err; }
for n in 131072 262144 1048576; do
  for p in 0 512 1024; do TAG=z${n}_p$p RC_DEC_PAIR=$p run --config zipf --global-chunks $n $B; done
  TAG=z${n}_spec RC_DEC_PAIR=0 RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_spec.so run --config zipf --global-chunks $n $B
done
TAG=u_default run --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream $B
TAG=u_spec RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_spec.so run --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream $B
echo done
