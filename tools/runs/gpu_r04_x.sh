# Round 4, call X: the N-rank bench path rehearsed on the one-GPU box (both ranks on device 0,
# gloo control): configs[4] sharded at 2^18 global chunks, the weak uniform leg at 2^17 per rank.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04x
mkdir -p $O
RC_BENCH_ONE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --global-chunks 262144 --chunks 131072 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { tail -20 $O/bench_rehearse2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_rehearse2.json')); print('rehearse2', d['value'], d['n_gpus'], d['scaling'], d['bit_exact_round_trip'], d['extras']['uniform_weak']['value'])"
