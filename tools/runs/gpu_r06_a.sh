# Round 6, call A: the new headline (configs[4] Zipf at every N) at N = 1 as the driver runs it,
# and the N = 2 rank path rehearsed on one device (shard counts only differ in the workload).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r06a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']); print(json.dumps(d['extras'].get('uniform_weak')))"
RC_BENCH_ONE_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --global-chunks 131072 --chunks 65536 --no-adaptive > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_n2.json')); print(d['value'], d['config']['workload'], d['roofline'])"
