# Round 4, call AK: the final build (after the f64 range / total for small non-power-of-two models): smoke, GPU suite, default bench + rocprofv3 stats, the strong
# sweep, and the binding-resource counters at all three shapes (2^20 uniform / Zipf, 2^17 shard).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04ak
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']['frac'], d['extras']['zipf1.2']['decode_gsym_s'], d['extras']['adaptive_c4']['decode_gsym_s'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
echo profiled
bash tools/strong_sweep.sh $O/strong
CONFIGS="uniform zipf shard" bash tools/pmc_bound.sh r04ak
# the N-rank bench path rehearsed on this one-GPU box (both ranks on device 0, gloo control)
RC_BENCH_ONE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --global-chunks 262144 --chunks 131072 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { tail -20 $O/bench_rehearse2.err; exit 1; }
tail -1 $O/bench_rehearse2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearse2', d['value'])"  # (gloo prints above the JSON line)
