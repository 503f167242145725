# Round 5, call S (the end-of-round build: R plus the service timeout counted only while its wave runs): smoke, the GPU
# suite, a same-box A/B (this build, the same with RC_PRIO=off, round 4's HEAD), the driver's
# bench command, the same under rocprofv3 --stats, and the strong sweep (the N = 8 shard shape).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05s
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 1200 bash tools/ab_bench.sh $O/ab 3 default default:RC_PRIO=off r04
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']['frac'], d['extras']['zipf1.2']['encode_gsym_s'], d['extras']['zipf1.2']['decode_gsym_s'], d['extras']['adaptive_c4']['decode_gsym_s'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
echo profiled
bash tools/strong_sweep.sh $O/strong
# per-call costs through the stream service (single-load polling, one release per request)
timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native.json 2> $O/percall_native.err || { tail -20 $O/percall_native.err; exit 1; }
cat $O/percall_native.json
RC_STREAM_SERVICE=0 timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native_launch.json 2> $O/percall_native_launch.err || { tail -20 $O/percall_native_launch.err; exit 1; }
cat $O/percall_native_launch.json
timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall.json 2> $O/percall.err || { tail -20 $O/percall.err; exit 1; }
cat $O/percall.json
RC_STREAM_SERVICE=0 timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall_launch.json 2> $O/percall_launch.err || { tail -20 $O/percall_launch.err; exit 1; }
cat $O/percall_launch.json
# the N-rank bench path rehearsed on this one-GPU box (both ranks on device 0, gloo control)
RC_BENCH_ONE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --global-chunks 262144 --chunks 131072 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { tail -20 $O/bench_rehearse2.err; exit 1; }
tail -1 $O/bench_rehearse2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearse2', d['value'])"
# HBM traffic of this build (traffic.json is keyed to its hash)
bash tools/profile.sh r05s
echo "profile done"
