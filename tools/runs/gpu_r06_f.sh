# Round 6, call F: call E's checks (suite, smoke, per-call, driver bench) and a same-box A/B of
# the LUT 4 select with its wait states filled (variants/librc_amd_selfill.so) against the tree.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r06f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native.json 2> $O/percall_native.err || { tail -20 $O/percall_native.err; exit 1; }
cat $O/percall_native.json
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']['frac']); print(json.dumps({k: d['extras'][k] for k in ('uniform_weak','adaptive_c4','adaptive_c4_128')}))"
timeout -k 10 900 bash tools/ab_bench.sh $O/ab 3 default selfill
