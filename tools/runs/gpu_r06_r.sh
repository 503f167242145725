# Round 6, call R: the end-of-round set on the final build: smoke, the GPU suite, the
# driver's bench command, and the default bench under rocprofv3 --kernel-trace --stats.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r
mkdir -p $O
export PYTHONUNBUFFERED=1
sha256sum range_coder_rust_amd/librc_amd.so > $O/lib.sha256
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']); print(json.dumps(d['extras']))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/bench_rocprof.json 2> $O/bench_rocprof.err || { tail -20 $O/bench_rocprof.err; exit 1; }
tail -1 $O/bench_rocprof.json | cut -c1-300
timeout -k 10 480 python3 -u tools/parity_soak.py 360 20261020 > $O/parity_soak.log 2>&1 || { tail -5 $O/parity_soak.log; exit 1; }
tail -1 $O/parity_soak.log | cut -c1-200
