# Round 6, call I: the driver's bench command and the default bench under rocprofv3
# --kernel-trace --stats, after the container / host legs moved to the uniform leg.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
export PYTHONUNBUFFERED=1
sha256sum range_coder_rust_amd/librc_amd.so > $O/lib.sha256
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']['frac']); print(json.dumps({k: v for k, v in d['extras'].items() if k in ('container', 'host_stream')}))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/bench_rocprof.json 2> $O/bench_rocprof.err || { tail -20 $O/bench_rocprof.err; exit 1; }
tail -1 $O/bench_rocprof.json | cut -c1-300
grep "k_decode_static<0, 1, 4, 512" $O/trace/run_kernel_stats.csv | cut -c1-250
