# Round 5, call G: the stream service with its block in LDS (rc_resume.hip) and the leaner
# Python decode call: the stream tests, then per-call costs, service and launch path.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -1 $O/pytest_stream.log
timeout -k 10 180 ./tools/percall_native 5000 > $O/percall_native.json 2> $O/percall_native.err || { tail -20 $O/percall_native.err; exit 1; }
cat $O/percall_native.json
RC_STREAM_SERVICE=0 timeout -k 10 180 ./tools/percall_native 5000 > $O/percall_native_launch.json 2> $O/percall_native_launch.err || { tail -20 $O/percall_native_launch.err; exit 1; }
cat $O/percall_native_launch.json
timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall.json 2> $O/percall.err || { tail -20 $O/percall.err; exit 1; }
cat $O/percall.json
RC_STREAM_SERVICE=0 timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall_launch.json 2> $O/percall_launch.err || { tail -20 $O/percall_launch.err; exit 1; }
cat $O/percall_launch.json
