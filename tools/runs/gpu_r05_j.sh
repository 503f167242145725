# Round 5, call J: where a stream-service call's time goes (rc_svc_probe_: the wave's stamps and
# the host's wait), after the stream tests.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -1 $O/pytest_stream.log
timeout -k 10 180 ./tools/percall_native 5000 > $O/percall_native.json 2> $O/percall_native.err || { tail -20 $O/percall_native.err; exit 1; }
cat $O/percall_native.json
timeout -k 10 180 ./tools/percall_native 5000 > $O/percall_native2.json 2> $O/percall_native2.err || { tail -20 $O/percall_native2.err; exit 1; }
cat $O/percall_native2.json
