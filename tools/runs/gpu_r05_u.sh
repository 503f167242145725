# Round 5, call U: the Python Decoder's trimmed per-call path (api.py): the stream tests, then
# tools/percall_bench.py twice.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05u
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -1 $O/pytest_stream.log
for r in 1 2; do
  timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall_$r.json 2> $O/percall_$r.err || { tail -20 $O/percall_$r.err; exit 1; }
  cat $O/percall_$r.json
done
