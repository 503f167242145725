set -e
# Container pack with one wave per chunk: container tests, then the default bench's container leg.
O=$GRAFT_REPO_ROOT/gpurun_out/r03x
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_container.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ct.log 2>&1 || { tail -40 $O/ct.log; exit 1; }
tail -1 $O/ct.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-adaptive --no-host-stream > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['extras']['container'])" $O/bench.json
