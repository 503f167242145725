set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03z
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
RC_BENCH_ONE_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --global-chunks 262144 --chunks 131072 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['n_gpus'], d['value'], d['config']['workload'], d['scaling'])" $O/n2.json
