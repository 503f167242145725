# Round 6, call B: the two-chunks-per-lane Zipf decoder (k_decode_ilp): its parity tests, then a
# same-box A/B of the headline (ILP vs RC_DEC_ILP=0), headline only.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r06b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ilp.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ilp.log 2>&1 || { tail -40 $O/pytest_ilp.log; exit 1; }
tail -1 $O/pytest_ilp.log
H="--no-uniform --no-adaptive --no-model-build --no-container --no-host-stream --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  for mode in 1 0; do
    RC_DEC_ILP=$mode timeout -k 10 300 python bench.py $H > $O/bench_ilp${mode}_$r.json 2> $O/bench_ilp${mode}_$r.err || { tail -20 $O/bench_ilp${mode}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_ilp${mode}_$r.json')); print('ilp=$mode', d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']['frac'])"
  done
done
