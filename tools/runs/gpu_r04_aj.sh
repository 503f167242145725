# Round 4, call AJ: range / total for small non-power-of-two models in two f64 steps (instead of
# the 64 x 64 high product): smoke and the full GPU suite (non-power-of-two totals 2049 ... 65535
# against the oracle), then a same-box A/B against the previous division (variants/
# librc_amd_divmagic.so, -DRC_DIV_F64=0) on bench.py's legs with non-power-of-two models
# (tools/div_probe.py: total 300 "uniform", Zipf(1.2) over 65521), 3 rounds.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04aj
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for lib in default divmagic; do
    L=""; [ "$lib" != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so
    RC_LIB_PATH=$L timeout -k 10 300 python3 tools/div_probe.py $ONE --steps 5 --warmup 1 > $O/${lib}_$r.json 2> $O/${lib}_$r.err || { tail -5 $O/${lib}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); z=d['extras']['zipf1.2']; print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], z['encode_gsym_s'], z['decode_gsym_s'], d['bit_exact_round_trip'] if 'bit_exact_round_trip' in d else '', z['bit_exact_round_trip'])" $O/${lib}_$r.json "$lib.$r"
  done
done
