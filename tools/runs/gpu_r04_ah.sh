# Round 4, call AH: the decoders' data update with the perm tied to the low half of data << k8
# (no v_mov of the high half per symbol: -1 VALU per symbol in every static decoder) - smoke and
# the full GPU suite, then a same-box A/B against the previous build (variants/librc_amd_base.so):
# uniform + Zipf at 2^20 (ab_bench.sh, 3 rounds) and Zipf at 2^17.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04ah
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab_bench.sh $O/ab 3 default base
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for lib in default base; do
    L=""; [ "$lib" != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so
    RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/${lib}_131072_$r.json 2> $O/${lib}_131072_$r.err || { tail -5 $O/${lib}_131072_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/${lib}_131072_$r.json "$lib 131072 $r"
  done
done
