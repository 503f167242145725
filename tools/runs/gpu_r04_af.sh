# Round 4, call AF: the LUT 4 bucket address from a second fma (ulp 2^la_shift) beside the hint -
# the encoder battery and the parity suite, then a same-box A/B against
# the previous build (variants/librc_amd_base10.so): uniform + Zipf at 2^20 (ab_bench.sh, 3
# rounds) and Zipf at 2^17.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04af
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh $O/ab 3 default base10
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for lib in default base10; do
    L=""; [ "$lib" != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so
    RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/${lib}_131072_$r.json 2> $O/${lib}_131072_$r.err || { tail -5 $O/${lib}_131072_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/${lib}_131072_$r.json "$lib 131072 $r"
  done
done
