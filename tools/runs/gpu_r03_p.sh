set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03p
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -1 $O/gpu.log
bash tools/ab_bench.sh $O/ab 2 default prev
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2; do for lib in default prev; do
  L=""; [ "$lib" != default ] && L="$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so"
  RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/z17_${lib}_$r.json 2> $O/z17_${lib}_$r.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'])" $O/z17_${lib}_$r.json "z17 $lib $r"
done; done
