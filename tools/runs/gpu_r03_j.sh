set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_container.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -2 $O/gpu.log
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for lib in default lut12 default lut12; do
  L=""; [ "$lib" != default ] && L="$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so"
  RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf $ONE --steps 5 --warmup 1 > $O/z_$lib.json 2> $O/z_$lib.err
  python3 -c "import json,sys; d=json.load(open('$O/z_$lib.json')); print('$lib', d['value'], {k:v for k,v in d.get('extras',{}).items() if 'gsym' in k.lower() or 'rate' in k.lower()})"
done
