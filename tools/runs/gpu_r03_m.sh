set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -1 $O/gpu.log
RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_b11o.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_b11o.log 2>&1 || { tail -40 $O/gpu_b11o.log; exit 1; }
tail -1 $O/gpu_b11o.log
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
timeout -k 10 300 python3 bench.py $ONE --steps 5 --warmup 1 > $O/u.json 2> $O/u.err
timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/z17.json 2> $O/z17.err
for lib in b11 b11o; do
  RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so timeout -k 10 300 python3 bench.py --config zipf $ONE --steps 5 --warmup 1 > $O/z_$lib.json 2> $O/z_$lib.err
done
python3 - "$O" <<'PY'
import json, sys
for f in ("u", "z17", "z_b11", "z_b11o"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, d["value"], d["encode_gsym_s"], d["decode_gsym_s"], d.get("extras", {}).get("zipf1.2", {}).get("decode_gsym_s"))
PY
