set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03l
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -2 $O/gpu.log
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
timeout -k 10 300 python3 bench.py $ONE --steps 5 --warmup 1 > $O/u.json 2> $O/u.err
timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/z17.json 2> $O/z17.err
python3 - "$O" <<'PY'
import json
for f in ("u", "z17"):
    import sys; d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, d["value"], d["encode_gsym_s"], d["decode_gsym_s"], d.get("extras", {}).get("zipf1.2", {}).get("decode_gsym_s"))
PY
