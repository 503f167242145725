# Round 4, call Q: LUT 4 with 2^12 buckets in 512-lane workgroups (variants/librc_amd_smb12.so,
# -DSMB_LUT_BITS=12u: no bucket misses on the Zipf model, same waves per SIMD): the parity and
# ring suites on it, then Zipf decode against the default (2^11 buckets, 256 lanes) at 2^20,
# 2^19 and 2^18 chunks, 3 interleaved rounds, one box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$GRAFT_REPO_ROOT/variants/librc_amd_smb12.so
RC_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
run() {  # tag lib n
  RC_LIB_PATH=$2 timeout -k 10 300 python3 bench.py --config zipf --global-chunks $3 $ONE --steps 5 --warmup 1 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/$1.json "$1"
}
for r in 1 2 3; do
  for n in 1048576 524288 262144; do
    run default_${n}_$r "" $n
    run smb12_${n}_$r $V $n
  done
done
