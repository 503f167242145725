# Round 4, call N: the pair-bucket decoder's select as v_cmp + v_cndmask_b32_sdwa (in-tree build,
# 40.4 -> 37.4 VALU per symbol): the parity / ring / stream suites, then Zipf decode at the
# configs[4] shard shapes against the previous build (variants/librc_amd_base2.so), and the
# 1024-lane pair decoder against LUT 4 at 2^18 and 2^19 chunks.  3 interleaved rounds, one box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04n
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
run() {  # tag lib pair n
  L=""; [ "$2" != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$2.so
  RC_DEC_PAIR=$3 RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks $4 $ONE --steps 5 --warmup 1 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['value'])" $O/$1.json "$1"
}
for r in 1 2 3; do
  run new_131072_$r default "" 131072
  run base_131072_$r base2 "" 131072
  for n in 262144 524288; do
    run new_lut4_${n}_$r default "" $n
    run new_p1024_${n}_$r default 1024 $n
  done
done
