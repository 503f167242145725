# Round 4, call Y: the adaptive encoder's output register shifted by four v_perm_b32 sharing one
# selector (out_push8): the adaptive and stream suites, then the adaptive C4 leg against the
# previous build (variants/librc_amd_base5.so), 3 interleaved rounds, one box.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04y
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaptive.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ONE="--no-cpu-baseline --no-zipf --no-model-build --no-container --no-host-stream"
for r in 1 2 3; do
  for lib in default base5; do
    L=""; [ "$lib" != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so
    RC_LIB_PATH=$L timeout -k 10 400 python3 bench.py $ONE --steps 2 --warmup 1 > $O/${lib}_$r.json 2> $O/${lib}_$r.err || { tail -5 $O/${lib}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); a=d['extras']['adaptive_c4']; print(sys.argv[2], a['encode_gsym_s'], a['decode_gsym_s'], a['bit_exact_round_trip'])" $O/${lib}_$r.json "$lib $r"
  done
done
