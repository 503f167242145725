# Round 4, call S: what the 2^17-chunk pair decoder waits on (timing-only scratch builds; their
# output is wrong by construction, so bench.py exits 3 after printing): the symbol bursts
# dropped (-DRC_EXP_DEC_NOSTORE), with and without the one-ahead table reads (-DDEC_XSPEC=1).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04s
mkdir -p $O
export PYTHONUNBUFFERED=1
ONE="--no-cpu-baseline --no-zipf --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2; do
  for lib in default xspec nostore xnostore; do
    L=""; [ "$lib" != default ] && L=$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so
    rc=0
    RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 $ONE --steps 5 --warmup 1 > $O/${lib}_$r.json 2> $O/${lib}_$r.err || rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -5 $O/${lib}_$r.err; exit 1; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'], d['bit_exact_round_trip'])" $O/${lib}_$r.json "$lib $r"
  done
done
