# Round 4, call D: scratch A/Bs at the configs[4] shard shapes (Zipf, 2^17 and 2^20 chunks):
#  encnoout - the encoder with its byte output dropped (RC_EXP_NOOUT: what a coder wave alone
#             would cost, the bound on splitting output work into a second wave; timing only)
#  pairld8  - the 512-lane pair decoder with 128-B load bursts (DEC_PAIR512_LD=8)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04d}
mkdir -p $O
export PYTHONUNBUFFERED=1
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for r in 1 2; do
for lib in default encnoout pairld8; do
  L=""; [ "$lib" != default ] && L="$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so"
  for n in 131072 1048576; do
    set +e
    RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks $n $ONE --steps 5 --warmup 1 > $O/${lib}_${n}_$r.json 2> $O/${lib}_${n}_$r.err
    rc=$?
    set -e
    # (encnoout fails the round trip check by design: exit 3 after its JSON line)
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -5 $O/${lib}_${n}_$r.err; exit 1; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'])" $O/${lib}_${n}_$r.json "$lib $n $r"
  done
done
done
