# scratch: cost of the per-symbol rare branch at the N = 8 shard (2^17) and at 2^20 (Zipf).
# The variants it compared were built with -DRC_EXP_NOBRANCH=1 / -DRC_EXP_RAREBODY=1,2, scratch
# switches removed from the sources after the measurement (DESIGN.md §5,
# profiles/r03/ab/branch_cost/); kept as the record of how the numbers were taken.
O=$GRAFT_REPO_ROOT/gpurun_out/exp_nb
mkdir -p $O
ONE="--no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream"
for r in ${ROUNDS:-1 2}; do
for lib in ${LIBS:-default nb}; do
  L=""; [ "$lib" != default ] && L="$GRAFT_REPO_ROOT/variants/librc_amd_$lib.so"
  for n in 131072 1048576; do
    RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks $n $ONE --steps 5 --warmup 1 > $O/${lib}_${n}_$r.json 2> $O/${lib}_${n}_$r.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['encode_gsym_s'], d['decode_gsym_s'])" $O/${lib}_${n}_$r.json "$lib $n $r" || exit 1
  done
done
done
