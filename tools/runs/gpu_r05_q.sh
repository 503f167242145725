# Round 5, call Q: the small bucket-model decoder (LUT 4, Zipf) at 2^11 buckets in 384-lane
# workgroups (-DSMB_LUT_BITS=11 -DRC_SMB_WG=384: 47 KiB of LDS, 3 workgroups = 18 waves per CU
# instead of 16) and at 2^11 buckets in 256-lane ones, against the shipped 2^12 / 512-lane
# form: the 2^20 A/B (3 rounds), then the 2^17 shard (Zipf, 5 steps) for each build.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05q
V=$GRAFT_REPO_ROOT/variants
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1200 bash tools/ab_bench.sh $O/ab 3 default smb384 smb384:RC_PRIO_LAST=1 smb11
for lib in default smb384 smb11; do
  L=""; [ "$lib" != default ] && L="$V/librc_amd_$lib.so"
  RC_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config zipf --global-chunks 131072 --steps 5 --warmup 2 --no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream > $O/shard_$lib.json 2> $O/shard_$lib.err || { tail -20 $O/shard_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/shard_$lib.json')); print('$lib shard', d['value'], d.get('encode_gsym_s'), d.get('decode_gsym_s'), d.get('bit_exact_round_trip'))"
done
