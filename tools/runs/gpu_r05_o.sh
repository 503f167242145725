# Round 5, call O: the bound counters (tools/pmc_bound.sh) on the end-of-round build, for the
# final evidence set (uniform, Zipf, the N = 8 shard).
set -e
export PYTHONUNBUFFERED=1
sha256sum range_coder_rust_amd/librc_amd.so
CONFIGS="uniform zipf shard" bash tools/pmc_bound.sh r05o
echo "bound done"
