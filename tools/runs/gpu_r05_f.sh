# Round 5, call F: HBM traffic of the shipping build (tools/profile.sh: the trace pass and the
# FETCH/WRITE/EA counter passes with their calibration runs; traffic.json is keyed to this
# library's hash), then the bound counters (tools/pmc_bound.sh) for the uniform, Zipf and N = 8
# shard configurations.
set -e
export PYTHONUNBUFFERED=1
bash tools/profile.sh r05
echo "profile done"
CONFIGS="uniform zipf shard" bash tools/pmc_bound.sh r05
echo "bound done"
