# Round 4, call E: same-box A/B of the LUT 4 small-bucket decoder (default) against the build
# before it (r4base: LUT 0 buckets), then the fill-cost series (tools/fill_cost.py).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04e
mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/ab_bench.sh $O/ab 3 default r4base
ROUNDS=2 timeout -k 10 900 python tools/fill_cost.py run $O/fill
