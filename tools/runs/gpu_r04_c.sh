# Round 4, call C: in-context issue cost of VALU instruction classes (tools/fill_cost.py).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04c}
mkdir -p $O
export PYTHONUNBUFFERED=1
ROUNDS=${ROUNDS:-2} timeout -k 10 1100 python tools/fill_cost.py run $O
