# Round 5, call M: randomised parity soak (batch, adaptive and stream coders) against the C oracle
# (tools/parity_soak.py), 240 s.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 330 python3 tools/parity_soak.py 240 20260519 > $O/soak.log 2>&1 || { tail -30 $O/soak.log; exit 1; }
tail -3 $O/soak.log
