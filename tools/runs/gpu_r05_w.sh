# Round 5, call W: the stream-service soak (tools/service_soak.py): per-call sessions through the
# Python mirror with idle exits and context re-creation, 120 s.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05w
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 tools/service_soak.py 120 7 > $O/service_soak.log 2>&1 || { tail -30 $O/service_soak.log; exit 1; }
tail -2 $O/service_soak.log
