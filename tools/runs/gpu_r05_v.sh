# Round 5, call V: where the Python mirror's caller-adaptive decode spends its host time.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05v
mkdir -p $O
timeout -k 10 300 python3 tools/percall_profile.py > $O/profile.txt 2>&1 || { tail -30 $O/profile.txt; exit 1; }
head -45 $O/profile.txt
