# Round 5, call T: two more 240-s parity soaks (tools/parity_soak.py) on the final build, other seeds.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05t
mkdir -p $O
export PYTHONUNBUFFERED=1
sha256sum range_coder_rust_amd/librc_amd.so
timeout -k 10 330 python3 tools/parity_soak.py 240 20260520 > $O/soak1.log 2>&1 || { tail -30 $O/soak1.log; exit 1; }
tail -1 $O/soak1.log | cut -c1-200
timeout -k 10 330 python3 tools/parity_soak.py 240 20260521 > $O/soak2.log 2>&1 || { tail -30 $O/soak2.log; exit 1; }
tail -1 $O/soak2.log | cut -c1-200
