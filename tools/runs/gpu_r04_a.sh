# Round 4, call A: smoke, the full GPU suite on the shipped library, the GPU parity and ring
# tests again on the RC_RING_GUARD scratch library (zero guard hits), and the guard probe.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_guard.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_guard.log 2>&1 || { tail -30 $O/pytest_guard.log; exit 1; }
tail -2 $O/pytest_guard.log
timeout -k 10 300 python tools/ring_guard.py probe > $O/guard_probe.json 2> $O/guard_probe.err || { tail -20 $O/guard_probe.err; exit 1; }
cat $O/guard_probe.json
