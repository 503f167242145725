set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_default.log 2>&1 || { tail -30 $O/gpu_default.log; exit 1; }
tail -3 $O/gpu_default.log
RC_LIB_PATH=$GRAFT_REPO_ROOT/variants/librc_amd_dec80.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_dec80.log 2>&1 || { tail -30 $O/gpu_dec80.log; exit 1; }
tail -3 $O/gpu_dec80.log
