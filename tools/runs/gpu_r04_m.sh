# Round 4, call M: the LUT 4 candidate select as v_cmp + v_cndmask_b32_sdwa (in-tree build):
# the parity, ring and encoder suites, then a same-box A/B against the previous build
# (variants/librc_amd_base.so), 3 rounds, uniform + Zipf at 2^20.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh $O/ab 3 default base
