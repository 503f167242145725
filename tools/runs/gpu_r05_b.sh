# Round 5, call B: the build with the stream service (rc_resume.hip) and the encoder's row-layout
# ring (ENC_ROWS): smoke, the GPU suite (with the service tests), per-call costs with the service
# on and off (Python and C++ mirrors), wave-priority policies for the end of a launch (stamps,
# 2^20 chunks), a same-box A/B against round 4's HEAD and the VCC-wait form, VCC select prices.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05b
V=$GRAFT_REPO_ROOT/variants
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall.json 2> $O/percall.err || { tail -20 $O/percall.err; exit 1; }
cat $O/percall.json
RC_STREAM_SERVICE=0 timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall_launch.json 2> $O/percall_launch.err || { tail -20 $O/percall_launch.err; exit 1; }
cat $O/percall_launch.json
timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native.json 2> $O/percall_native.err || { tail -20 $O/percall_native.err; exit 1; }
cat $O/percall_native.json
RC_STREAM_SERVICE=0 timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native_launch.json 2> $O/percall_native_launch.err || { tail -20 $O/percall_native_launch.err; exit 1; }
cat $O/percall_native_launch.json
# end-of-launch wave priority (rc_static.h): none; by quarter of the grid; the last 1280
# workgroups; rotating priorities (round-robin issue) at 2^10 / 2^12 ticks; the decoder held to
# 4 waves per SIMD by LDS (4 even rounds) alone and with rotation
run_stamp() {
  local tag=$1 cfg=$2 ch=$3; shift 3
  ( env "$@" RC_LIB_PATH=$V/librc_amd_stamp.so timeout -k 10 300 python tools/stamp_probe.py run $O/stamp_${cfg}_$tag --config $cfg --chunks $ch > $O/stamp_${cfg}_$tag.log 2>&1 ) || { tail -20 $O/stamp_${cfg}_$tag.log; return 1; }
  echo "$cfg $tag"; cut -c1-150 $O/stamp_${cfg}_$tag.log | grep -E "^(encode|decode)"
}
run_stamp none uniform 1048576
run_stamp step1024 uniform 1048576 RC_PRIO_STEP=1024
run_stamp last1280 uniform 1048576 RC_PRIO_LAST=1280
run_stamp rot10 uniform 1048576 RC_PRIO_ROT=10
run_stamp rot12 uniform 1048576 RC_PRIO_ROT=12
run_stamp pad4 uniform 1048576 RC_DEC_LDS_PAD=16384
run_stamp pad4rot10 uniform 1048576 RC_DEC_LDS_PAD=16384 RC_PRIO_ROT=10
run_stamp none zipf "65536 131072 1048576"
run_stamp rot10 zipf "131072 1048576" RC_PRIO_ROT=10
run_stamp step1024 zipf 1048576 RC_PRIO_STEP=1024
# same-box A/B: this tree, round 4's HEAD, and this tree without the VCC wait states in the
# small-model decoders' candidate selects (round 4's form)
timeout -k 10 900 bash tools/ab_bench.sh $O/ab 2 default r04 novccwait
# in-loop price of a VCC-reading select vs the same through an SGPR pair (DESIGN.md §5 VCC claim)
OPS=24,25 ROUNDS=2 timeout -k 10 600 python tools/fill_cost.py run $O/fill > $O/fill.log 2>&1 || { tail -20 $O/fill.log; exit 1; }
cat $O/fill.log
# the adaptive decoder at 8 instead of 5 waves per CU (a 128-symbol C4 model, tree rows 1..128)
timeout -k 10 300 python tools/adapt_occ_probe.py 65536 2 > $O/adapt_occ_small.json 2> $O/adapt_occ_small.err || { tail -20 $O/adapt_occ_small.err; exit 1; }
cat $O/adapt_occ_small.json
timeout -k 10 300 python tools/adapt_occ_probe.py 1048576 3 > $O/adapt_occ.json 2> $O/adapt_occ.err || { tail -20 $O/adapt_occ.err; exit 1; }
cat $O/adapt_occ.json
