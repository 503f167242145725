# Round 5, call C: wave-priority policies for the end of a launch, in rounds of the kernel's own
# residency R (rc_prio_policy): the last round(s) at priority 1, the last three rounds graded,
# rotating priorities, and combinations; the direct-table decoder with its ring in 32-B rows
# (DEC_ROWS: 4 waves per SIMD, one VALU fewer per symbol).  Stamps at 2^20 (uniform, Zipf) and
# at the 2^17 N = 8 shard (Zipf).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05c
V=$GRAFT_REPO_ROOT/variants
mkdir -p $O
export PYTHONUNBUFFERED=1
run_stamp() {
  local lib=$1 tag=$2 cfg=$3 ch=$4; shift 4
  ( env "$@" RC_LIB_PATH=$V/librc_amd_$lib.so timeout -k 10 300 python tools/stamp_probe.py run $O/${lib}_${cfg}_$tag --config $cfg --chunks $ch > $O/${lib}_${cfg}_$tag.log 2>&1 ) || { tail -20 $O/${lib}_${cfg}_$tag.log; return 1; }
  echo "$lib $cfg $tag"; cut -c1-120 $O/${lib}_${cfg}_$tag.log | grep -E "^(encode|decode)"
}
run_stamp stamp none uniform 1048576
run_stamp stamp last1 uniform 1048576 RC_PRIO_LAST=1
run_stamp stamp last1.5 uniform 1048576 RC_PRIO_LAST=1.5
run_stamp stamp rank uniform 1048576 RC_PRIO_RANK=1
run_stamp stamp last1rot12 uniform 1048576 RC_PRIO_LAST=1 RC_PRIO_ROT=12
run_stamp stamp rot12 uniform 1048576 RC_PRIO_ROT=12
run_stamp stamp_decrows none uniform 1048576
run_stamp stamp_decrows rot12 uniform 1048576 RC_PRIO_ROT=12
run_stamp stamp_decrows last1 uniform 1048576 RC_PRIO_LAST=1
run_stamp stamp_decrows rank uniform 1048576 RC_PRIO_RANK=1
run_stamp stamp none zipf "131072 1048576"
run_stamp stamp rot10 zipf "131072 1048576" RC_PRIO_ROT=10
run_stamp stamp rot11 zipf "131072 1048576" RC_PRIO_ROT=11
run_stamp stamp rot12 zipf "131072 1048576" RC_PRIO_ROT=12
run_stamp stamp last1rot10 zipf "131072 1048576" RC_PRIO_LAST=1 RC_PRIO_ROT=10
run_stamp stamp rank zipf 1048576 RC_PRIO_RANK=1
run_stamp stamp none2 uniform 1048576
# the stream service with the one-burst request read: its tests, then per-call costs
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -1 $O/pytest_stream.log
timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native.json 2> $O/percall_native.err || { tail -20 $O/percall_native.err; exit 1; }
cat $O/percall_native.json
RC_STREAM_SERVICE=0 timeout -k 10 120 ./tools/percall_native 5000 > $O/percall_native_launch.json 2> $O/percall_native_launch.err || { tail -20 $O/percall_native_launch.err; exit 1; }
cat $O/percall_native_launch.json
timeout -k 10 300 python tools/percall_bench.py 262144 2000 > $O/percall.json 2> $O/percall.err || { tail -20 $O/percall.err; exit 1; }
cat $O/percall.json
