# Round 5, call A: per-wave stamps of the static coders (tools/stamp_probe.py) at 2^16 .. 2^20
# chunks, uniform and Zipf; the direct-table decoder held to 4 waves per SIMD by LDS padding
# (same code); the half-wave issue probe; a same-box A/B against round 4; filler prices.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05a
V=$GRAFT_REPO_ROOT/variants
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 ./tools/ubench_halfwave > $O/ubench_halfwave.json
cat $O/ubench_halfwave.json
RC_LIB_PATH=$V/librc_amd_stamp.so timeout -k 10 420 python tools/stamp_probe.py run $O/stamp --config uniform > $O/stamp_uniform.log 2>&1 || { tail -30 $O/stamp_uniform.log; exit 1; }
cut -c1-400 $O/stamp_uniform.log
RC_LIB_PATH=$V/librc_amd_stamp.so timeout -k 10 300 python tools/stamp_probe.py run $O/stamp --config zipf --chunks 131072 262144 1048576 > $O/stamp_zipf.log 2>&1 || { tail -30 $O/stamp_zipf.log; exit 1; }
cut -c1-400 $O/stamp_zipf.log
RC_LIB_PATH=$V/librc_amd_stamp_pad4.so timeout -k 10 300 python tools/stamp_probe.py run $O/stamp_pad4 --config uniform --chunks 262144 1048576 > $O/stamp_pad4.log 2>&1 || { tail -30 $O/stamp_pad4.log; exit 1; }
cut -c1-400 $O/stamp_pad4.log
# same-box A/B: this tree (decoder verification as failing-lane ballots) against round 4's HEAD,
# and with the encoder's row-layout ring (ENC_ROWS, v_and_or_b32 slot address)
timeout -k 10 900 bash tools/ab_bench.sh $O/ab 2 default r04 encrows
# in-loop price of the non-VALU classes (SALU, compare + branch, LDS read) beside v_add
OPS=0,20,21,22,23 ROUNDS=2 timeout -k 10 900 python tools/fill_cost.py run $O/fill > $O/fill.log 2>&1 || { tail -20 $O/fill.log; exit 1; }
cat $O/fill.log
