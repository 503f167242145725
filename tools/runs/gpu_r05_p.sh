# Round 5, call P: the wave-priority defaults against their neighbours on one box (environment
# overrides of rc_prio_policy; RC_PRIO_ROT applies to every kernel, so its direct-decoder column
# is last-round + rotation): default, RC_PRIO_LAST=0.8 / 1.25 (direct decoder), RC_PRIO_ROT=11 /
# 13 (encoder, LUT 4).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05p
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1500 bash tools/ab_bench.sh $O/ab 3 default default:RC_PRIO_LAST=0.8 default:RC_PRIO_LAST=1.25 default:RC_PRIO_ROT=11 default:RC_PRIO_ROT=13
