# Round 6, call Q: end-of-round evidence for the final build (ranked encoder flush, rolled slow path, segment-clamped decoder loads): the
# bench under rocprofv3 (kernel stats) and the traffic counter passes for the headline (Zipf)
# and the uniform load, the bound counters (Zipf, uniform, the N = 8 shard), the strong-scaling
# sweep, and the N = 2 rank path rehearsed on one device at the real configs[4] size.
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r06q
mkdir -p $O
sha256sum range_coder_rust_amd/librc_amd.so > $O/lib.sha256
timeout -k 10 1200 bash tools/profile.sh r06qz > $O/profile_z.log 2>&1 || { tail -20 $O/profile_z.log; exit 1; }
echo "profile zipf done"
SKIP_TRACE=1 CONFIG=uniform timeout -k 10 900 bash tools/profile.sh r06qu > $O/profile_u.log 2>&1 || { tail -20 $O/profile_u.log; exit 1; }
echo "profile uniform done"
CONFIGS="zipf shard uniform" timeout -k 10 900 bash tools/pmc_bound.sh r06q > $O/bound.log 2>&1 || { tail -20 $O/bound.log; exit 1; }
echo "bound done"
timeout -k 10 600 bash tools/strong_sweep.sh $O/strong > $O/strong.log 2>&1 || { tail -20 $O/strong.log; exit 1; }
echo "strong done"
RC_BENCH_ONE_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 --chunks 131072 --no-adaptive > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { tail -20 $O/bench_rehearse2.err; exit 1; }
tail -1 $O/bench_rehearse2.json
