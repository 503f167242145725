# Round 4, call O: encode / decode overlap probe (tools/overlap_probe.py) at the configs[4] shard
# shapes, Zipf(1.2), and uniform at 2^18.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r04o
mkdir -p $O
export PYTHONUNBUFFERED=1
for n in 131072 262144 524288; do
  timeout -k 10 300 python3 tools/overlap_probe.py --chunks $n --steps 5 > $O/zipf_$n.json 2> $O/zipf_$n.err || { tail -5 $O/zipf_$n.err; exit 1; }
  cat $O/zipf_$n.json
done
timeout -k 10 300 python3 tools/overlap_probe.py --chunks 262144 --config uniform > $O/uniform_262144.json 2> $O/uniform_262144.err || { tail -5 $O/uniform_262144.err; exit 1; }
cat $O/uniform_262144.json
