# Round 4, call B: the default bench, then its rocprofv3 kernel trace + stats.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04b}
mkdir -p $O
export PYTHONUNBUFFERED=1
# the default bench, then its rocprofv3 kernel trace + stats
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
echo profiled
