# Round 5, call N: the mailbox round trip with relaxed polls and with four polls in flight
# (tools/ubench_mailbox.hip variants 6, 7), twice.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05n
mkdir -p $O
timeout -k 10 180 ./tools/ubench_mailbox 20000 > $O/ubench_mailbox.json 2> $O/ubench_mailbox.err || { tail -20 $O/ubench_mailbox.err; exit 1; }
cat $O/ubench_mailbox.json
timeout -k 10 180 ./tools/ubench_mailbox 20000 > $O/ubench_mailbox2.json 2> $O/ubench_mailbox2.err || { tail -20 $O/ubench_mailbox2.err; exit 1; }
cat $O/ubench_mailbox2.json
