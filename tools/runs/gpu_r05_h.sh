# Round 5, call H: the stream-service round trip, piece by piece (tools/ubench_mailbox.hip).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r05h
mkdir -p $O
timeout -k 10 120 ./tools/ubench_mailbox 20000 > $O/ubench_mailbox.json 2> $O/ubench_mailbox.err || { tail -20 $O/ubench_mailbox.err; exit 1; }
cat $O/ubench_mailbox.json
timeout -k 10 120 ./tools/ubench_mailbox 20000 > $O/ubench_mailbox2.json 2> $O/ubench_mailbox2.err || { tail -20 $O/ubench_mailbox2.err; exit 1; }
cat $O/ubench_mailbox2.json
