#!/bin/bash
# Round 6, call T: the driver's bench command on the final build, on another box (the spread)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN_TAG:-r06t}
mkdir -p $O
export PYTHONUNBUFFERED=1
sha256sum range_coder_rust_amd/librc_amd.so > $O/lib.sha256
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['encode_gsym_s'], d['decode_gsym_s'], d['roofline']['frac'], d['extras']['uniform_weak']['value'], d['extras']['uniform_weak']['decode_gsym_s'])"
