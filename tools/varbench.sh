#!/bin/bash
# Bench decoder build variants side by side (k_decode_static table).  Build each
# variant first, on the CPU, as range_coder_rust_amd/var/librc_<NAME>.so, e.g.
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DRC_DEV_ONLY -DDEC_LD=2 -Iinclude \
#     -c range_coder_rust_amd/csrc/rc_decode_pow2.hip -o var/k_C.o
#   hipcc --offload-arch=gfx950 -shared -o range_coder_rust_amd/var/librc_C.so var/k_C.o <other .o>
# (knobs: DEC_LD, DEC_PF, DEC_RING, DEC_OUT_BURST, DEC_MIRROR, DEC_TAB_LDS), then on the box:
#   VARS="A C" bash tools/varbench.sh   -> gpurun_out/v_<NAME>.json
set -e
mkdir -p gpurun_out
for n in ${VARS:-A B C D}; do
  RC_LIB_PATH=range_coder_rust_amd/var/librc_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-adaptive --no-model-build --no-container --no-host-stream > gpurun_out/v_$n.json 2> gpurun_out/v_$n.err
  echo "$n done"
done
