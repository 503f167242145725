#!/bin/bash
# Build the two variants of the 88-VGPR repro (tools/vgpr88/README.md) on the CPU:
#   r1_88: the round-1 coder as it was (k_encode_static allocates 88 VGPRs)
#   r1_96: the same source with one clobbered register (allocation 96)
# and their ISA with the kernel descriptors stripped, for the diff.
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
mkdir -p out
gcc -O2 -fPIC -c ../../oracle/rc_oracle.c -o out/rc_oracle.o
for v in 88 96; do
  D=""; [ $v = 96 ] && D="-DRC_R1_FLOOR96"
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $D -Rpass-analysis=kernel-resource-usage \
    rc_kernels_r1.hip -o out/librc_r1_$v.so 2> out/remarks_$v.txt
  grep -o "Function Name: [^ ]*\|    VGPRs: [0-9]*" out/remarks_$v.txt | paste - - \
    | grep "k_encode_static\|k_decode_static" > out/vgprs_$v.txt
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $D -S --cuda-device-only rc_kernels_r1.hip \
    -o out/isa_$v.s 2>/dev/null
  grep -v "amdhsa_next_free_vgpr\|amdhsa_accum_offset\|vgpr_count\|NumVgprs\|TotalNumVgpr\|Occupancy\|vgpr floor\|ASMSTART\|ASMEND\|^\s*;" \
    out/isa_$v.s > out/isa_$v.stripped.s
  $HIPCC --offload-arch=gfx950 -O2 -std=c++17 -I. -c repro.cpp -o out/repro.o
  $HIPCC --offload-arch=gfx950 out/repro.o out/rc_oracle.o -o out/repro_$v -Lout -lrc_r1_$v \
    "-Wl,-rpath,\$ORIGIN"
done
cat out/vgprs_88.txt out/vgprs_96.txt
if diff -q out/isa_88.stripped.s out/isa_96.stripped.s >/dev/null; then
  echo "ISA identical apart from the VGPR allocation"
else
  echo "ISA differs:"; diff out/isa_88.stripped.s out/isa_96.stripped.s | head -20
fi
