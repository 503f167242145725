#!/bin/bash
# Build the variants of the 88-VGPR repro (tools/vgpr88/README.md) on the CPU:
#   88   the round-1 coder as it was (k_encode_static allocates 88 VGPRs)
#   96   the same source with one clobbered register (allocation 96)
#   p88  88 + the wave probe (HW_ID / GPR_ALLOC / LDS_ALLOC / XCC_ID / start+end clock per wave)
#   p96c 96 + the probe + a canary in v88..v95 (inside the allocation, above every named register)
# For each: the library, the repro binary, the ISA, the ISA with the register-count lines
# stripped, and the raw kernel descriptors (tools/vgpr88/kd.py).
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
LLVM=/opt/rocm/lib/llvm/bin
mkdir -p out
gcc -O2 -fPIC -c ../../oracle/rc_oracle.c -o out/rc_oracle.o
declare -A DEFS=([88]="" [96]="-DRC_R1_FLOOR96" [p88]="-DRC_PROBE"
                 [p96c]="-DRC_PROBE -DRC_R1_FLOOR96 -DRC_CANARY")
for v in ${VARIANTS:-88 96 p88 p96c}; do
  D="${DEFS[$v]}"
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $D \
    rc_kernels_r1.hip -o out/librc_r1_$v.so
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $D -S --cuda-device-only rc_kernels_r1.hip \
    -o out/isa_$v.s 2>/dev/null
  grep -v "amdhsa_next_free_vgpr\|amdhsa_accum_offset\|vgpr_count\|NumVgprs\|TotalNumVgpr\|Occupancy\|vgpr floor\|ASMSTART\|ASMEND\|^\s*;" \
    out/isa_$v.s > out/isa_$v.stripped.s
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $D --cuda-device-only -c rc_kernels_r1.hip \
    -o out/dev_$v.o 2>/dev/null
  $LLVM/clang-offload-bundler --type=o --input=out/dev_$v.o \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=out/co_$v.elf --unbundle
  $HIPCC --offload-arch=gfx950 -O2 -std=c++17 $D -I. -c repro.cpp -o out/repro_$v.o
  $HIPCC --offload-arch=gfx950 out/repro_$v.o out/rc_oracle.o -o out/repro_$v -Lout -lrc_r1_$v \
    "-Wl,-rpath,\$ORIGIN"
done
python3 kd.py out/co_88.elf out/co_96.elf out/co_p88.elf out/co_p96c.elf
if diff -q out/isa_88.stripped.s out/isa_96.stripped.s >/dev/null; then
  echo "88 vs 96: ISA identical apart from the VGPR allocation"
else
  echo "88 vs 96: ISA differs:"; diff out/isa_88.stripped.s out/isa_96.stripped.s | head -20
fi
# the descriptor-patching runner (same instructions, allocation rewritten at load time)
$HIPCC --offload-arch=gfx950 -O2 -std=c++17 -c patchrun.cpp -o out/patchrun.o
$HIPCC --offload-arch=gfx950 out/patchrun.o out/rc_oracle.o -o out/patchrun
