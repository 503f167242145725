#!/bin/bash
# Build librc_amd.so as it was at a git revision, for same-box A/B runs against the current tree:
#   bash tools/build_rev.sh REV TAG   ->  variants/librc_amd_TAG.so  (load with RC_LIB_PATH)
# The revision's csrc/ and include/ are exported into scratch/rev_TAG and compiled with build()'s
# flags (no ISA check: a committed revision already passed it).
set -euo pipefail
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
S=$ROOT/scratch/rev_$TAG
rm -rf "$S"; mkdir -p "$S" "$ROOT/variants"
git -C "$ROOT" archive "$REV" range_coder_rust_amd/csrc include | tar -x -C "$S"
objs=()
for f in "$S"/range_coder_rust_amd/csrc/*.hip; do
  o=$S/$(basename "$f").o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Wno-unused-result \
    -I"$S/include" ${RC_REV_FLAGS:-} -o "$o" "$f" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o "$ROOT/variants/librc_amd_$TAG.so" "${objs[@]}"
echo "built variants/librc_amd_$TAG.so from $REV"
