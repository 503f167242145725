#!/bin/bash
# One run per VGPR allocation of the same k_encode_static machine code (tools/vgpr88/patchrun.cpp):
# 327680 chunks x 1024 symbols = up to 5 workgroups per CU, so waves sit at 5 VGPR bases.
# Usage: patchsweep.sh <out.txt> <co.elf> <alloc...>
set -o pipefail
out=$1; co=$2; shift 2
cd "$(dirname "$0")/out"
for a in "$@"; do
  timeout -k 10 120 ./patchrun "$co" "$a" 327680 1024 >> "$out" 2>&1 || { echo "alloc $a: exit $?" >> "$out"; exit 1; }
done
