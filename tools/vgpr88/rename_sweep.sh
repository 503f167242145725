#!/bin/bash
# The register-renamed variants of tools/vgpr88/rename.py, each at the allocations given.
set -o pipefail
out=$1
cd "$(dirname "$0")/out"
run() { echo "== $1" >> "$out"; shift; for a in "$@"; do :; done; }
for spec in "rn_shift6.elf 96 104" "rn_top2.elf 96 104" "rn_one87.elf 96" "rn_one86.elf 96" "rn_mid.elf 96" "rn_low.elf 96" "co_p88.elf 88 96"; do
  set -- $spec; co=$1; shift
  echo "== $co" >> "$out"
  for a in "$@"; do
    timeout -k 10 120 ./patchrun "$co" "$a" 327680 1024 >> "$out" 2>&1 || { echo "exit $?" >> "$out"; exit 1; }
  done
done
