#!/bin/bash
# Lehmer inner step: variant 2 (kept) vs 3 (fdiv20, unguarded operands), prep16 stamps, interleaved x3
set -o pipefail
O=gpurun_out/r5ac; mkdir -p $O
for r in 1 2 3; do
  for v in "" _i3; do
    echo "== i${v:-_i2}" >> $O/stamps.txt
    timeout -k 10 60 tools/ubench/prep16_stamps_ubench$v >> $O/stamps.txt 2>&1 || exit $?
  done
done
