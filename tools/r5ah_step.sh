#!/bin/bash
# Lehmer inner step: two steps per branch (i4) vs one (kept, variant 3); prep16 stamps, interleaved x3
set -o pipefail
O=gpurun_out/r5ah; mkdir -p $O
for r in 1 2 3; do
  for v in "" _i4; do
    echo "== i3$v" >> $O/stamps.txt
    timeout -k 10 60 tools/ubench/prep16_stamps_ubench$v >> $O/stamps.txt 2>&1 || exit $?
  done
done
