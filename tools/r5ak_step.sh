#!/bin/bash
# SHA rounds with h+K+W added first (pf: FD_SHA_T1_EARLY) vs not; prep16 stamps, interleaved x3
set -o pipefail
O=gpurun_out/r5ak; mkdir -p $O
for r in 1 2 3; do
  for v in "" _pf; do
    echo "== base$v" >> $O/stamps.txt
    timeout -k 10 60 tools/ubench/prep16_stamps_ubench$v >> $O/stamps.txt 2>&1 || exit $?
  done
done
