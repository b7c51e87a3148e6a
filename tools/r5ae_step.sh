#!/bin/bash
# two-wave SHA-512: K+W precombined in LDS and the words read a group ahead (kw) vs before; prep16 stamps x3
set -o pipefail
O=gpurun_out/r5ae; mkdir -p $O
for r in 1 2 3; do
  for v in "" _kw; do
    echo "== base$v" >> $O/stamps.txt
    timeout -k 10 60 tools/ubench/prep16_stamps_ubench$v >> $O/stamps.txt 2>&1 || exit $?
  done
done
