#!/bin/bash
# prep16 hash blocks of 32 (main) / 16 / 8 messages per pair of waves: small batches, interleaved x3
set -o pipefail
O=gpurun_out/r5an; mkdir -p $O
timeout -k 10 500 tools/ab_small.sh 3 1,64,256,512 r16 main l16 l8 > $O/ab_small.txt 2>&1 || exit $?
for v in l16 l8; do
  FD_ED25519_HIP_LIB=build/variants/$v/libfd_ed25519_hip.so timeout -k 10 300 python -u -m pytest -q --timeout 150 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py -k "r16" > $O/tests_$v.log 2>&1 || exit $?
done
