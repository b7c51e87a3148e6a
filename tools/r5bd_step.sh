#!/bin/bash
# dsm16 skipping the identity addition of a zero digit (main) vs always adding (addall): parity, small batches
set -o pipefail
O=gpurun_out/r5bd; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -k "r16 or small_chunks or dropin" > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/ab_small.sh 3 1,256 r16 addall main > $O/ab_small.txt 2>&1 || exit $?
