#!/bin/bash
# integer Lehmer, branch-free quotients: parts ubench (new and the f64 form), parity, small and C2 A/B
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
timeout -k 10 60 tools/ubench/prep_parts_ubench > $O/prep_parts.txt 2>&1 || exit $?
timeout -k 10 60 tools/ubench/prep_parts_ubench_prev > $O/prep_parts_prev.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_half.py \
  tests/test_gpu_halfcheck.py tests/test_gpu_parity.py tests/test_gpu_dropin.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/ab_small.sh 2 1,256 r16 prev main > $O/ab_small.txt 2>&1 || exit $?
timeout -k 10 400 tools/ab.sh 2 prev main > $O/ab_c2.txt 2>&1 || exit $?
