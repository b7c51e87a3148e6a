#!/bin/bash
# broadcast-routed r16 group ops + two multiply-add chains: parity, then the
# small-batch A/B against the previous tree and the accumulator variants
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 tools/ab_small.sh 3 1,256,512 r16 prev main r16acc1 r16acc4 > $O/ab_small.txt 2>&1 || exit $?
