#!/bin/bash
# integer Lehmer rounds: the half-size search on the device against the host
# build, parity (all forms, fault-injection check), the parts ubench, small
# batches and the throughput A/B against the previous tree
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_half.py \
  tests/test_gpu_halfcheck.py tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_c3.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/ubench/prep_parts_ubench > $O/prep_parts.txt 2>&1 || exit $?
timeout -k 10 300 tools/ab_small.sh 2 1,256,512 r16 prev main > $O/ab_small.txt 2>&1 || exit $?
timeout -k 10 400 tools/ab.sh 3 prev main > $O/ab_c2.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_latency.json > $O/dropin.txt 2>&1 || exit $?
