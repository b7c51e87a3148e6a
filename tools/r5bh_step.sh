#!/bin/bash
# direct drop-in launches return when their codes land in the pinned block (main) vs a stream sync (dsync)
set -o pipefail
O=gpurun_out/r5bh; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dropin.py \
  tests/test_gpu_dropin_threads.py tests/test_gpu_dropin_large.py tests/test_gpu_dropin_fault.py \
  tests/test_gpu_fullsize.py -k "dropin or Dropin" > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in dsync main; do
    lib=build/variants/$v/libfd_ed25519_hip.so; [ $v = main ] && lib=firedancer_amd/_lib/libfd_ed25519_hip.so
    FD_ED25519_HIP_LIB=$lib timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_${v}_$rep.json > $O/dropin_${v}_$rep.txt 2>&1 || exit $?
  done
done
