#!/bin/bash
# dsm16 in-flight gate A/B: in-process latency by rate, deployed at high load
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_tile.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in main r16if1 r16if3 r16if9; do
  lib=build/variants/$v/libfd_ed25519_hip.so; [ $v = main ] && lib=firedancer_amd/_lib/libfd_ed25519_hip.so
  FD_ED25519_HIP_LIB=$lib GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/latency_rates_probe.py \
    --rates 0,28000,570000,2400000,4300000 --slots 8 --runs 2 --txns 60000 > $O/inproc_${v}_$rep.txt 2>&1 || exit $?
done
done
for v in main r16if9; do
  svc=build/variants/$v/fd_verify_hip_service; [ $v = main ] && svc=firedancer_amd/_lib/fd_verify_hip_service
  for r in 0 3400000 4200000; do
    timeout -k 10 200 python -u tools/deployed_probe.py --mode host-parse --rate $r --runs 2 --txns 200000 --slots 8 \
      --hw-queues 8 --pin --service $svc > $O/deployed_${v}_$r.txt 2>&1 || exit $?
  done
done
