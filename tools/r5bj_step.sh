#!/bin/bash
# pipe slots of codes only done when their codes land (main) vs at the stream event (pevent): tile / service / mux
# tests, the pipe round trip and in-process C5, interleaved
set -o pipefail
O=gpurun_out/r5bj; mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tile.py \
  tests/test_gpu_mux_tile.py tests/test_gpu_service_fault.py tests/test_gpu_pool_fault.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in pevent main; do
    lib=build/variants/$v/libfd_ed25519_hip.so; [ $v = main ] && lib=firedancer_amd/_lib/libfd_ed25519_hip.so
    echo "== $v" >> $O/inproc.txt
    FD_ED25519_HIP_LIB=$lib GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/latency_rates_probe.py \
      --rates 28000,570000,2400000,4000000 --runs 3 >> $O/inproc.txt 2>&1 || exit $?
    for b in 1 256; do
      echo "== $v batch $b" >> $O/pipe.txt
      FD_ED25519_HIP_LIB=$lib timeout -k 10 120 python -u tools/pipe_latency_probe.py --batch $b --slots 8 --reps 100 \
        >> $O/pipe.txt 2>&1 || exit $?
    done
  done
done
