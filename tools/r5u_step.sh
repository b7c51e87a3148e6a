#!/bin/bash
# dsm16 base prefetch A/B; pipe round trip of 1- and 256-signature batches; in-process latency at 28K/s by slot count
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/ab_small.sh 2 1,256 r16 prev main > $O/ab_small.txt 2>&1 || exit $?
for b in 1 256; do
  timeout -k 10 120 python -u tools/pipe_latency_probe.py --batch $b --slots 8 --reps 100 > $O/pipe_$b.txt 2>&1 || exit $?
done
for s in 1 4 8; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/latency_rates_probe.py --rates 28000 --slots $s --runs 2 > $O/inproc_s$s.txt 2>&1 || exit $?
done
