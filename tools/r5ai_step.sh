#!/bin/bash
# Lehmer step variant 4 (two steps per branch) as the default: GPU tests, small-batch A/B against
# the variant-3 build, the throughput scalar phase of both, drop-in latency
set -o pipefail
O=gpurun_out/r5ai; mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_half.py tests/test_gpu_halfcheck.py tests/test_gpu_dropin.py tests/test_gpu_tile.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/ab_small.sh 3 1,256 r16 i3 main > $O/ab_small.txt 2>&1 || exit $?
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-txns 0 --host-reps 0 --deployed-txns 0 --c4-signatures 0"
for r in 1 2; do
  for v in i3 main; do
    lib=build/variants/$v/libfd_ed25519_hip.so; [ $v = main ] && lib=firedancer_amd/_lib/libfd_ed25519_hip.so
    FD_ED25519_HIP_LIB=$lib timeout -k 10 200 $B > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit $?
  done
done
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_main.json > $O/dropin_main.txt 2>&1 || exit $?
