#!/bin/bash
# full-length items in prep16 (no flag scan after dsm16): parity + drop-in/tile/half tests,
# small-batch A/B against the scan build, drop-in latency of both
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_gpu_tile.py tests/test_gpu_half.py tests/test_gpu_halfcheck.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/ab_small.sh 3 1,64,256,512 r16 scan main > $O/ab_small.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_main.json > $O/dropin_main.txt 2>&1 || exit $?
FD_ED25519_HIP_LIB=build/variants/scan/libfd_ed25519_hip.so timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 \
  --out $O/dropin_scan.json > $O/dropin_scan.txt 2>&1 || exit $?
