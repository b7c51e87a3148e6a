#!/bin/bash
# prep16 with the hash over two waves: parity (every form, digests path), small-batch A/B, drop-in latency
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_gpu_dropin_large.py tests/test_gpu_c3.py tests/test_gpu_tile.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/ab_small.sh 2 1,256,512 r16 prev main > $O/ab_small.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_latency.json > $O/dropin.txt 2>&1 || exit $?
