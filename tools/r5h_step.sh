#!/bin/bash
# prep16 (lane-split decompression): parity, smoke, small-batch latency, drop-in latency
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_gpu_c3.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/small_batch_probe.py --sizes 64,1,64,256,512,1024,2048 --batches 20 --dsm r16 \
    > $O/small_r16.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/small_batch_probe.py --sizes 64,64,256,1024 --batches 20 --forms 0,0 \
    > $O/small_wide.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_latency.json > $O/dropin.txt 2>&1 || exit $?
