#!/bin/bash
# dsm16 re-validation after the container restore: parity (dsm16 forced and by
# size), drop-ins, smoke; the lane-split ubench and permlane probe; small-batch
# latency by form; drop-in per-call latency.
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 60 tools/ubench/permlane_probe > $O/permlane_probe.txt 2>&1 || exit $?
timeout -k 10 120 tools/ubench/fe_lanesplit_ubench > $O/lanesplit_ubench.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
for f in r16 oct; do
  timeout -k 10 200 python -u tools/small_batch_probe.py --sizes 1,64,256,512,1024,2048 --batches 20 --dsm $f \
    > $O/small_$f.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_latency.json > $O/dropin.txt 2>&1 || exit $?
