#!/bin/bash
# full GPU suite + smoke + default bench line on the prep16/dsm16 tree
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc $?" >> $O/bench.err
