#!/bin/bash
# round-5 validation (final tree, drop-in codes polled): the whole GPU suite, smoke, the default bench line,
# rocprofv3 kernel trace + PMC of the bench workload, a kernel trace of the
# latency form (1- and 256-signature batches), drop-in latency
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5bi; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 700 tools/profile.sh r5bi_prof > $O/profile.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/small_trace -o run --output-format csv -- \
  python3 tools/small_batch_probe.py --sizes 1,256 --batches 40 > $O/small_trace.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/dropin_latency.py --calls 2000 --out $O/dropin_latency.json > $O/dropin.txt 2>&1 || exit $?
