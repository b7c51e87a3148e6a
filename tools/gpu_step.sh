#!/bin/bash
# One GPU call of the build -> measure loop: the GPU tests named (or all),
# then, only if pytest itself finished (0 all passed, 1 some failed -- no
# time limit, crash or abort), one default bench.py line.
#   tools/gpu_step.sh OUTDIR [pytest targets...]
out=$1; shift
mkdir -p "$out"
timeout -k 10 780 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu "$@" > "$out/tests.log" 2>&1
rc=$?
echo "pytest rc $rc" >> "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
brc=$?
echo "bench rc $brc" >> "$out/bench.err"
exit $brc
