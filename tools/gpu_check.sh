#!/bin/bash
# One GPU round trip: parity tests, then the benchmark (JSON on stdout).
# usage: tools/gpu_check.sh [tag] [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}; shift
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $R/gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 $R/gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { tail -40 $R/gpurun_out/${TAG}_tests.log; exit $rc; }
timeout -k 10 300 python -u $R/bench.py "$@" > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}_bench.err
rc=$?
tail -3 $R/gpurun_out/${TAG}_bench.err
cat $R/gpurun_out/${TAG}_bench.json
exit $rc
