#!/bin/bash
# Round-3 GPU evidence in one box session (run via gpurun):
#   1. the GPU test suite
#   2. the drop-in thread-scaling and device-bytes records (pytest -s output)
#   3. the bench with the host-fed leg last (default) and first (--host-first)
# Outputs under gpurun_out/r3e_*; every GPU step has its own time limit and
# the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 400 $T $R/tests -m gpu > $O/r3e_tests.log 2>&1 || { tail -40 $O/r3e_tests.log; exit 1; }
tail -2 $O/r3e_tests.log
timeout -k 10 200 $T -s $R/tests/test_gpu_dropin_threads.py $R/tests/test_gpu_mux_tile.py > $O/r3e_dropin_mux.log 2>&1 \
  || { tail -40 $O/r3e_dropin_mux.log; exit 1; }
grep -E '^\{' $O/r3e_dropin_mux.log || true
timeout -k 10 300 python -u $R/bench.py > $O/r3e_bench_last.json 2> $O/r3e_bench_last.err || { tail -20 $O/r3e_bench_last.err; exit 1; }
timeout -k 10 300 python -u $R/bench.py --host-first > $O/r3e_bench_first.json 2> $O/r3e_bench_first.err \
  || { tail -20 $O/r3e_bench_first.err; exit 1; }
for f in last first; do
  python3 -c "import json,sys;d=json.load(open('$O/r3e_bench_$f.json'));h=d['host_fed'];print('$f', 'value %.2fM'%(d['value']/1e6), 'host_fed %.2fM'%(h['value']/1e6), 'frac_of_pcie %.3f'%h['frac_of_pcie_bound'])"
done
