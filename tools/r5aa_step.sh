#!/bin/bash
# C5 in-process at high and low offered load under the kernel tracer: do
# concurrent batches stretch each other's kernels (tools/concurrency_stats.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5aa; mkdir -p $O
for r in 4000000 500000; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$r -o run --output-format csv -- \
    python3 tools/latency_rates_probe.py --rates $r --txns 200000 --runs 1 > $O/probe_$r.txt 2>&1 || exit $?
done
