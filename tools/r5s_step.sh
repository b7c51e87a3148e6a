#!/bin/bash
# the full default bench line on the current tree (C5 legs after the latency-form changes)
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc $?" >> $O/bench.err
