#!/bin/bash
# the final tree under the driver's multi-rank launch shape: two ranks on one GPU (C2 weak scaling + C4 halves)
set -o pipefail
O=gpurun_out/r5ap; mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 2 --allow-shared-device --steps 5 --warmup 1 --no-cpu-baseline \
  --latency-txns 0 --deployed-txns 0 > $O/bench_n2_shared.json 2> $O/bench_n2_shared.err || exit $?
