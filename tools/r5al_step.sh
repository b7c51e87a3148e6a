#!/bin/bash
# where the deployed path's p99 tail lies at ~95% of its peak (bench.py's leg settings)
set -o pipefail
O=gpurun_out/r5al; mkdir -p $O
timeout -k 10 400 python -u tools/deployed_probe.py --mode host-parse --rate 3600000 --runs 5 --slots 8 --hw-queues 8 \
  --pin --slow-ms 0.5 --txns 300000 > $O/probe.txt 2>&1 || exit $?
mkdir -p $O/npy && mv gpurun_out/dprobe_host-parse_*.npy $O/npy/
