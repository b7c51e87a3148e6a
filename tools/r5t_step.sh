#!/bin/bash
# where the latency goes at low load: in-process vs deployed at the same offered rates
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 300 python -u tools/latency_rates_probe.py --rates 28000,57000,570000,2400000 > $O/inproc_rates.txt 2>&1 || exit $?
for r in 28000 570000; do
  timeout -k 10 200 python -u tools/deployed_probe.py --mode host-parse --rate $r --runs 2 --txns 20000 --slots 8 \
    --hw-queues 8 --pin > $O/deployed_$r.txt 2>&1 || exit $?
done
