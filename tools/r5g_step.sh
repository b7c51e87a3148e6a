#!/bin/bash
# where the latency form's prep time goes: the one-lane phase kernels at small sizes
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 200 python -u tools/small_batch_probe.py --sizes 64,64,256,1024 --batches 20 --forms 0,0 \
    > $O/small_wide.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/small_batch_probe.py --sizes 64,64,256,1024 --batches 20 --dsm r16 \
    > $O/small_r16.txt 2>&1 || exit $?
