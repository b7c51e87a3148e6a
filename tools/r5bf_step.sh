#!/bin/bash
# issue rate of the latency form's kernels: one PMC pass (SQ counters only) over 1-signature batches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5bf; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d $O/pmc -o run --output-format csv -- \
  python3 tools/small_batch_probe.py --sizes 1 --batches 20 --dsm r16 > $O/probe.txt 2> $O/pmc.err || exit $?
