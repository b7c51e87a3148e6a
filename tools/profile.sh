#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box via gpurun):
#   1. kernel trace + stats of the full bench (durations per kernel)
#   2. separate PMC passes (no tracing domains mixed in): VALU mix, HBM
#      read (FETCH_SIZE), HBM write (WRITE_SIZE), stalls / LDS / VMEM
# Summaries land in gpurun_out/<tag>_*; copy what is to be judged to profiles/.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
N=${2:-262144}
O=$R/gpurun_out/$TAG
mkdir -p $O
# one batch in flight: each kernel runs alone, so the trace durations are
# comparable with the bench's per-phase HIP events
B="python3 $R/bench.py --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --latency-txns 0 --host-reps 0 --deployed-txns 0 --c4-signatures 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B \
  > $O/trace_bench.json 2> $O/trace.err || exit $?
P="python3 $R/bench.py --n $N --steps 2 --warmup 0 --no-cpu-baseline --latency-txns 0 --host-reps 0 --deployed-txns 0 --c4-signatures 0"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmc$i -o run --output-format csv -- $P > /dev/null 2> $O/pmc$i.err || exit $?
done
python3 $R/tools/pmc_summary.py $O/pmc_summary.json $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 --n $N > $O/pmc_summary.txt
cat $O/trace/run_kernel_stats.csv | cut -d, -f1-4
cat $O/pmc_summary.txt
