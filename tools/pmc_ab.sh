#!/bin/bash
# PMC comparison of variant libraries (tools/build_variant.sh) on the bench
# workload: VALU mix and HBM read per kernel.  usage: tools/pmc_ab.sh N variant...
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
P="python3 $R/bench.py --n $N --steps 2 --warmup 0 --no-cpu-baseline --latency-txns 0 --deployed-txns 0 --host-reps 0 --c4-signatures 0"
for name in "$@"; do
  lib=$R/build/variants/$name/libfd_ed25519_hip.so
  [ "$name" = "main" ] && lib=$R/firedancer_amd/_lib/libfd_ed25519_hip.so
  O=$R/gpurun_out/pmcab_$name
  mkdir -p $O
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_SALU" \
             "FETCH_SIZE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"; do
    i=$((i+1))
    FD_ED25519_HIP_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmc$i -o run --output-format csv -- $P \
      > /dev/null 2> $O/pmc$i.err || exit $?
  done
  echo "== $name"
  python3 $R/tools/pmc_summary.py $O/pmc_summary.json $O/pmc1 $O/pmc2 $O/pmc3 --n $N | grep -E "dsm|fix|decode|hash_kernel"
done
