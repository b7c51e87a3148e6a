#!/bin/bash
# Per-kernel PMC counters of variant libraries (tools/build_variant.sh) on the
# bench workload, one rocprofv3 pass per counter set (each set must fit the
# hardware's per-block limits: <= 8 SQ_, <= 4 TCC_, ...).
#   usage: tools/pmc_sets_ab.sh N "SET1" ["SET2" ...] -- variant...
# Prints one line per (variant, kernel) with every counter averaged per dispatch.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
SETS=()
while [ "$1" != "--" ]; do SETS+=("$1"); shift; done
shift
P="python3 $R/bench.py --n $N --steps 2 --warmup 0 --no-cpu-baseline --latency-txns 0 --host-reps 0"
for name in "$@"; do
  lib=$R/build/variants/$name/libfd_ed25519_hip.so
  [ "$name" = "main" ] && lib=$R/firedancer_amd/_lib/libfd_ed25519_hip.so
  O=$R/gpurun_out/pmcsets_$name
  rm -rf $O; mkdir -p $O
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    FD_ED25519_HIP_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmc$i -o run --output-format csv -- $P \
      > /dev/null 2> $O/pmc$i.err || exit $?
  done
  python3 $R/tools/pmc_summary.py $O/summary.json $O/pmc* --n $N > /dev/null || exit $?
  python3 - $O/summary.json $name <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("fd_ed25519_dsm_kernel", "fd_ed25519_decode_kernel", "fd_ed25519_hash_kernel"):
    if k in d:
        per = d[k]["per_dispatch"]
        print(sys.argv[2], k.replace("fd_ed25519_", ""), " ".join(f"{c}={v:.4g}" for c, v in sorted(per.items())))
EOF
done
