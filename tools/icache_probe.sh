#!/bin/bash
# Instruction-cache PMC passes over the bench workload (one pass per counter
# group, no tracing domains): SQC I-cache hits/misses, SQ instruction fetches
# and issue waits per kernel.  usage: tools/icache_probe.sh TAG [N] [lib]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-icache}; N=${2:-262144}; LIB=${3:-$R/firedancer_amd/_lib/libfd_ed25519_hip.so}
O=$R/gpurun_out/$TAG
mkdir -p $O
P="python3 $R/bench.py --n $N --steps 2 --warmup 0 --no-cpu-baseline --latency-txns 0 --host-reps 0"
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  FD_ED25519_HIP_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmc$i -o run --output-format csv -- $P \
    > /dev/null 2> $O/pmc$i.err || { echo "pass $i ($set) failed"; tail -5 $O/pmc$i.err; }
done
python3 $R/tools/pmc_summary.py $O/pmc_summary.json $O/pmc1 $O/pmc2 $O/pmc3 --n $N > /dev/null
python3 - $O/pmc_summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    p = v["per_dispatch"]
    h, m = p.get("SQC_ICACHE_HITS", 0), p.get("SQC_ICACHE_MISSES", 0)
    print(f"{k:40s} icache hit {h:.3g} miss {m:.3g} ({m / max(h + m, 1):.4f}) dup {p.get('SQC_ICACHE_MISSES_DUPLICATE', 0):.3g} "
          f"ifetch {p.get('SQ_IFETCH', 0):.3g} valu {p.get('SQ_INSTS_VALU', 0):.3g} "
          f"wait_inst/wave_cyc {p.get('SQ_WAIT_INST_ANY', 0) / max(p.get('SQ_WAVE_CYCLES', 1), 1):.3f}")
PY
