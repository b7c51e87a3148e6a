#!/bin/bash
# Batches in flight x engine streams, interleaved (run on the box).
# usage: tools/inflight_ab.sh REPS STEPS "SPEC" ...   SPEC = bench.py arguments
R=${GRAFT_REPO_ROOT:-$(pwd)}
REPS=$1; STEPS=$2; shift 2
B="python3 $R/bench.py --steps $STEPS --no-cpu-baseline --latency-txns 0 --host-reps 0"
for rep in $(seq $REPS); do
  for spec in "$@"; do
    out=$(timeout -k 10 200 $B $spec 2>/dev/null) || { echo "$spec FAILED"; exit 1; }
    echo "$out" | python3 -c "import json,sys;d=json.load(sys.stdin);c=d['config'];print('%-34s %.2fM/s  in flight %d, %s, ok=%s'%('$spec' or 'default',d['value']/1e6,c['batches_in_flight'],c['engine_streams'],d['verdicts_match_reference_labels']))"
  done
done
