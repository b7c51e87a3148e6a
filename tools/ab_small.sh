#!/bin/bash
# small-batch latency A/B of variant libraries (tools/build_variant.sh), interleaved
# usage: tools/ab_small.sh REPS SIZES DSM variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
REPS=$1; SIZES=$2; DSM=$3; shift 3
for rep in $(seq $REPS); do
  for name in "$@"; do
    lib=$R/build/variants/$name/libfd_ed25519_hip.so
    [ "$name" = "main" ] && lib=$R/firedancer_amd/_lib/libfd_ed25519_hip.so
    FD_ED25519_HIP_LIB=$lib timeout -k 10 120 python3 $R/tools/small_batch_probe.py --sizes $SIZES --batches 20 --dsm $DSM \
      | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); p=d['phase_ms_p50']
    print('%-10s n=%-5d wall %.4f  prep %.4f  dsm %.4f' % ('$name', d['n'], d['wall_ms']['p50'], p['hash'], p['dsm']))" || exit 1
  done
done
