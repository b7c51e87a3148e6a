#!/bin/bash
# A/B of variant libraries (build/variants/NAME, tools/build_variant.sh) against the in-tree one:
# bench.py kernel_ms_per_launch and value, interleaved REPS times.  usage: tools/ab_variant.sh REPS NAME...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
REPS=$1; shift
O=$R/gpurun_out; mkdir -p $O
for k in $(seq $REPS); do
  for v in base "$@"; do
    if [ $v = base ]; then L=$R/firedancer_amd/_lib/libfd_ed25519_hip.so; else L=$R/build/variants/$v/libfd_ed25519_hip.so; fi
    FD_ED25519_HIP_LIB=$L timeout -k 10 200 python -u $R/bench.py --no-cpu-baseline > $O/ab_${v}_$k.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/ab_${v}_$k.json'));k=d['kernel_ms_per_launch'];print('$v', '%.2fM'%(d['value']/1e6), ' '.join('%s %.3f'%(a,b) for a,b in k.items()), 'match', d['verdicts_match_reference_labels'])"
  done
done
