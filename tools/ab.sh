#!/bin/bash
# A/B variant libraries (tools/build_variant.sh) in one GPU session, interleaved.
# usage: tools/ab.sh REPS SPEC...   SPEC = variant[,ENV=VAL...]   (variant "main" = in-tree lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
REPS=$1; shift
for rep in $(seq $REPS); do
  for spec in "$@"; do
    name=${spec%%,*}; envs=""
    [ "$spec" != "$name" ] && envs=$(echo ${spec#*,} | tr ',' ' ')
    lib=$R/build/variants/$name/libfd_ed25519_hip.so
    [ "$name" = "main" ] && lib=$R/firedancer_amd/_lib/libfd_ed25519_hip.so
    out=$(env FD_ED25519_HIP_LIB=$lib $envs timeout -k 10 200 python3 $R/bench.py --steps 10 --no-cpu-baseline \
          --latency-txns 0 --deployed-txns 0 --host-reps 0 --c4-signatures 0 2>/dev/null)
    rc=$?
    # rc 1 with a JSON line = verdict mismatch (expected for timing-only variants); anything else is fatal
    { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } && [ -n "$out" ] || { echo "$spec FAILED rc=$rc"; exit 1; }
    echo "$out" | python3 -c "import json,sys;d=json.load(sys.stdin);k=d['kernel_ms_per_launch'];print('%-28s %7.2fM/s  hash %.3f  decode %.3f  dsm %.3f  scalar %.3f  ok=%s'%('$spec',d['value']/1e6,k['hash'],k['decode'],k['dsm'],k.get('scalar',0),d['verdicts_match_reference_labels']))"
  done
done
