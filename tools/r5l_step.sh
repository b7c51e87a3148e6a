#!/bin/bash
# parity of the broadcast-routed dsm16; the hash -> scalar chain's parts; then
# the records the round owes: 2-rank C4 rehearsal on one GPU, the LDS
# base-table A/B (time + PMC), fdctl's multi-tile topology curve
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_dropin.py tests/test_gpu_tile.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/ubench/prep_parts_ubench > $O/prep_parts.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --gpus 2 --allow-shared-device --steps 5 --warmup 1 --no-cpu-baseline \
  --latency-txns 0 --deployed-txns 0 > $O/bench_n2_shared.json 2> $O/bench_n2_shared.err || exit $?
timeout -k 10 400 tools/ab.sh 3 main lds_base > $O/ab_lds.txt 2>&1 || exit $?
timeout -k 10 300 tools/pmc_ab.sh 262144 main lds_base > $O/pmc_lds.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/deployed_tiles.py --tiles 1,2,4,8 --runs 2 > $O/deployed_tiles.jsonl 2> $O/deployed_tiles.err
