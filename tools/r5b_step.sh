set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_dropin_fault.py > $O/tests.log 2>&1; echo "pytest rc $?" >> $O/tests.log
timeout -k 10 400 tools/ab.sh 3 main lds_base > $O/ab_lds.txt 2>&1 || exit $?
timeout -k 10 300 tools/pmc_ab.sh 262144 main lds_base > $O/pmc_lds.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/deployed_tiles.py --tiles 1,2,4,8 --runs 2 > $O/deployed_tiles.jsonl 2> $O/deployed_tiles.err
