set -o pipefail
for r in 1 2 3; do for h in extended strict; do
timeout -k 10 200 python3 bench.py --steps 10 --no-cpu-baseline --latency-txns 0 --half $h 2>/dev/null | python3 -c "import json,sys;d=json.load(sys.stdin);k=d['kernel_ms_per_launch'];print('%-9s %7.2fM/s dsm %.3f decode %.3f scalar %.3f ok=%s'%('$h',d['value']/1e6,k['dsm'],k['decode'],k['scalar'],d['verdicts_match_reference_labels']))" || exit 1
done; done
