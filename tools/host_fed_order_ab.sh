R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
for spec in "" "--host-first" "--inflight 2 --one-stream 0"; do
  out=$(timeout -k 10 200 python3 $R/bench.py --steps 10 --no-cpu-baseline --latency-txns 0 $spec 2>/dev/null) || { echo "$spec FAILED"; exit 1; }
  echo "$out" | python3 -c "import json,sys;d=json.load(sys.stdin);print('%-30s value %.2fM  host_fed %.2fM'%('$spec' or 'default',d['value']/1e6,d['host_fed']['value']/1e6))"
done; done
