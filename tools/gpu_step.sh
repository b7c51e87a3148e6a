#!/bin/bash
# One GPU call of the build -> measure loop, as a list of named steps, each
# under its own time limit; the call ends at the first step that fails
# (pytest's rc 1, some tests failed, still lets the next steps run).
#
#   tools/gpu_step.sh OUTDIR STEP [STEP ...]
#
# STEP is NAME[=ARGS][@SECONDS]; ARGS is comma-separated (commas become
# spaces, then '+' becomes ',' for a list inside one argument):
#   tests[=targets]      python -m pytest -m gpu (default: tests)
#   smoke                __graft_entry__.smoke()
#   bench[=args]         python bench.py args      -> OUTDIR/bench.json
#   profile=TAG          tools/profile.sh TAG      (kernel trace + PMC passes)
#   dropin[=calls]       tools/dropin_latency.py   -> OUTDIR/dropin_latency.json
#   small_trace          rocprofv3 kernel trace of 1- and 256-signature batches
#   py=script,args       python -u script args     -> OUTDIR/<script>.txt
#   trace=script,args    rocprofv3 --kernel-trace --stats of python3 script args
#   env=NAME=VALUE       export NAME=VALUE for the steps after it (unset=NAME: unset)
#
# Round 5 ran one hand-written script per session (tools/r5*_step.sh, cited
# by some profiles/r5_* records); they are in git history at 55c5e83.
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%[=@]*}
  if [ "$name" = env ]; then export "${step#env=}"; echo "export ${step#env=}"; continue; fi
  if [ "$name" = unset ]; then unset "${step#unset=}"; continue; fi
  secs=300
  [[ $step == *@* ]] && secs=${step##*@} && step=${step%@*}
  args=""
  [[ $step == *=* ]] && args=${step#*=} && args=${args//,/ } && args=${args//+/,}
  log="$out/$n-$name.log"
  echo "[$(date +%T)] step $n: $name $args (limit ${secs}s)"
  case $name in
    tests)  timeout -k 10 "$secs" python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu ${args:-tests} > "$log" 2>&1
            rc=$?; echo "pytest rc $rc" >> "$log"; tail -3 "$log"
            [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)  timeout -k 10 "$secs" python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$log" 2>&1 || exit $? ;;
    bench)  timeout -k 10 "$secs" python -u bench.py $args > "$out/bench$n.json" 2> "$log" || exit $?
            cat "$out/bench$n.json" | cut -c1-400 ;;
    profile) timeout -k 10 "$secs" tools/profile.sh $args > "$log" 2>&1 || exit $? ;;
    dropin) timeout -k 10 "$secs" python -u tools/dropin_latency.py --calls ${args:-2000} --out "$out/dropin_latency.json" > "$log" 2>&1 || exit $? ;;
    small_trace)
            timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$out/small_trace" -o run --output-format csv -- \
              python3 tools/small_batch_probe.py --sizes 1,256 --batches 40 > "$log" 2>&1 || exit $? ;;
    py)     timeout -k 10 "$secs" python -u $args > "$log" 2>&1 || exit $? ;;
    trace)  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$out/trace$n" -o run --output-format csv -- \
              python3 $args > "$log" 2>&1 || exit $? ;;
    *)      echo "unknown step $name"; exit 2 ;;
  esac
done
echo "[$(date +%T)] all steps done"
