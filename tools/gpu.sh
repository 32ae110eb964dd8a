#!/bin/bash
# One parameterised GPU-box runner (replaces the per-session scripts).
# usage (from gpurun): bash tools/gpu.sh <outdir> <step> [<step> ...]
#   tests[=<pytest -k expr>]   the -m gpu suite (or a subset; '+' separates words), one process, per-test timeout
#   smoke                      __graft_entry__.smoke()
#   bench[=<args>]             python bench.py <args> > bench.json (args: '+' separates words)
#   prof[=<args>]              rocprofv3 --kernel-trace --stats of bench.py <args>
#   profstat[=<args>]          prof, keeping only the --stats summary
#   pmc[=<args>]               FETCH_SIZE then WRITE_SIZE, one --pmc pass each, of bench.py <args>
#   py=<script>[+args]         python -u <script> <args>
#   exe=<binary>[+args]        a built probe binary
#   sq=<CTRS>@<kernel re>@<args>  one --pmc pass of SQ counters (tools/sq_summary.py), list: rocprofv3 -L
#   pmcpy=<CTRS>@<kernel re>@<script+args>  one --pmc pass of a python script
#   pmcr=<CTRS>@<kernel re>@<iteration range>@<args>  --pmc pass of bench.py on a dispatch range
#   setenv=NAME=VALUE / unsetenv=NAME   environment of the steps that follow
# Every step runs under its own timeout; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p "$O"
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  args=${arg//+/ }
  echo "step $n $step start $(date +%T)" >> "$O/progress.txt"
  case $name in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu -k "$args" -p no:cacheprovider --timeout 400 \
          --timeout-method thread > "$O/tests_$n.txt" 2>&1
      else
        timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 400 \
          --timeout-method thread > "$O/tests_$n.txt" 2>&1
      fi ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$n.txt" 2>&1 ;;
    bench) timeout -k 10 900 python -u bench.py $args > "$O/bench_$n.json" 2> "$O/bench_$n.txt" ;;
    prof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o kt --output-format csv -- \
        python3 bench.py $args > "$O/prof_$n.json" 2> "$O/prof_$n.txt" ;;
    profstat)
      # as prof, keeping only the summary (the per-dispatch trace of a many-launch run is large)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/profstat_$n" -o kt --output-format csv -- \
        python3 bench.py $args > "$O/profstat_$n.json" 2> "$O/profstat_$n.txt"
      rc0=$?; rm -f "$O/profstat_$n/kt_kernel_trace.csv"; (exit $rc0) ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d "$O/pmc_${n}_$c" -o p --output-format csv -- \
          python3 bench.py $args > "$O/pmc_${n}_$c.json" 2> "$O/pmc_${n}_$c.txt" || break
      done ;;
    sq)
      # sq=<COUNTER,COUNTER,...>@<kernel regex>@<bench args>: one --pmc pass (at most 8 SQ_ counters)
      IFS=@ read -r ctrs kre bargs <<< "$arg"
      timeout -s KILL 300 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace --kernel-include-regex "$kre" -d "$O/sq_$n" -o p \
        --output-format csv -- python3 bench.py ${bargs//+/ } > "$O/sq_$n.json" 2> "$O/sq_$n.txt" ;;
    pmcpy)
      # pmcpy=<COUNTER,...>@<kernel regex>@<script+args>: one --pmc pass of a python script
      IFS=@ read -r ctrs kre sargs <<< "$arg"
      timeout -s KILL 600 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace --kernel-include-regex "$kre" -d "$O/pmcpy_$n" -o p \
        --output-format csv -- python3 ${sargs//+/ } > "$O/pmcpy_$n.json" 2> "$O/pmcpy_$n.txt" ;;
    pmcr)
      # pmcr=<COUNTER,...>@<kernel regex>@<iteration range>@<bench args>: one --pmc pass of bench.py
      # counting only the given dispatch iterations of each matching kernel (e.g. [1-400])
      IFS=@ read -r ctrs kre rng bargs <<< "$arg"
      timeout -s KILL 900 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace --kernel-include-regex "$kre" \
        --kernel-iteration-range "$rng" -d "$O/pmcr_$n" -o p --output-format csv -- python3 bench.py ${bargs//+/ } \
        > "$O/pmcr_$n.json" 2> "$O/pmcr_$n.txt" ;;
    list) timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 ;;
    setenv) export "$arg" ;;          # setenv=NAME=VALUE for the steps that follow
    unsetenv) unset "$arg" ;;
    py) timeout -k 10 900 python -u $args > "$O/py_$n.txt" 2>&1 ;;
    exe) timeout -k 10 600 $args > "$O/exe_$n.txt" 2>&1 ;;
    *) echo "unknown step $step" >> "$O/progress.txt"; exit 2 ;;
  esac
  rc=$?
  echo "step $n $step rc=$rc $(date +%T)" >> "$O/progress.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
