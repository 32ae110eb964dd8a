#!/bin/bash
# the other configs' bench lines on the final tree (one process each)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_lines}
mkdir -p $out
run() { name=$1; shift; echo "$name start $(date +%T)" >> $out/progress.txt
  timeout -k 10 500 python3 -u bench.py "$@" > $out/$name.json 2> $out/$name.log; rc=$?
  echo "$name rc=$rc $(date +%T)" >> $out/progress.txt; return $rc; }
run c3 --config c3 || exit $?
run c2 --config c2 --steps 20 --warmup 3 || exit $?
run mcmc --method mcmc --no-cpu-baseline || exit $?
run multihot --config multihot --no-cpu-baseline || exit $?
run online --config c3 --method vb_online --no-cpu-baseline
