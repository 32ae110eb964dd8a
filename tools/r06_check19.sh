#!/bin/bash
# placement on / off on one fresh lease: C3 and C4 lines
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_c19}
mkdir -p $out
run() { name=$1; shift; echo "$name start $(date +%T)" >> $out/progress.txt
  timeout -k 10 500 env "$@" > $out/$name.json 2> $out/$name.log; rc=$?
  echo "$name rc=$rc $(date +%T)" >> $out/progress.txt; return $rc; }
run c3_place VBFM_PLACE=1 python3 -u bench.py --config c3 --no-cpu-baseline || exit $?
run c3_noplace VBFM_PLACE=0 python3 -u bench.py --config c3 --no-cpu-baseline || exit $?
run c4_noplace VBFM_PLACE=0 python3 -u bench.py --no-cpu-baseline || exit $?
run c4_place VBFM_PLACE=1 python3 -u bench.py --no-cpu-baseline
