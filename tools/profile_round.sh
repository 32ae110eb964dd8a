#!/bin/bash
# Round profile of the default bench workload: rocprofv3 kernel-trace --stats of the bench
# command itself, then FETCH_SIZE / WRITE_SIZE in separate --pmc passes (k=4 to keep them
# short; the per-launch counts of the level kernel do not depend on k).
# usage: tools/profile_round.sh <tag> [extra bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-run}; shift
export TMPDIR=/tmp
out=gpurun_out/prof_${tag}
mkdir -p $out
echo "kt start $(date +%T)" >> $out/progress.txt
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $out/kt_bench.json 2> $out/kt.log
rc=$?; echo "kt rc=$rc $(date +%T)" >> $out/progress.txt; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c start $(date +%T)" >> $out/progress.txt
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d $out/$c -o p --output-format csv -- \
    python3 bench.py --k 4 --steps 1 --warmup 0 --no-cpu-baseline "$@" > $out/$c.json 2> $out/$c.log
  rc=$?; echo "pass $c rc=$rc $(date +%T)" >> $out/progress.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
