#!/bin/bash
# Round profile of the DEFAULT bench command: rocprofv3 kernel-trace --stats of `bench.py`
# itself (its JSON line kept beside the summary), then FETCH_SIZE / WRITE_SIZE in separate
# --pmc passes over a k=4 run (per-launch bytes of the level kernel do not depend on k).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_final3
mkdir -p $out
echo "kt start $(date +%T)" >> $out/progress.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py > $out/bench.json 2> $out/bench.txt
rc=$?; echo "kt rc=$rc $(date +%T)" >> $out/progress.txt; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c start $(date +%T)" >> $out/progress.txt
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d $out/$c -o p --output-format csv -- \
    python3 bench.py --k 4 --steps 1 --warmup 0 --no-cpu-baseline > $out/$c.json 2> $out/$c.txt
  rc=$?; echo "pass $c rc=$rc $(date +%T)" >> $out/progress.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
