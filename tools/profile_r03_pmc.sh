#!/bin/bash
# Round-3 PMC passes of the driver's bench command (C4, k = 100): FETCH_SIZE and WRITE_SIZE in
# separate passes, counters on the level kernel only. One iteration (4000 level dispatches):
# the tool segfaulted in its dispatch hook after ~8000 counted dispatches of a 3-step run
# (gpurun_out/prof_r03/FETCH_SIZE.txt); the per-launch bytes do not depend on the step count.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_r03
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c start $(date +%T)" >> $out/progress.txt
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex k_level_lord -d $out/$c -o p \
    --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 0 --no-cpu-baseline \
    > $out/$c.json 2> $out/$c.txt
  rc=$?; echo "pass $c rc=$rc $(date +%T)" >> $out/progress.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
