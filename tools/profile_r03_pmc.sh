#!/bin/bash
# Round-3 PMC passes of the driver's bench command (C4 rows, 3 steps): FETCH_SIZE and WRITE_SIZE
# in separate passes, counters on the level kernel only, k = 4. A counted dispatch costs tens of
# ms (an iteration at k = 100 -- 4000 level dispatches -- ran > 3 min without finishing, and a
# 3-step k = 100 pass segfaulted in the tool's dispatch hook after ~8000 dispatches,
# gpurun_out/prof_r03/FETCH_SIZE.txt); a level launch's bytes do not depend on k or the step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-prof_r03}
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c start $(date +%T)" >> $out/progress.txt
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex k_level_lord -d $out/$c -o p \
    --output-format csv -- python3 bench.py --gpus 1 --k 4 --steps 3 --warmup 0 --no-cpu-baseline \
    > $out/$c.json 2> $out/$c.txt
  rc=$?; echo "pass $c rc=$rc $(date +%T)" >> $out/progress.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
