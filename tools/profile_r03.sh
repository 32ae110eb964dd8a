#!/bin/bash
# Round-3 profile of the DRIVER's bench command on the final tree, in one lease (VERDICT r02
# item 5): rocprofv3 --kernel-trace --stats of `bench.py --gpus 1 --steps 20 --warmup 5` itself
# (its JSON line -- ms_per_step, the HIP-event launch time -- kept beside the summary), then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes of the same command at 3 steps.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_r03
mkdir -p $out
echo "kt start $(date +%T)" >> $out/progress.txt
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.txt
rc=$?; echo "kt rc=$rc $(date +%T)" >> $out/progress.txt; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c start $(date +%T)" >> $out/progress.txt
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d $out/$c -o p --output-format csv -- \
    python3 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $out/$c.json 2> $out/$c.txt
  rc=$?; echo "pass $c rc=$rc $(date +%T)" >> $out/progress.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
