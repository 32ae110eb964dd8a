#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per pass) of one bench step, with progress.
# usage: tools/profile_pmc.sh <config> <tag> [extra bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
cfg=${1:-c3}; tag=${2:-run}; shift 2
export TMPDIR=/tmp
out=gpurun_out/pmc_${tag}
mkdir -p $out
B="bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline $*"
for c in FETCH_SIZE WRITE_SIZE; do
  echo "pass $c start $(date +%T)" >> $out/progress.txt
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d $out/$c -o p --output-format csv -- python3 $B > $out/$c.log 2>&1
  rc=$?; echo "pass $c rc=$rc $(date +%T)" >> $out/progress.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
