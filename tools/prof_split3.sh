#!/bin/bash
# C4 rows, k=8: deferred split with and without non-temporal record loads, same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_split3
for nt in 0 1; do
VBFM_DEFER_NT=$nt VBFM_FORCE_SPLIT=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split3/nt$nt -o kt --output-format csv -- python3 bench.py --k 8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_split3/nt$nt.json 2> gpurun_out/prof_split3/nt$nt.txt || exit $?
done
