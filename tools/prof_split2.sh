#!/bin/bash
# C4 rows, k=8: deferred split (VBFM_FORCE_SPLIT=1) and fused level kernels, same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_split2
VBFM_FORCE_SPLIT=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split2/split -o kt --output-format csv -- python3 bench.py --k 8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_split2/split.json 2> gpurun_out/prof_split2/split.txt || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split2/fused -o kt --output-format csv -- python3 bench.py --k 8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_split2/fused.json 2> gpurun_out/prof_split2/fused.txt
