#!/bin/bash
# C2 (ML-1M shape) line + kernel trace; one N = 8 rank's level, split vs fused, under the kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r06_c5
mkdir -p $out
timeout -k 10 300 python3 -u bench.py --config c2 --steps 10 --warmup 2 > $out/c2_bench.json 2> $out/c2_bench.log || exit $?
echo "c2 done $(date +%T)" >> $out/progress.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c2_kt -o kt --output-format csv -- \
  python3 bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $out/c2_kt_bench.json 2> $out/c2_kt.log || exit $?
echo "c2 kt done $(date +%T)" >> $out/progress.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/split_kt -o kt --output-format csv -- \
  python3 bench.py --rows 12500000 --k 8 --one-rank-comm --steps 3 --warmup 1 --no-cpu-baseline > $out/split_kt_bench.json 2> $out/split_kt.log || exit $?
echo "split kt done $(date +%T)" >> $out/progress.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/fused_kt -o kt --output-format csv -- \
  python3 bench.py --rows 12500000 --k 8 --steps 3 --warmup 1 --no-cpu-baseline > $out/fused_kt_bench.json 2> $out/fused_kt.log
