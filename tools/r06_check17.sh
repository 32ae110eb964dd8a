#!/bin/bash
# C4 strong scaling at N = 8 rehearsed on one GPU: eight rank processes (1.25e7 rows each) through the
# host exchange, against one rank over all 1e8 rows, same steps (placement search off: eight searches
# would share one card's memory)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_c17
mkdir -p $out
export VBFM_PLACE=0
echo "n1 start $(date +%T)" >> $out/progress.txt
timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/n1.json 2> $out/n1.log || exit $?
echo "n8 start $(date +%T)" >> $out/progress.txt
timeout -k 10 700 python3 -u bench.py --gpus 8 --transport host --steps 1 --warmup 1 --no-cpu-baseline > $out/n8_host.json 2> $out/n8_host.log
echo "n8 rc=$? $(date +%T)" >> $out/progress.txt
