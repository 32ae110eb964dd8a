#!/bin/bash
# C5 (-method mcmc, C4 data, k = 100) at N = 8 rehearsed on one GPU through the host exchange, against one rank
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_c18
mkdir -p $out
export VBFM_PLACE=0
echo "n1 start $(date +%T)" >> $out/progress.txt
timeout -k 10 400 python3 -u bench.py --method mcmc --steps 1 --warmup 1 --no-cpu-baseline > $out/n1.json 2> $out/n1.log || exit $?
echo "n8 start $(date +%T)" >> $out/progress.txt
timeout -k 10 700 python3 -u bench.py --method mcmc --gpus 8 --transport host --steps 1 --warmup 1 --no-cpu-baseline > $out/n8_host.json 2> $out/n8_host.log
echo "n8 rc=$? $(date +%T)" >> $out/progress.txt
