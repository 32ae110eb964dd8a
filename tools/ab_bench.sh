#!/bin/bash
# Interleaved A/B of library variants through bench.py (separate processes, A B A B ...):
#   tools/ab_bench.sh <out> <rounds> "<bench args>" label=lib ...   (lib relative to the repo root)
# prints per run the per-level launch time (roofline avg_launch_ms) and ms_per_step
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; rounds=$2; args=$3; shift 3
mkdir -p $out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    label=${spec%%=*}; lib=${spec#*=}
    VBFM_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py $args > $out/${label}_$r.json 2> $out/${label}_$r.log || exit $?
    python3 -c "import json,sys; d=json.load(open('$out/${label}_$r.json')); print('$label', $r, round(d['roofline']['avg_launch_ms']*1e3,1), 'us/level', round(d['ms_per_step'],1), 'ms/step')" | tee -a $out/summary.txt
  done
done
