#!/bin/bash
# Interleaved A/B of environment settings through bench.py (separate processes):
#   tools/ab_env.sh <out> <rounds> "<bench args>" "label:VAR=V,VAR=V" ...
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; rounds=$2; args=$3; shift 3
mkdir -p $out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python3 bench.py $args > $out/${label}_$r.json 2> $out/${label}_$r.log || exit $?
    python3 -c "import json; d=json.load(open('$out/${label}_$r.json')); print('$label', $r, round(d['roofline']['avg_launch_ms']*1e3,1), 'us/launch', round(d['ms_per_step'],3), 'ms/step', d['value'])" | tee -a $out/summary.txt
  done
done
