#!/bin/bash
# placement budget A/B on one lease: 48 GiB (8 candidates at C4) vs 96 GiB (16), alternating
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_budget}
mkdir -p $out
for i in 1 2; do
  for b in 48 96; do
    VBFM_PLACE_BUDGET_GB=$b timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/b${b}_$i.json 2> $out/b${b}_$i.log || exit 1
  done
done
