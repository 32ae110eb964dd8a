#!/bin/bash
# the placement search over a wider span: 24 candidates, 160 GB budget (C4 records), scores only
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_c20}
mkdir -p $out
VBFM_PLACE_TRIES=24 VBFM_PLACE_BUDGET_GB=160 VBFM_PLACE_LOG=1 timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 0 --k 8 --no-cpu-baseline > $out/wide.json 2> $out/wide.log
