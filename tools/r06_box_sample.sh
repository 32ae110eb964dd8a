#!/bin/bash
# the C4 level on whatever box this lease is: a short default-workload bench (no CPU leg)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_box}
mkdir -p $out
timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.log
