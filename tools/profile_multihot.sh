#!/bin/bash
# Kernel trace + FETCH_SIZE / WRITE_SIZE passes of the multi-hot bench on the entry store
# (k = 8 for the counter passes: the per-launch counts do not depend on k).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_multihot
mkdir -p $out
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py --config multihot --steps 1 --warmup 1 --no-launch-events > $out/kt_bench.json 2> $out/kt.log || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d $out/$c -o p --output-format csv -- \
    python3 bench.py --config multihot --k 8 --steps 1 --warmup 0 --no-launch-events > $out/$c.json 2> $out/$c.log || exit $?
done
exit 0
