#!/bin/bash
# kernel trace of the default workload on the final tree (the CPU leg skips itself under the profiler)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r06_kt_final}
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o kt -- python3 -u bench.py --steps 2 --warmup 1 > $out/bench.json 2> $out/bench.log
