#!/bin/bash
# C3 (BASELINE configs[2], "rocprof HBM GB/s vs roofline"): the bench line and a kernel trace of the
# default C3 bench on the final tree (the PMC passes: r06_c3_pmc.sh, one counter per pass)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r06_c3_trace}
mkdir -p $out
timeout -k 10 400 python3 -u bench.py --config c3 --steps 3 --warmup 1 > $out/bench.json 2> $out/bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 -u bench.py --config c3 --steps 2 --warmup 1 > $out/bench_kt.json 2> $out/bench_kt.log
