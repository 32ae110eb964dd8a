#!/bin/bash
# online VB on the per-batch level-ordered store: parity tests, C3 bench, kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r17
timeout -k 10 600 python -u -m pytest tests/test_online_gpu.py tests/test_cli_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r17/tests.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --method vb_online --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r17/bench_c3.json 2> gpurun_out/r17/bench_c3.txt || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r17/prof -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --method vb_online --config c3 --steps 1 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r17/bench_c3_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r17/bench_c3_prof.txt
