#!/bin/bash
# the 96 GiB default: placement tests, then the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_budget_check}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_placement_gpu.py > $out/tests.txt 2>&1 && \
timeout -k 10 900 python3 -u bench.py > $out/bench.json 2> $out/bench.log
