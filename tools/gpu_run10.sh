#!/bin/bash
# Re-validate the restored tree: full GPU parity suite, smoke, default bench (C4 VB).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r10
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r10/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r10/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/r10/bench.json 2> gpurun_out/r10/bench.log || exit $?
