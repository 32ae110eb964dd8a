#!/bin/bash
# MCMC deferred split: parity tests, forced-split C4 bench at k=8
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r19
timeout -k 10 600 python -u -m pytest tests/test_mcmc_gpu.py tests/test_cli_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r19/tests.txt 2>&1 || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 600 python bench.py --method mcmc --k 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r19/mc_split_k8.json 2> gpurun_out/r19/mc_split_k8.txt || exit $?
