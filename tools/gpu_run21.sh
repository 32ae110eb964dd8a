#!/bin/bash
# packed deferred payload: full GPU suite, forced-split C4 benches (VB, MCMC) at k=8
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r21
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > gpurun_out/r21/tests.txt 2>&1 || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r21/vb_split_k8.json 2> gpurun_out/r21/vb_split_k8.txt || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 600 python bench.py --method mcmc --k 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r21/mc_split_k8.json 2> gpurun_out/r21/mc_split_k8.txt || exit $?
timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r21/vb_fused_k8.json 2> gpurun_out/r21/vb_fused_k8.txt || exit $?
