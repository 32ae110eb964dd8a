#!/bin/bash
# resident-run prefetch of x / next positions in the fused level kernels (VB, MCMC)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r25
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.txt || exit $?
timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/vb_fused_k8.json 2> $O/vb_fused_k8.txt || exit $?
VBFM_LX=1 timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/vb_fused_k8_lx.json 2> $O/vb_fused_k8_lx.txt || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/vb_split_k8.json 2> $O/vb_split_k8.txt || exit $?
timeout -k 10 600 python bench.py --method mcmc --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/mc_fused_k8.json 2> $O/mc_fused_k8.txt || exit $?
