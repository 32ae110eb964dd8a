#!/bin/bash
# column-gather kernels: entry loads and record gathers issued unconditionally (all in flight)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r32
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_level.py 3 head_col=$L/ab/libvbfm_head.so:VBFM_LAYOUT=column col=$L/libvbfm.so:VBFM_LAYOUT=column > $O/ab.txt 2>&1 || exit $?
