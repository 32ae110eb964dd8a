#!/bin/bash
# straight-line scatter (LDS reads before the stores) vs r28
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r29
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_level.py 3 r28=$L/ab/libvbfm_head.so sc=$L/libvbfm.so r28_split=$L/ab/libvbfm_head.so:VBFM_FORCE_SPLIT=1 sc_split=$L/libvbfm.so:VBFM_FORCE_SPLIT=1 > $O/ab.txt 2>&1 || exit $?
