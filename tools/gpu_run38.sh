#!/bin/bash
# long-column (chunked) path: x / next positions prefetched per chunk. GPU suite + skewed-data A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r38
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_skew.py 3 head=$L/ab/libvbfm_head.so new=$L/libvbfm.so > $O/ab.txt 2>&1 || exit $?
