#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r37
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 350 --timeout-method thread > $O/multirank.txt 2>&1 || exit $?
