#!/bin/bash
# multi-rank tests (2-3 ranks sharing the GPU through the host exchange), then the whole GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r23
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 350 --timeout-method thread > $O/multirank.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
