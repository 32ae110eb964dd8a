#!/bin/bash
# long columns split into segment workgroups: parity test, GPU suite, skewed-data A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r39
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k long_columns -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/long.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_skew.py 2 noseg=$L/libvbfm.so:VBFM_LONG=0 seg=$L/libvbfm.so > $O/ab.txt 2>&1 || exit $?
