#!/bin/bash
# long columns on the column layout too; full suite; skew A/B on the column layout; round-end rehearsal
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r40
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k long_columns -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/long.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_skew.py 1 col_noseg=$L/libvbfm.so:VBFM_LAYOUT=column,VBFM_LONG=0 col_seg=$L/libvbfm.so:VBFM_LAYOUT=column > $O/ab.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.txt || exit $?
