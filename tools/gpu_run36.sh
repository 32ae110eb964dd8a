#!/bin/bash
# round-end rehearsal: the driver's three GPU steps on the committed tree
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r36
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.txt || exit $?
