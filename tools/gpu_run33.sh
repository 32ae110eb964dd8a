#!/bin/bash
# pattern probe with all loads in flight, beside the bench kernel in the same call; smoke
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r33
mkdir -p $O
timeout -k 10 300 ./tools/probe_mlp > $O/probe_mlp.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/vb_k8.json 2> $O/vb_k8.txt || exit $?
timeout -k 10 300 ./tools/probe_mlp > $O/probe_mlp2.txt 2>&1 || exit $?
