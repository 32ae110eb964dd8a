#!/bin/bash
# refreshed bench lines after the load overlap: MCMC C4 (config 5 on one GPU), VB C3, VB C4 column layout
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r31
mkdir -p $O
timeout -k 10 600 python bench.py --method mcmc --no-cpu-baseline > $O/mcmc_c4.json 2> $O/mcmc_c4.txt || exit $?
timeout -k 10 600 python bench.py --config c3 > $O/vb_c3.json 2> $O/vb_c3.txt || exit $?
timeout -k 10 600 python bench.py --layout column --steps 2 --no-cpu-baseline > $O/vb_c4_column.json 2> $O/vb_c4_column.txt || exit $?
