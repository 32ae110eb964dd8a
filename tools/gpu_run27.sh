#!/bin/bash
# all stage-in loads in flight (straight-line, unconditional LDS writes): GPU suite + A/B vs 31a33db
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r27
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_level.py 4 head=$L/ab/libvbfm_head.so mlp=$L/libvbfm.so > $O/ab.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.txt || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 600 python bench.py --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/vb_split_k8.json 2> $O/vb_split_k8.txt || exit $?
