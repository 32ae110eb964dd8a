#!/bin/bash
# deferred split: payload / record / posterior loads overlapped (PAY8 template, unconditional gather)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r28
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 900 python -u tools/ab_level.py 3 head_split=$L/ab/libvbfm_head.so:VBFM_FORCE_SPLIT=1 split=$L/libvbfm.so:VBFM_FORCE_SPLIT=1 fused=$L/libvbfm.so > $O/ab.txt 2>&1 || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 600 python bench.py --method mcmc --k 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/mc_split_k8.json 2> $O/mc_split_k8.txt || exit $?
