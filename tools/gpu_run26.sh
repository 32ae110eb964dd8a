#!/bin/bash
# A/B: HEAD level kernel (x array, no prefetch) vs prefetch with x array vs prefetch without x
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r26
mkdir -p $O
L=scalable-variational-bayesian-factorization-machine_amd/lib
timeout -k 10 1000 python -u tools/ab_level.py 4 head=$L/ab/libvbfm_head.so pf_lx=$L/libvbfm.so:VBFM_LX=1 pf=$L/libvbfm.so > $O/ab.txt 2>&1 || exit $?
