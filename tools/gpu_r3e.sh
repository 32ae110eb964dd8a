#!/bin/bash
# round 3: the entry store under row shards on one GPU: multi-hot bench
# lines, fused vs the deferred / two-pass split through a 1-rank RCCL communicator; MCMC too
set -o pipefail
out=gpurun_out/r3e
mkdir -p $out
T="timeout -k 10 300"
run() { local name=$1; shift; env "$@" > $out/$name.json 2> $out/$name.txt || exit $?; }
run mh_vb_fused $T python -u bench.py --config multihot --steps 3 --warmup 1
run mh_vb_split_deferred $T python -u bench.py --config multihot --steps 3 --warmup 1 --one-rank-comm
run mh_vb_split_twopass VBFM_DEFER=0 $T python -u bench.py --config multihot --steps 3 --warmup 1 --one-rank-comm
run mh_mcmc_fused $T python -u bench.py --config multihot --method mcmc --steps 3 --warmup 1
run mh_mcmc_split $T python -u bench.py --config multihot --method mcmc --steps 3 --warmup 1 --one-rank-comm
