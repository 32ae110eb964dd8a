#!/bin/bash
# One lease: the bench line of every path on the current tree (stdout JSON per run under
# gpurun_out/$1/): C4 VB (the metric), C4 MCMC (config 5's Gibbs sweep), C3 online epochs,
# multi-hot rows on the entry store, and C4's per-rank shape on 8 GPUs through a 1-rank RCCL
# communicator (the split kernels every rank of the N = 8 run executes).
set -o pipefail
out=gpurun_out/${1:-bench_all}
mkdir -p $out
run() {
	local name=$1; shift
	timeout -k 10 $1 python -u bench.py "${@:2}" > $out/$name.json 2> $out/$name.err || exit $?
}
run c4_vb 420 --steps 5 --warmup 1
run c4_mcmc 300 --method mcmc --steps 3 --warmup 1
run c3_online 200 --config c3 --method vb_online --steps 3 --warmup 1
run multihot 300 --config multihot --steps 3 --warmup 1 --no-launch-events
run c4_rank_of_8 200 --rows 12500000 --one-rank-comm --steps 5 --warmup 1 --no-cpu-baseline
