#!/bin/bash
# round 3: the entry store's split forms without a communicator (kernel cost alone) and the
# column layout's split (the N > 1 fallback of round 2) on the multi-hot bench
set -o pipefail
out=gpurun_out/r3f
mkdir -p $out
T="timeout -k 10 300"
run() { local name=$1; shift; env "$@" > $out/$name.json 2> $out/$name.txt || exit $?; }
run mh_vb_split_deferred_nocomm VBFM_FORCE_SPLIT=1 $T python -u bench.py --config multihot --steps 3 --warmup 1 --no-cpu-baseline
run mh_vb_split_twopass_nocomm VBFM_FORCE_SPLIT=1 VBFM_DEFER=0 $T python -u bench.py --config multihot --steps 3 --warmup 1 --no-cpu-baseline
run mh_vb_column_split $T python -u bench.py --config multihot --layout column --steps 3 --warmup 1 --one-rank-comm
run mh_vb_column_fused $T python -u bench.py --config multihot --layout column --steps 3 --warmup 1
