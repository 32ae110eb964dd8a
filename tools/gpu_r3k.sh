#!/bin/bash
# kernel trace of the deferred split at the per-rank size of C4 on 8 GPUs (1.25e7 rows), no
# communicator, against the fused kernel: where the split's extra time per level goes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/r3k
mkdir -p $out
B="bench.py --rows 12500000 --k 8 --steps 2 --warmup 1 --no-cpu-baseline"
VBFM_FORCE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/split -o kt --output-format csv -- \
  python3 $B > $out/split.json 2> $out/split.txt || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/fused -o kt --output-format csv -- \
  python3 $B > $out/fused.json 2> $out/fused.txt || exit $?
