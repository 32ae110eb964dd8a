#!/bin/bash
# A/B: the per-level exchange at the per-rank size of C4 on 8 GPUs (1.25e7 rows, 125k columns per
# level): deferred split kernels alone (no communicator), then through a 1-rank RCCL communicator
# with 1, 2 and 4 chunks per level
set -o pipefail
out=gpurun_out/r3j
mkdir -p $out
T="timeout -k 10 300"
B="python -u bench.py --rows 12500000 --k 16 --steps 3 --warmup 1 --no-cpu-baseline"
for r in 1 2; do
  VBFM_FORCE_SPLIT=1 $T $B > $out/nocomm_r$r.json 2> $out/nocomm_r$r.txt || exit $?
  for c in 1 2 4; do
    VBFM_AR_CHUNKS=$c $T $B --one-rank-comm > $out/c${c}_r$r.json 2> $out/c${c}_r$r.txt || exit $?
  done
done
