#!/bin/bash
# A/B: launch shape at the per-rank size of C4 on 8 GPUs (1.25e7 rows: 100 entries per column and
# level, right at the 64x2 / 256x1 threshold), fused and through a 1-rank RCCL communicator
set -o pipefail
out=gpurun_out/r3i
mkdir -p $out
T="timeout -k 10 300"
for r in 1 2; do
  for sm in 96 128; do
    for fl in fused split; do
      x=""; [ $fl = split ] && x="--one-rank-comm"
      VBFM_SMALL_MAX=$sm $T python -u bench.py --rows 12500000 --k 16 --steps 3 --warmup 1 --no-cpu-baseline $x \
        > $out/s${sm}_${fl}_r$r.json 2> $out/s${sm}_${fl}_r$r.txt || exit $?
    done
  done
done
