#!/bin/bash
# A/B of the occupancy-aware launch shape on the multi-hot bench (interleaved processes)
set -o pipefail
out=gpurun_out/r3h
mkdir -p $out
T="timeout -k 10 300"
for r in 1 2; do
  for v in 0 1; do
    VBFM_SHAPE_ROUNDS=$v $T python -u bench.py --config multihot --steps 3 --warmup 1 \
      > $out/mh_shape${v}_r$r.json 2> $out/mh_shape${v}_r$r.txt || exit $?
  done
done
