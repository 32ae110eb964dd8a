#!/bin/bash
# the deferred split's grid-stride form (VBFM_DEFER_GS=<workgroups per CU>) against one workgroup per
# column, at one N = 8 rank's shape through a 1-rank communicator, alternating; free energy and RMSE
# must be identical (bit for bit)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_gs_ab}
mkdir -p $out
for r in 1 2; do
  for g in 0 16 8 32; do
    if [ $g = 0 ]; then unset VBFM_DEFER_GS; else export VBFM_DEFER_GS=$g; fi
    timeout -k 10 300 python3 -u bench.py --rows 12500000 --one-rank-comm --steps 3 --warmup 1 --no-cpu-baseline \
      > $out/gs${g}_$r.json 2> $out/gs${g}_$r.log || exit $?
  done
done
