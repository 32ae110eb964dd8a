#!/bin/bash
# the grid-stride deferred split, records loaded one chunk ahead too (VBFM_DEFER_GS_REC=1), at one
# N = 8 rank's shape through a 1-rank communicator, alternating with the default
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_gs_ab2}
mkdir -p $out
for r in 1 2; do
  for v in off r8 r16 r4; do
    unset VBFM_DEFER_GS VBFM_DEFER_GS_REC
    case $v in r*) export VBFM_DEFER_GS=${v#r} VBFM_DEFER_GS_REC=1;; esac
    timeout -k 10 300 python3 -u bench.py --rows 12500000 --one-rank-comm --steps 3 --warmup 1 --no-cpu-baseline \
      > $out/${v}_$r.json 2> $out/${v}_$r.log || exit $?
  done
done
