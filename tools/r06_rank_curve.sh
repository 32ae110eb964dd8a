#!/bin/bash
# one rank of the N = 2 / 4 / 8 C4 strong-scaling runs on one GPU: the row-sharded split level
# through a 1-rank RCCL communicator (the compute side of the 1 -> 8 curve)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_rank_curve}
mkdir -p $out
for rows in 50000000 25000000 12500000; do
  timeout -k 10 400 python3 -u bench.py --rows $rows --one-rank-comm --steps 2 --warmup 1 --no-cpu-baseline \
    > $out/rank_$rows.json 2> $out/rank_$rows.log || exit $?
done
