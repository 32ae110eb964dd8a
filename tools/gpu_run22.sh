#!/bin/bash
# multi-rank rehearsal on one GPU (2 ranks over RCCL sharing the card) + forced-split C4 k=100
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r22
mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 pass, 1 ordinary failure: go on; anything else: stop
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 tools/multirank_check.py > $O/multirank.txt 2>&1; rc=$?; echo "multirank rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --rows 5000000 --k 8 --steps 2 --warmup 1 > $O/bench_n2_small.json 2> $O/bench_n2_small.txt; rc=$?; echo "bench n2 rc=$rc"; ok $rc || exit $rc
(while true; do rocm-smi --showmeminfo vram --csv 2>/dev/null | tail -1 >> $O/vram.csv; sleep 5; done) &
SMI=$!
VBFM_FORCE_SPLIT=1 timeout -k 10 700 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/split_c4.json 2> $O/split_c4.txt; rc=$?
kill $SMI
echo "split c4 rc=$rc"
exit $rc
