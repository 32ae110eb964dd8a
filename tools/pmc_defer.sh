#!/bin/bash
# SQ counters of the deferred split kernels (slot 0 vs slot 1), C4 rows, k=4, one iteration
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc_defer
mkdir -p $out
VBFM_FORCE_SPLIT=1 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $out/sq -o p --output-format csv -- python3 bench.py --k 4 --steps 1 --warmup 0 --no-cpu-baseline > $out/sq.json 2> $out/sq.txt
