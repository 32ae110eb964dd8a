#!/bin/bash
set -o pipefail
out=gpurun_out/r06_c4
mkdir -p $out
VBFM_COMM_TRACE=1 timeout -k 10 150 python -u tools/stall_diag.py 3 > $out/stall3.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_comm_failure_gpu.py tests/test_placement_gpu.py -m gpu -v --timeout 200 \
  --timeout-method thread > $out/tests.log 2>&1 || exit $?
VBFM_LIB=$PWD/tools/ab_nobarrier/lib/libvbfm.so timeout -k 10 400 python -u -m pytest tests/test_skew_gpu.py -m gpu -v \
  --timeout 200 --timeout-method thread > $out/skew_nobarrier.log 2>&1
echo "nobarrier rc=$?" >> $out/skew_nobarrier.log
timeout -k 10 400 python -u bench.py --rows 12500000 --one-rank-comm --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/bench_orc.json 2> $out/bench_orc.log
