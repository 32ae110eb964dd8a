#!/bin/bash
# round 6: the exchange's failure handling, the skew guard (product and no-barrier variant) and a
# one-rank-comm bench line with the exchange fields
set -o pipefail
out=gpurun_out/r06_c1
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_comm_failure_gpu.py tests/test_skew_gpu.py -m gpu -v --timeout 200 \
  --timeout-method thread > $out/tests.log 2>&1 || exit $?
# the guard must catch the race: the same test against the library without the barriers (expected to FAIL)
VBFM_LIB=$PWD/tools/ab_nobarrier/lib/libvbfm.so timeout -k 10 400 python -u -m pytest tests/test_skew_gpu.py -m gpu -v \
  --timeout 200 --timeout-method thread > $out/skew_nobarrier.log 2>&1
echo "nobarrier rc=$?" >> $out/skew_nobarrier.log
timeout -k 10 400 python -u bench.py --rows 12500000 --one-rank-comm --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/bench_orc.json 2> $out/bench_orc.log
