#!/bin/bash
set -o pipefail
out=gpurun_out/r06_c3
mkdir -p $out
VBFM_COMM_TRACE=1 timeout -k 10 150 python -u tools/stall_diag.py 3 > $out/stall3.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_placement_gpu.py tests/test_checkpoint_gpu.py -m gpu -v --timeout 200 \
  --timeout-method thread > $out/tests.log 2>&1
