#!/bin/bash
# the -m gpu suite from test_mcmc_gpu.py on (the files after the first run's failure), then smoke()
set -o pipefail
out=gpurun_out/${1:-suite_rest}
mkdir -p $out
timeout -k 10 1100 python -u -m pytest -m gpu -v --timeout 900 --timeout-method thread \
  tests/test_mcmc_gpu.py tests/test_multihot_gpu.py tests/test_multirank_gpu.py tests/test_online_gpu.py \
  tests/test_ref_binding_gpu.py tests/test_schedule_gpu.py > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
