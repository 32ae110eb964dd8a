#!/bin/bash
# round 3: the entry-store tests after the two-pass default
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_multihot_gpu.py \
  tests/test_multirank_gpu.py tests/test_checkpoint_gpu.py "tests/test_mcmc_gpu.py::test_mcmc_als_chain_vs_reference" \
  > gpurun_out/r3g/tests.log 2>&1
