#!/bin/bash
# round 3: C3 k=50 against the reference's fixture; the one-rank-comm bench line; the default
# bench with the concurrent CPU leg (2e7-row sample)
set -o pipefail
mkdir -p gpurun_out/r3d
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 500 --timeout-method thread \
  "tests/test_configs_gpu.py::test_c3_k50_two_iterations_vs_reference" > gpurun_out/r3d/c3k50.log 2>&1 || exit $?
$T 300 python -u bench.py --k 8 --steps 3 --warmup 1 --no-cpu-baseline --one-rank-comm \
   > gpurun_out/r3d/ab_chunks4.json 2> gpurun_out/r3d/ab_chunks4.err || exit $?
$T 900 python -u bench.py > gpurun_out/r3d/bench_default.json 2> gpurun_out/r3d/bench_default.err
