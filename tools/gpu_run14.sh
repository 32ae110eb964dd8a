#!/bin/bash
# new parity test (fused train prediction), C2 / C3 bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r14
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_train_prediction or wave_prediction or generated_data" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r14/tests.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r14/bench_c2.json 2> gpurun_out/r14/bench_c2.txt || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 > gpurun_out/r14/bench_c3.json 2> gpurun_out/r14/bench_c3.txt || exit $?
