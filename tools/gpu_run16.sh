#!/bin/bash
# full GPU suite; MCMC C4 bench (pipelined wave prediction); online C3 bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r16/tests.txt 2>&1 || exit $?
timeout -k 10 900 python bench.py --method mcmc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r16/bench_mcmc_c4.json 2> gpurun_out/r16/bench_mcmc_c4.txt || exit $?
timeout -k 10 600 python bench.py --method vb_online --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r16/bench_online_c3.json 2> gpurun_out/r16/bench_online_c3.txt || exit $?
