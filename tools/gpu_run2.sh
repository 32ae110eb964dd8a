set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --method mcmc --steps 1 --warmup 1 > gpurun_out/bench_c4_mcmc_level.json 2> gpurun_out/bench_c4_mcmc_level.log || exit $?
timeout -k 10 300 python bench.py --method mcmc --layout column --steps 1 --warmup 1 > gpurun_out/bench_c4_mcmc_column.json 2> gpurun_out/bench_c4_mcmc_column.log
