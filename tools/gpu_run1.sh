set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_level.json 2> gpurun_out/bench_c4_level.log
