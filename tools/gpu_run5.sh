set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || exit $?
VBFM_FORCE_SPLIT=1 timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_split.json 2> gpurun_out/bench_split.log
