set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash tools/prof_split.sh
