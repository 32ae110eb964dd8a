#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_c16
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "long or c2" > $out/tests.log 2>&1 || exit $?
tools/ab_env.sh r06_c16/ab 3 "--config c2 --steps 20 --warmup 3 --no-cpu-baseline" "overlap:VBFM_LONG_OVERLAP=1" "serial:VBFM_LONG_OVERLAP=0"
