#!/bin/bash
# round 3: chunked per-level exchange parity + A/B on one GPU, and the C4/C5 k=100 config tests
set -o pipefail
mkdir -p gpurun_out/r3b
T="timeout -k 10"
$T 900 python -u -m pytest -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity.py::test_trace_movielens_split_vs_reference" \
  "tests/test_gpu_parity.py::test_chunked_exchange_is_bit_identical" \
  tests/test_multirank_gpu.py tests/test_multihot_gpu.py tests/test_levels_gpu.py \
  > gpurun_out/r3b/parity.log 2>&1 || exit $?
for v in fused chunks4 chunks1; do
  case $v in
    fused) ENVS=""; FL="" ;;
    chunks4) ENVS=""; FL="--one-rank-comm" ;;
    chunks1) ENVS="VBFM_AR_CHUNKS=1"; FL="--one-rank-comm" ;;
  esac
  env $ENVS $T 300 python -u bench.py --k 8 --steps 3 --warmup 1 --no-cpu-baseline $FL \
     > gpurun_out/r3b/ab_$v.json 2> gpurun_out/r3b/ab_$v.err || exit $?
done
$T 1200 python -u -m pytest -v --timeout 900 --timeout-method thread tests/test_configs_gpu.py -k "c4_k100 or c5_k100" \
  > gpurun_out/r3b/configs.log 2>&1
