#!/bin/bash
# round 3: the entry-store MCMC split after the dispatch fix, the per-level tests, then the
# one-GPU A/B of the chunked exchange and the C4 / C5 k=100 config tests
set -o pipefail
mkdir -p gpurun_out/r3c
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_multihot_gpu.py::test_entry_store_split_mcmc_equals_fused" \
  "tests/test_multirank_gpu.py::test_mcmc_row_shards_match_one_rank" \
  tests/test_levels_gpu.py > gpurun_out/r3c/parity.log 2>&1 || exit $?
for v in fused chunks4 chunks1; do
  case $v in
    fused) ENVS=""; FL="" ;;
    chunks4) ENVS=""; FL="--one-rank-comm" ;;
    chunks1) ENVS="VBFM_AR_CHUNKS=1"; FL="--one-rank-comm" ;;
  esac
  env $ENVS $T 300 python -u bench.py --k 8 --steps 3 --warmup 1 --no-cpu-baseline $FL \
     > gpurun_out/r3c/ab_$v.json 2> gpurun_out/r3c/ab_$v.err || exit $?
done
$T 1200 python -u -m pytest -v --timeout 900 --timeout-method thread tests/test_configs_gpu.py -k "c4_k100 or c5_k100" \
  > gpurun_out/r3c/configs.log 2>&1
