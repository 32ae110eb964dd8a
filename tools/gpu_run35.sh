#!/bin/bash
# online per-batch store kernel: staging loads overlapped. GPU online tests + C3 epoch A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r35
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_online_gpu.py tests/test_cli_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 350 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
L=scalable-variational-bayesian-factorization-machine_amd/lib
for r in 0 1 2; do
  VBFM_LIB=$L/ab/libvbfm_head.so timeout -k 10 300 python bench.py --config c3 --method vb_online --no-cpu-baseline > $O/head_$r.json 2> $O/head_$r.txt || exit $?
  timeout -k 10 300 python bench.py --config c3 --method vb_online --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.txt || exit $?
done
