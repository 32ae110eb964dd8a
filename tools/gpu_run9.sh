set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/online
timeout -k 10 600 python -m pytest tests/test_online_gpu.py tests/test_cli_gpu.py -q -x > gpurun_out/online/tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --method vb_online --config c3 --steps 2 --warmup 1 > gpurun_out/online/bench_c3.json 2> gpurun_out/online/bench_c3.log || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/online/prof -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --method vb_online --config c3 --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/gpurun_out/online/bench_c3_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/online/bench_c3_prof.log
