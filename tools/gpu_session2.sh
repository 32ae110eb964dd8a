#!/bin/bash
# GPU session: parity tests, smoke, c3 and c4 benches. Stops at the first GPU fault/timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ $1 -gt 128 ] && return 0; return 1; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; if fatal $rc; then echo "fatal pytest"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log; rc=$?
echo "bench c3 rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 900 python bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log; rc=$?
echo "bench c4 rc=$rc"
exit 0
