#!/bin/bash
# the round-end tiers as the driver runs them: the whole -m gpu suite, then smoke()
set -o pipefail
out=gpurun_out/${1:-suite}
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 900 --timeout-method thread ${2:+-k "$2"} \
  > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
