#!/bin/bash
# the round-end tiers as the driver runs them: the full -m gpu suite, then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r06_full}
mkdir -p $out
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 900 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
