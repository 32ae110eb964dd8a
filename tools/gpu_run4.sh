set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python - > gpurun_out/replay_c4.log 2>&1 <<'PY'
import sys, time
sys.path.insert(0, "scalable-variational-bayesian-factorization-machine_amd")
import vbfm
k, D = 100, 5_000_001
g = vbfm.FMLearnVB(1, 1, k, D)
t = time.time(); g.init_replay(1, 0.1); t1 = time.time() - t
t = time.time(); g.init_replay(1, 0.1); t2 = time.time() - t
print("replay init k=%d D=%d: %.2f s (first), %.2f s (second)" % (k, D, t1, t2))
PY
