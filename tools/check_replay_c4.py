"""One-off full-size check: vbfm_init_params_replay == vbfm_init_params_host at C4's model
size (k = 100, D = 5e6 + 1: ~1e9 normals, ~2.7e9 glibc outputs). Prints both timings."""
import sys
import time

import numpy as np

sys.path.insert(0, "scalable-variational-bayesian-factorization-machine_amd")
import vbfm  # noqa: E402

k, D, seed = 100, 5_000_001, 7
a = vbfm.FMLearnVB(1, 1, k, D)
t = time.time()
a.init(seed, 0.1)
th = time.time() - t
pa = a.get_params()
a.close()
b = vbfm.FMLearnVB(1, 1, k, D)
t = time.time()
b.init_replay(seed, 0.1)
tr = time.time() - t
pb = b.get_params()
ok = all(np.array_equal(pa[x], pb[x]) for x in ("mu_w", "sigma_w", "mu_v", "sigma_v"))
print("host init %.1f s (incl. upload), device replay %.2f s, identical: %s" % (th, tr, ok))
sys.exit(0 if ok else 1)
