"""Time and sanity-check the MCMC / ALS reference-RNG path at the c5_*_k100_r1e7 fixture's size
(1e7 rows of the C4 data set, k = 100) before the fixture exists: prints one JSON line per
method with the first iteration's Train= / Test= values and the time per call."""
import json
import sys
import time

sys.path.insert(0, "scalable-variational-bayesian-factorization-machine_amd")
import vbfm  # noqa: E402

for method in sys.argv[1:] or ["mcmc", "als"]:
    t0 = time.time()
    F, S, n = 40, 125000, 10_000_000
    g = vbfm.FMLearnMCMC(1, 1, 100, F * S + 1, min_target=1.0, max_target=5.0, method=method)
    g.init(3, 0.1, rng=vbfm.RNG_REFERENCE)
    t1 = time.time()
    g.synth(0, n, F, S, 1000, 0)
    g.synth(1, 100000, F, S, 500000, 0)
    g.init_caches()
    t2 = time.time()
    st = g.iterate()
    t3 = time.time()
    print(json.dumps({"method": method, "layout": g.layout(), "init_s": t1 - t0, "data_s": t2 - t1, "iter_s": t3 - t2,
                      "train": st.train_rmse, "rmse_all": st.rmse_all, "rng_skipped": st.rng_skipped}), flush=True)
    g.close()
