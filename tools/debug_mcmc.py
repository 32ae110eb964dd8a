"""Side-by-side MCMC/ALS chain: GPU learner vs oracle, per iteration (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd"))
import oracle_ctypes as oc  # noqa: E402
import vbfm  # noqa: E402

case, method, dim, iters, seed = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
d = os.path.join(ROOT, "tests", "golden", case)
trp, tep = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
k0, k1, k = [int(x) for x in dim.split(",")]
tr, te = oc.Data(trp), oc.Data(tep)
D = oc.num_all_attribute(tr, te)
o = oc.ALS(k0, k1, k, D, method=method)
o.init_params(seed, 0.1)
o.attach(tr, te)
train, test = vbfm.DataSubset.load(trp), vbfm.DataSubset.load(tep)
g = vbfm.FMLearnMCMC(k0, k1, k, D, min_target=train.min_target, max_target=train.max_target, method=method)
g.init(seed, 0.1)
g.set_data(train, test)
g.init_caches()
p0g, p0o = g.get_params(), o.params()
print("init v diff", np.max(np.abs(p0g["v"] - p0o["v"])), "w diff", np.max(np.abs(p0g["w"] - p0o["w"])))
for it in range(iters):
    ra, rt, trn = o.iterate()
    st = g.iterate()
    pg, po = g.get_params(), o.params()
    dv = np.abs(pg["v"] - po["v"]).reshape(k, D) if k else np.zeros((0, D))
    dw = np.abs(pg["w"] - po["w"])
    print("iter", it, "rmse_all", st.rmse_all, ra, "train", st.train_rmse, trn, "w0", pg["w0"], po["w0"],
          "alpha", pg["alpha"], po["alpha"], "skips", st.rng_skipped, "nan_v", st.nan_v, st.inf_v, "nan_w", st.nan_w,
          st.inf_w)
    print("   max dw %.3g at %d; max dv %.3g" % (dw.max(), dw.argmax(), dv.max() if dv.size else 0))
    if dv.size and dv.max() > 1e-12:
        f, j = np.unravel_index(dv.argmax(), dv.shape)
        print("   worst v f=%d j=%d gpu=%r ora=%r" % (f, j, pg["v"][f * D + j], po["v"][f * D + j]))
        print("   per-factor max:", dv.max(axis=1))
        print("   features off (f0):", np.nonzero(dv[0] > 1e-12)[0][:20])
    rows = g.rows()
    print("   e diff", np.max(np.abs(rows["e"] - oc.arr(o.s.e, o.s.n_train))))
