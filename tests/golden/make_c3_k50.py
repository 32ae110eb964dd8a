#!/usr/bin/env python3
"""Generate tests/golden/c3_k50/ (and c4_k100_r1e7/) from the COMPILED REFERENCE at the
BASELINE configs' own sizes.

C3: 1e7 train rows x 40 one-hot fields x 25,000 ids (D = 1e6 + 1), nnz 4e8,
k = 50; test = 1e5 rows. Data: tests/synth.py `generate` (train seed 1000, test seed 500000,
xmode 1 = real-valued x, model seed 7), written in the reference's binary format
(.x/.xt/.y, fmatrix.h:46-52) and loaded by the reference's own Data::load (Data.h:112-171).
Run: oracle/_ref/ref_driver vb (the reference's fm_learn_vb_simultaneous + update_all
compiled from /root/reference/src, fm_learn_vb_simultaneous.h:75-258) with --seed 3
--init_stdev 0.1 --dim 1,1,50 for ITERS iterations. About 30 min of one CPU core per
iteration in the build container.

The committed fixture is small: the per-iteration trace the reference prints at 17 digits
(test RMSE, MAE, the train quirk, alpha, sigma_0, mu_0_dash, sigma_0_dash, free energy and the
sums sq_mu_w / sum_sigma_w / sq_mu_v / sum_sigma_v), plus, of the final parameters (SURVEY §4
item 2), the sum and sum of squares of every array, all hyper parameters, and the values at
4096 fixed indices of mu_w / sigma_w / mu_v / sigma_v (and of the initial caches e, t and the
initial test prediction). The GPU test (tests/test_configs_gpu.py) regenerates the same data on
the device (bit-exact generator) and compares.

Case c4_k100_r1e7: config 4's feature space and k (40 one-hot fields x 125,000 ids, D = 5e6 + 1,
k = 100) on the first 1e7 rows of the bench's own C4 data set (train seed 1000, x = 1; test: the
first 1e5 rows of its test set, seed 500000) -- the full 1e8 rows need more memory than the
build container has and ~9 h per reference iteration; one iteration here takes ~2.5 h.

Cases c5_mcmc_k100_r1e7 / c5_als_k100_r1e7 (config 5): the same data as c4_k100_r1e7, run through
the reference's fm_learn_mcmc_simultaneous (ref_driver mcmc | als, fm_learn_mcmc_simultaneous.h:
50-305) with k = 100, seed 3, init_stdev 0.1, no -regular, one iteration: the per-iteration
"#Iter=" trace at 17 digits (train quirk, test RMSE of the averaged prediction), w0 and alpha,
the sums and 4096 sampled values of the final v, w and hyper-priors (w_mu, w_lambda, v_mu,
v_lambda).

Usage: python tests/golden/make_c3_k50.py [--case c3_k50|c4_k100_r1e7|c5_mcmc_k100_r1e7|c5_als_k100_r1e7]
       [--iter 2] [--ref ...] [--tmp DIR (data kept there, shared between cases)]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import synth  # noqa: E402
from make_golden import parse_mcmc, parse_vb  # noqa: E402

CASES = {
    "c3_k50": {"n_rows": 10_000_000, "n_fields": 40, "ids_per_field": 25_000, "seed": 1000, "xmode": 1,
               "test_rows": 100_000, "test_seed": 500000, "model_seed": synth.MODEL_SEED,
               "dim": "1,1,50", "init_stdev": 0.1, "ref_seed": 3},
    "c4_k100_r1e7": {"n_rows": 10_000_000, "n_fields": 40, "ids_per_field": 125_000, "seed": 1000, "xmode": 0,
                     "test_rows": 100_000, "test_seed": 500000, "model_seed": synth.MODEL_SEED,
                     "dim": "1,1,100", "init_stdev": 0.1, "ref_seed": 3},
}
for _mode in ("mcmc", "als"):
    CASES["c5_%s_k100_r1e7" % _mode] = dict(CASES["c4_k100_r1e7"], mode=_mode)
MCMC_ARRAYS = ("final_fm_v", "final_fm_w", "final_mcmc_scalars", "final_w_mu", "final_w_lambda", "final_v_mu",
               "final_v_lambda")
VB_ARRAYS = ("final_mu_w", "final_sigma_w", "final_mu_v", "final_sigma_v", "final_hyp_sigma_w",
             "final_hyp_sigma_v", "final_scalars", "init_mu_w", "init_mu_v", "init_e", "init_t", "init_test_e")
SPEC = CASES["c3_k50"]
N_SAMPLE = 4096


def sample_index(n, salt):
    """4096 fixed indices into an array of n values (the same on both sides of the test)."""
    return np.unique((synth.h(4242, salt, np.arange(N_SAMPLE, dtype=np.uint64)) % np.uint64(n)).astype(np.int64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.path.join(HERE, "..", "..", "oracle", "_ref", "ref_driver"))
    ap.add_argument("--iter", type=int, default=2)
    ap.add_argument("--case", default="c3_k50", choices=sorted(CASES))
    ap.add_argument("--tmp", default="")
    args = ap.parse_args()
    ref = os.path.abspath(args.ref)
    tmp = os.path.abspath(args.tmp or tempfile.mkdtemp(prefix="c3k50_"))
    os.makedirs(tmp, exist_ok=True)
    s = CASES[args.case]
    F, S = s["n_fields"], s["ids_per_field"]
    t0 = time.time()
    if not os.path.exists(os.path.join(tmp, "train.y")):
        rp, f, v, y = synth.generate(s["n_rows"], F, S, s["seed"], s["xmode"])
        synth.write_binary(os.path.join(tmp, "train"), F * S, rp, f, v, y)
        del rp, f, v, y
        rp, f, v, y = synth.generate(s["test_rows"], F, S, s["test_seed"], s["xmode"])
        synth.write_binary(os.path.join(tmp, "test"), F * S, rp, f, v, y)
        del rp, f, v, y
    print("data written in %.0f s" % (time.time() - t0), flush=True)
    dump = os.path.join(tmp, "dump_" + args.case)
    os.makedirs(dump, exist_ok=True)
    t0 = time.time()
    mode = s.get("mode", "vb")
    cmd = [ref, mode, "--train", os.path.join(tmp, "train"), "--test", os.path.join(tmp, "test"),
           "--dim", s["dim"], "--iter", str(args.iter), "--seed", str(s["ref_seed"]),
           "--init_stdev", str(s["init_stdev"]), "--dump", dump]
    res = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True, check=True)
    ref_s = time.time() - t0
    print("reference run %.0f s" % ref_s, flush=True)
    with open(os.path.join(tmp, "ref_stdout_%s.txt" % args.case), "w") as fh:
        fh.write(res.stdout)
    nums, trace = (parse_vb if mode == "vb" else parse_mcmc)(res.stdout)

    def load(name):
        return np.fromfile(os.path.join(dump, name + ".f64"), dtype="<f8")

    sums, samples = {}, {}
    for name in (VB_ARRAYS if mode == "vb" else MCMC_ARRAYS):
        a = load(name)
        sums[name] = [float(np.sum(a)), float(np.sum(a * a)), int(a.size)]
        if a.size > N_SAMPLE:
            idx = sample_index(a.size, len(samples) + 11)
            samples[name + "__idx"] = idx
            samples[name] = a[idx]
        else:
            samples[name] = a
    out = os.path.join(HERE, args.case)
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "trace.json"), "w") as fh:
        json.dump({"nums": nums, "trace": trace, "array_sums": sums,
                   "meta": dict(s, iter=args.iter, ref_seconds=ref_s,
                                generator="tests/golden/make_c3_k50.py")}, fh, indent=1)
    np.savez_compressed(os.path.join(out, "arrays.npz"), **samples)
    print("fixture written under", out, flush=True)
    if not args.tmp:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
