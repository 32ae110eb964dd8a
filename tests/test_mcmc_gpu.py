"""Parity of the MCMC / ALS learner on the GPU (vbfm_mcmc_* through the C-ABI) with the
compiled reference's -method mcmc | als runs (tests/golden, pinned bit for bit by the oracle in
test_oracle_golden.py::test_mcmc_als_trace_bit_exact).

With VBFM_RNG_REFERENCE the library takes every random number from the reference's own
stream (srand(seed), glibc rand(), Leva normals, Marsaglia-Tsang gammas) in the reference's
order, so a sampled chain follows the reference's chain. The only differences are the
summation order of the column and data-set reductions (fixed tree on the device, sequential
in the reference): held to REL = 1e-9 relative over the whole chain (north star: 1e-6).
"""
import os

import numpy as np
import pytest

import vbfm
from conftest import GOLDEN, load_case

pytestmark = pytest.mark.gpu
REL = 1e-9

# tiny_dup/als (no regularization) is pinned on the oracle only: its chain is unstable
# (|v| ~ 1e22 by iteration 3, tools/debug_mcmc.py), so summation-order differences of 1e-16
# grow without bound; tiny_dup/als_reg runs the same data with -regular 0.5,1,2.
CASES = ["tiny/als", "synth_als", "tiny/mcmc", "tiny_dup/mcmc", "tiny/mcmc_meta", "tiny/als_reg", "tiny_dup/als_reg",
         "tiny/als_meta_reg", "synth_mcmc", "sa_mcmc"]


def rel_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    scale = max(1e-300, float(np.max(np.abs(b))) if b.size else 1.0)
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def case_files(case, synth_files, sa_split):
    if case.startswith("synth"):
        return synth_files["train"], synth_files["test"]
    if case.startswith("sa_"):
        return sa_split["train"], sa_split["test"]
    d = os.path.join(GOLDEN, case.split("/")[0])
    return os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")


def run_case(case, synth_files, sa_split, rng=vbfm.RNG_REFERENCE):
    t, a = load_case(case)
    m = t["meta"]
    trp, tep = case_files(case, synth_files, sa_split)
    train, test = vbfm.DataSubset.load(trp), vbfm.DataSubset.load(tep)
    k0, k1, k = [int(x) for x in m["dim"].split(",")]
    D = vbfm.num_all_attribute(train, test)
    groups = None
    if "meta" in m:
        groups = vbfm.load_meta(os.path.join(GOLDEN, case.split("/")[0], m["meta"]), D)
    fml = vbfm.FMLearnMCMC(k0, k1, k, D, attr_group=groups, min_target=train.min_target,
                           max_target=train.max_target, method="mcmc" if "mcmc" in case else "als")
    fml.init(m["seed"], m["init_stdev"], regular=m.get("regular", ()), rng=rng)
    stats = list(fml.learn(train, test, m["iter"]))
    return t, a, fml, stats


# data sets whose every dependency level holds each row once: the level-ordered store applies
COMPLETE = ("synth_als", "synth_mcmc", "sa_mcmc")


# layout column is a separate case only where auto picks another layout (the complete-level
# data sets); elsewhere auto already runs the column layout or the entry store
CHAIN_CASES = [(c, s, l) for c in CASES for s in ("fused", "split") for l in ("auto", "column")
               if l == "auto" or c in COMPLETE]


@pytest.mark.parametrize("case,split,layout", CHAIN_CASES)
def test_mcmc_als_chain_vs_reference(case, split, layout, synth_files, sa_split, monkeypatch):
    """The whole chain: per-iteration Train= / Test= values, then the final parameters and
    hyper-priors. split: the row-sharded kernels (statistics, then draw + correction);
    layout auto = the level-ordered row store on the complete-level data sets."""
    if split == "split":
        monkeypatch.setenv("VBFM_FORCE_SPLIT", "1")
    monkeypatch.setenv("VBFM_LAYOUT", layout)
    t, a, fml, stats = run_case(case, synth_files, sa_split)
    if layout == "column":
        expect = "column"
    elif case in COMPLETE:
        expect = "level"
    else:   # levels that miss rows: the entry store (fused, or the two-pass split under row shards),
        # unless a row lists a feature twice
        expect = "column" if case.startswith("tiny_dup") else "entry"
    assert fml.layout() == expect
    for it, st in enumerate(stats):
        ref = t["trace"][it]
        assert st.rng_skipped == 0
        assert abs(st.rmse_all - ref["rmse_all"]) <= REL * ref["rmse_all"], (it, st.rmse_all, ref["rmse_all"])
        assert abs(st.train_rmse - ref["train"]) <= REL * ref["train"], (it, st.train_rmse, ref["train"])
    p = fml.get_params()
    if "final_fm_v" in a:
        assert rel_err(p["v"], a["final_fm_v"]) <= REL
        assert rel_err(p["w"], a["final_fm_w"]) <= REL
    w0, alpha = a["final_mcmc_scalars"]
    assert abs(p["w0"] - w0) <= REL * max(abs(w0), 1e-300)
    assert abs(p["alpha"] - alpha) <= REL * alpha
    for key in ("w_mu", "w_lambda", "v_mu", "v_lambda"):
        if "final_" + key in a:
            assert rel_err(p[key], a["final_" + key]) <= REL, key


def test_mcmc_rccl_one_rank_vs_reference(sa_split, monkeypatch):
    """Every RCCL call of the row-sharded MCMC path through a real 1-rank communicator."""
    monkeypatch.setenv("VBFM_FORCE_COMM", "1")
    t, a = load_case("sa_mcmc")
    m = t["meta"]
    train, test = vbfm.DataSubset.load(sa_split["train"]), vbfm.DataSubset.load(sa_split["test"])
    D = vbfm.num_all_attribute(train, test)
    fml = vbfm.FMLearnMCMC(1, 1, 8, D, min_target=train.min_target, max_target=train.max_target)
    fml.comm_init(1, 0, vbfm.FMLearnMCMC.comm_unique_id())
    fml.init(m["seed"], m["init_stdev"])
    for it, st in enumerate(fml.learn(train, test, m["iter"])):
        assert abs(st.rmse_all - t["trace"][it]["rmse_all"]) <= REL * t["trace"][it]["rmse_all"]


def test_mcmc_predict_is_mean_of_clipped_draws(sa_split):
    """fm_learn_mcmc::predict: pred_sum_all / num_iter, clipped (fm_learn_mcmc.h:355-381);
    its RMSE is the last Test= value."""
    t, a, fml, stats = run_case("sa_mcmc", None, sa_split)
    test = vbfm.DataSubset.load(sa_split["test"])
    pred = fml.predict()
    rmse = float(np.sqrt(np.mean((pred - test.target.astype(np.float64)) ** 2)))
    assert abs(rmse - stats[-1].rmse_all) <= 1e-12 * rmse


def test_device_rng_fused_equals_split_and_is_deterministic(synth_files, monkeypatch):
    """Device-RNG mode: the per-attribute normals are keyed (seed, iteration, factor,
    attribute), so the fused and the row-sharded kernels draw the same chain bit for bit,
    and so does a second run."""
    runs = []
    for split in ("0", "1", "0"):
        monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
        _, _, fml, stats = run_case("synth_mcmc", synth_files, None, rng=vbfm.RNG_DEVICE)
        runs.append(([s.rmse_all for s in stats], fml.get_params()["v"]))
        fml.close()
    assert runs[0][0] == runs[1][0] == runs[2][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    np.testing.assert_array_equal(runs[0][1], runs[2][1])


def test_device_rng_chain_is_statistically_equivalent(synth_files):
    """A different stream, the same posterior: the averaged-prediction RMSE of the device-RNG
    chain stays close to the reference-stream chain's (parity of an MCMC run is statistical
    once the stream differs)."""
    t, _ = load_case("synth_mcmc")
    _, _, _, stats = run_case("synth_mcmc", synth_files, None, rng=vbfm.RNG_DEVICE)
    ref = t["trace"][-1]["rmse_all"]
    assert np.isfinite(stats[-1].rmse_all)
    assert abs(stats[-1].rmse_all - ref) <= 0.05 * ref, (stats[-1].rmse_all, ref)


def test_device_rng_layouts_agree(synth_files, monkeypatch):
    """Device-RNG chain on both row layouts: the column statistics and draws are identical,
    only the data-set sums (alpha, w0) add the rows in another order."""
    runs = {}
    for layout in ("column", "level"):
        monkeypatch.setenv("VBFM_LAYOUT", layout)
        _, _, fml, stats = run_case("synth_mcmc", synth_files, None, rng=vbfm.RNG_DEVICE)
        assert fml.layout() == layout
        runs[layout] = ([s.rmse_all for s in stats], fml.get_params()["v"])
        fml.close()
    assert rel_err(runs["level"][0], runs["column"][0]) <= 1e-10
    assert rel_err(runs["level"][1], runs["column"][1]) <= 1e-10


@pytest.mark.parametrize("case", ["synth_als", "sa_mcmc", "tiny/mcmc_meta"])
def test_wave_prediction_compact_chain_vs_reference(case, synth_files, sa_split, monkeypatch):
    """The per-iteration re-prediction in its large-data form (VBFM_PREDICT=wave): the
    factors read from a compact copy of v (vbk::predict_e_compact, half the bytes of the
    {v, 0} pairs), the cross-factor sums in a butterfly (~1 ulp from the reference's order).
    The whole chain still follows the reference's to REL."""
    monkeypatch.setenv("VBFM_PREDICT", "wave")
    t, a, fml, stats = run_case(case, synth_files, sa_split)
    for it, st in enumerate(stats):
        ref = t["trace"][it]
        assert abs(st.rmse_all - ref["rmse_all"]) <= REL * ref["rmse_all"], (it, st.rmse_all, ref["rmse_all"])
        assert abs(st.train_rmse - ref["train"]) <= REL * ref["train"], (it, st.train_rmse, ref["train"])
    p = fml.get_params()
    if "final_fm_v" in a:
        assert rel_err(p["v"], a["final_fm_v"]) <= REL


def _fused_pair(run, monkeypatch):
    """run() twice: the train re-prediction as its own pass (VBFM_MC_FUSED_PREDICT=0, exact
    reference order) and fused into the v sweeps + the final row pass (default)."""
    monkeypatch.setenv("VBFM_PREDICT", "exact")
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("VBFM_MC_FUSED_PREDICT", fused)
        out.append(run())
    return out


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("case", ["synth_als", "sa_mcmc", "tiny_dup/mcmc", "tiny/mcmc_meta"])
def test_fused_train_prediction_is_bit_identical(case, split, synth_files, sa_split, monkeypatch):
    """The train re-prediction of draw_all's end (fm_learn_mcmc.h:117-348) accumulated inside
    the v sweeps (factor f-1's terms while factor f is swept) + one final row pass: the same
    operations in the reference's order, so every iteration's Train= / Test= values, the final
    parameters and the rows' e equal the separate exact-order prediction's bit for bit (level
    store and column layout, fused and row-sharded split kernels, a repeated feature)."""
    monkeypatch.setenv("VBFM_FORCE_SPLIT", split)

    def run():
        _, _, fml, stats = run_case(case, synth_files, sa_split)
        r = ([(s.rmse_all, s.rmse_this, s.train_rmse, s.alpha, s.w0) for s in stats], fml.get_params()["v"],
             fml.rows()["e"])
        fml.close()
        return r

    a, b = _fused_pair(run, monkeypatch)
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])


@pytest.mark.parametrize("layout", ["level", "column", "entry"])
@pytest.mark.parametrize("k", [0, 1, 2, 3])
def test_fused_train_prediction_few_factors(k, layout, monkeypatch):
    """k = 0 (w terms only), 1 (no accumulating sweep), 2 (one), 3: the fused re-prediction
    against the separate one, device-RNG MCMC on synthetic field data, bit for bit."""
    import synth

    rp, f, v, y = synth.generate(20000, 5, 150, 3, 1)
    rpt, ft, vt, yt = synth.generate(500, 5, 150, 4, 1)
    nf = 5 * 150

    def run():
        fml = vbfm.FMLearnMCMC(1, 1, k, nf + 1, min_target=float(y.min()), max_target=float(y.max()), method="mcmc",
                               layout=layout)
        fml.init_device(9)
        stats = list(fml.learn(vbfm.DataSubset.from_csr(rp, f, v, y, nf),
                               vbfm.DataSubset.from_csr(rpt, ft, vt, yt, nf), 3))
        assert fml.layout() == layout
        r = ([(s.rmse_all, s.train_rmse, s.alpha, s.w0) for s in stats], fml.rows()["e"])
        fml.close()
        return r

    a, b = _fused_pair(run, monkeypatch)
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("method", ["als", "mcmc"])
def test_entry_store_equals_column_layout_mcmc(method):
    """MCMC / ALS on multi-hot rows (levels that miss rows): the entry store and the column
    layout sweep every column's entries in the same order and the data-set sums in row order,
    so the chains agree bit for bit (device-RNG draws keyed by attribute)."""
    import synth

    n, D, lo, hi, k = 15_000, 2000, 3, 30, 4
    tr = synth.generate_multihot(n, D, lo, hi, 5, 1)
    te = synth.generate_multihot(1500, D, lo, hi, 6, 1)
    res = {}
    for layout in ("entry", "column"):
        fml = vbfm.FMLearnMCMC(1, 1, k, D + 1, min_target=1.0, max_target=5.0, method=method, layout=layout)
        fml.init_device(3)
        stats = list(fml.learn(vbfm.DataSubset.from_csr(*tr, D), vbfm.DataSubset.from_csr(*te, D), 3))
        assert fml.layout() == layout
        res[layout] = ([(s.rmse_all, s.train_rmse, s.alpha, s.w0) for s in stats], fml.get_params()["v"],
                       fml.rows()["e"])
        fml.close()
    assert res["entry"][0] == res["column"][0]
    np.testing.assert_array_equal(res["entry"][1], res["column"][1])
    np.testing.assert_array_equal(res["entry"][2], res["column"][2])
