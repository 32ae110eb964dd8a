"""Pin the oracle (C restatement, oracle/vbfm_oracle.c) against the compiled reference.

The fixtures in tests/golden/ were produced by oracle/_ref/ref_driver, i.e. by the
reference's own fm_learn_vb / fm_learn_mcmc code (tests/golden/make_golden.py). The oracle
must reproduce them BIT FOR BIT: same expressions, same loop order, plain IEEE doubles.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_ctypes as oc
from conftest import GOLDEN, load_case


def test_glibc_rand_restatement_matches_fixture_and_libc():
    kat = json.load(open(os.path.join(GOLDEN, "rng", "glibc_rand.json")))
    libc = ctypes.CDLL(None)
    for seed, expect in kat.items():
        oc.lib().or_srand(int(seed))
        got = [oc.lib().or_rand() for _ in range(len(expect))]
        assert got == expect, seed
        libc.srand(ctypes.c_uint(int(seed)))
        assert [libc.rand() for _ in range(len(expect))] == expect, seed


def _tiny(case):
    d = os.path.join(GOLDEN, case)
    return oc.Data(os.path.join(d, "train.libfm")), oc.Data(os.path.join(d, "test.libfm"))


@pytest.mark.parametrize("case", ["tiny", "tiny_dup"])
def test_loader_counts(case):
    tr, te = _tiny(case)
    t, _ = load_case(case + "/steps")
    n = t["nums"]
    assert tr.num_rows == n["train_rows"] and te.num_rows == n["test_rows"]
    assert tr.num_feature == n["train_nf"] and te.num_feature == n["test_nf"]
    assert oc.num_all_attribute(tr, te) == n["D"]


@pytest.mark.parametrize("case", ["tiny", "tiny_dup"])
def test_vb_steps_bit_exact(case):
    """update_all step by step (fm_learn_vb.h:383-440): every cache and parameter equal."""
    t, a = load_case(case + "/steps")
    m = t["meta"]
    tr, te = _tiny(case)
    k0, k1, k = [int(x) for x in m["dim"].split(",")]
    vb = oc.VB(k0, k1, k, oc.num_all_attribute(tr, te))
    vb.init_params(m["seed"], m["init_stdev"])
    s = vb.s
    np.testing.assert_array_equal(oc.arr(s.fm_v, s.k * s.D), a["init_fm_v"])
    np.testing.assert_array_equal(oc.arr(s.fm_w, s.D), a["init_fm_w"])
    np.testing.assert_array_equal(vb.params()["mu_w"], a["s0_mu_w"])
    np.testing.assert_array_equal(vb.params()["mu_v"], a["s0_mu_v"])
    vb.attach(tr, te)
    vb.init_caches()

    def check_rows(tag):
        r = vb.rows()
        for key in ("e", "t"):
            np.testing.assert_array_equal(r[key], a[tag + "_" + key], err_msg=tag + key)

    check_rows("s0_init")
    np.testing.assert_array_equal(oc.arr(s.e_test, s.n_test), a["s0_init_test_e"])
    vb.step("update_w0")
    check_rows("s1_w0")
    np.testing.assert_array_equal(vb.params()["scalars"], a["s1_scalars"][:4])
    vb.step("update_w_all")
    check_rows("s2_w")
    np.testing.assert_array_equal(vb.params()["mu_w"], a["s2_mu_w"])
    np.testing.assert_array_equal(vb.params()["sigma_w"], a["s2_sigma_w"])
    for f in range(k):
        vb.step("add_main_q", f)
        r = vb.rows()
        for key in ("q", "tq", "tz"):
            np.testing.assert_array_equal(r[key], a["s3_f%d_q_%s" % (f, key)])
        vb.step("update_v_all", f)
        r = vb.rows()
        for key in ("e", "t", "q", "tq", "tz"):
            np.testing.assert_array_equal(r[key], a["s4_f%d_v_%s" % (f, key)])
        p = vb.params()
        np.testing.assert_array_equal(p["mu_v"], a["s4_f%d_v_mu_v" % f])
        np.testing.assert_array_equal(p["sigma_v"], a["s4_f%d_v_sigma_v" % f])


@pytest.mark.parametrize("case", ["tiny", "tiny_dup"])
def test_level_by_level_sweep_ends_at_the_ascending_sweep(case):
    """The reference's update_w / update_v called one dependency level at a time (ref_driver
    levels, tests/golden/<case>/levels) end each sweep exactly where the ascending sweep
    (steps) ends, bit for bit -- the exactness argument of the level schedule
    checked on the reference's own code -- and the levels are the schedule's definition
    (tests/shards.py) on the loaded rows."""
    import shards
    t, a = load_case(case + "/levels")
    _, s = load_case(case + "/steps")
    L = t["meta"]["num_levels"]
    k = int(t["meta"]["dim"].split(",")[2])
    tr, _ = _tiny(case)
    rp, rf, _, _ = tr.csr()
    np.testing.assert_array_equal(a["levels"], shards.levels(rp, rf, tr.num_feature))
    for key in ("e", "t"):
        np.testing.assert_array_equal(a["l_w_l%d_%s" % (L - 1, key)], s["s2_w_" + key])
    for f in range(k):
        for key in ("e", "t", "q", "tq", "tz"):
            np.testing.assert_array_equal(a["l_f%d_l%d_%s" % (f, L - 1, key)], s["s4_f%d_v_%s" % (f, key)])
        for key in ("mu_v", "sigma_v"):
            np.testing.assert_array_equal(a["l_f%d_l%d_%s" % (f, L - 1, key)], s["s4_f%d_v_%s" % (f, key)])
    # intermediate levels are genuinely intermediate (each level changes the caches)
    assert not np.array_equal(a["l_f0_l0_e"], a["l_f0_l%d_e" % (L - 1)])


def _run_vb_trace(case, tr, te, attr_group=None):
    t, a = load_case(case)
    m = t["meta"]
    k0, k1, k = [int(x) for x in m["dim"].split(",")]
    vb = oc.VB(k0, k1, k, oc.num_all_attribute(tr, te), attr_group)
    vb.init_params(m["seed"], m["init_stdev"])
    vb.attach(tr, te)
    vb.init_caches()
    got = []
    for it in range(m["iter"]):
        rmse, mae, trq = vb.iterate()
        got.append((rmse, mae, trq, vb.s.alpha, vb.s.last_free_energy, vb.s.mu_0_dash, vb.params()))
    return t, a, got


def _check_trace(t, a, got, exact=True):
    for it, (rmse, mae, trq, alpha, fe, mu0, p) in enumerate(got):
        ref = t["trace"][it]
        cmp = (lambda x, y: x == y) if exact else (lambda x, y: abs(x - y) <= 1e-12 * max(1.0, abs(y)))
        assert cmp(rmse, ref["rmse"]), (it, rmse, ref["rmse"])
        assert cmp(mae, ref["mae"]), (it, mae, ref["mae"])
        assert cmp(trq, ref["train"]), (it, trq, ref["train"])
        assert cmp(alpha, ref["alpha"]), (it, alpha, ref["alpha"])
        assert cmp(mu0, ref["mu_0_dash"]), it
        assert cmp(fe, ref["free_energy"]), (it, fe, ref["free_energy"])
        key = "iter%d_mu_v" % it
        if key in a:
            np.testing.assert_array_equal(p["mu_v"], a[key])
            np.testing.assert_array_equal(p["sigma_v"], a["iter%d_sigma_v" % it])
            np.testing.assert_array_equal(p["mu_w"], a["iter%d_mu_w" % it])
            np.testing.assert_array_equal(p["hyp_sigma_v"], a["iter%d_hyp_sigma_v" % it])


@pytest.mark.parametrize("case", ["tiny", "tiny_dup"])
def test_vb_trace_tiny_bit_exact(case):
    tr, te = _tiny(case)
    t, a, got = _run_vb_trace(case + "/vb", tr, te)
    _check_trace(t, a, got)


def test_vb_trace_meta_groups_bit_exact():
    tr, te = _tiny("tiny")
    groups = np.loadtxt(os.path.join(GOLDEN, "tiny", "groups.meta"), dtype=np.uint32)
    t, a, got = _run_vb_trace("tiny/vb_meta", tr, te, groups)
    _check_trace(t, a, got)


def test_vb_trace_synth_bit_exact(synth_files):
    tr, te = oc.Data(synth_files["train"]), oc.Data(synth_files["test"])
    t, a, got = _run_vb_trace("synth", tr, te)
    _check_trace(t, a, got)
    p = got[-1][-1]
    np.testing.assert_array_equal(p["mu_v"], a["final_mu_v"])
    np.testing.assert_array_equal(p["sigma_w"], a["final_sigma_w"])


def test_vb_trace_movielens_split_bit_exact(sa_split):
    tr, te = oc.Data(sa_split["train"]), oc.Data(sa_split["test"])
    t, a, got = _run_vb_trace("sa_k8", tr, te)
    _check_trace(t, a, got)
    np.testing.assert_array_equal(got[-1][-1]["mu_w"], a["final_mu_w"])


def regular_to_lambdas(reg, G, k):
    """-regular for mcmc/als (libfm.cpp:367-411) -> (reg0, w_lambda[G], v_lambda[G*k])."""
    reg = list(reg or [])
    if len(reg) == 0:
        r0 = rw = rv = 0.0
    elif len(reg) == 1:
        r0 = rw = rv = reg[0]
    elif len(reg) == 3:
        r0, rw, rv = reg
    else:
        assert len(reg) == 1 + 2 * G
        wl = np.array(reg[1:1 + G])
        vl = np.repeat(np.array(reg[1 + G:1 + 2 * G]), k)
        return reg[0], wl, vl
    return r0, np.full(G, rw), np.full(G * k, rv)


MCMC_CASES = ["tiny/als", "tiny_dup/als", "synth_als", "tiny/mcmc", "tiny_dup/mcmc", "tiny/mcmc_meta",
              "tiny/als_reg", "tiny_dup/als_reg", "tiny/als_meta_reg", "synth_mcmc", "sa_mcmc"]


def run_mcmc_oracle(case, synth_files, sa_split=None):
    t, a = load_case(case)
    m = t["meta"]
    if case.startswith("synth"):
        tr, te = oc.Data(synth_files["train"]), oc.Data(synth_files["test"])
    elif case.startswith("sa_"):
        tr, te = oc.Data(sa_split["train"]), oc.Data(sa_split["test"])
    else:
        tr, te = _tiny(case.split("/")[0])
    k0, k1, k = [int(x) for x in m["dim"].split(",")]
    D = oc.num_all_attribute(tr, te)
    groups = None
    if "meta" in m:
        groups = np.loadtxt(os.path.join(GOLDEN, case.split("/")[0], m["meta"]), dtype=np.uint32)
    method = "mcmc" if "mcmc" in case else "als"
    G = 1 if groups is None else int(groups.max()) + 1
    reg0, wl, vl = regular_to_lambdas(m.get("regular"), G, k)
    als = oc.ALS(k0, k1, k, D, groups, method=method, reg0=reg0)
    als.init_params(m["seed"], m["init_stdev"])
    als.set_lambda(wl, vl)
    als.attach(tr, te)
    got = [als.iterate() for _ in range(m["iter"])]
    return t, a, als, got


@pytest.mark.parametrize("case", MCMC_CASES)
def test_mcmc_als_trace_bit_exact(case, synth_files, sa_split):
    """fm_learn_mcmc_simultaneous::_learn with draw_all, including the hyper-prior draws
    and the rand() stream (glibc restatement), reproduces the reference bit for bit."""
    t, a, als, got = run_mcmc_oracle(case, synth_files, sa_split)
    for it, (rmse_all, rmse_this, train) in enumerate(got):
        ref = t["trace"][it]
        assert rmse_all == ref["rmse_all"], (it, rmse_all, ref["rmse_all"])
        assert train == ref["train"], (it, train, ref["train"])
    p = als.params()
    if "final_fm_v" in a:
        np.testing.assert_array_equal(p["v"], a["final_fm_v"])
        np.testing.assert_array_equal(p["w"], a["final_fm_w"])
    assert p["w0"] == a["final_mcmc_scalars"][0]
    assert p["alpha"] == a["final_mcmc_scalars"][1]
    for key in ("w_mu", "w_lambda", "v_mu", "v_lambda"):
        if "final_" + key in a:
            np.testing.assert_array_equal(p[key], a["final_" + key])


def test_feature_sharded_oracle_one_shard_is_update_all():
    """The feature-sharded restatement with one shard is update_all (up to the e0 + (e - e0)
    rounding of the merge); with two shards it is a different (Jacobi) sweep."""
    import synth
    from shards import feature_shards
    n, F, S, k = 3000, 5, 40, 3
    rp, f, v, y = synth.generate(n, F, S, 12, 1)
    rpt, ft, vt, yt = synth.generate(300, F, S, 13, 1)
    res = {}
    for P in (0, 1, 2):
        o = oc.VB(1, 1, k, F * S + 1)
        o.init_params(4, 0.1)
        o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(300, rpt, ft, vt, yt)))
        o.init_caches()
        for _ in range(2):
            if P == 0:
                o.step("update_all")
            else:
                o.update_all_fsharded(feature_shards(rp, f, F * S, P))
        res[P] = (o.rows()["e"].copy(), o.params()["mu_v"].copy(), o.s.last_free_energy)
    e0, v0, fe0 = res[0]
    e1, v1, fe1 = res[1]
    assert np.max(np.abs(e1 - e0)) <= 1e-12 * np.max(np.abs(e0))
    assert np.max(np.abs(v1 - v0)) <= 1e-12 * np.max(np.abs(v0))
    assert abs(fe1 - fe0) <= 1e-12 * abs(fe0)
    e2, v2, fe2 = res[2]
    assert np.all(np.isfinite(e2)) and np.isfinite(fe2)
    assert np.max(np.abs(v2 - v0)) > 1e-9   # Jacobi across shards: not the sequential sweep


def test_feature_shards_match_level_schedule():
    """tests/shards.py levels == the field index on field-structured data (one level per field)."""
    import synth
    from shards import levels
    rp, f, v, y = synth.generate(2000, 6, 30, 3, 0)
    lv = levels(rp, f, 180)
    present = np.bincount(f, minlength=180) > 0
    np.testing.assert_array_equal(lv[present], (np.arange(180) // 30 + 1)[present])


ONLINE_CASES = ["tiny/online_b3", "tiny/online_b5", "tiny/online_b1", "tiny_dup/online_b3", "tiny_dup/online_b5",
                "tiny_dup/online_b1", "tiny/online_meta", "synth_online", "sa_online"]


def run_online_oracle(case, synth_files, sa_split):
    """OVBFM (-method vb_online) on the oracle. D = largest feature id of train/test + 1: the
    online path sizes the model from find_max_feature (libfm.cpp:167-170, 528-600)."""
    t, a = load_case(case)
    m = t["meta"]
    if case.startswith("synth"):
        tr, te = oc.Data(synth_files["train"]), oc.Data(synth_files["test"])
    elif case.startswith("sa_"):
        tr, te = oc.Data(sa_split["train"]), oc.Data(sa_split["test"])
    else:
        tr, te = _tiny(case.split("/")[0])
    k0, k1, k = [int(x) for x in m["dim"].split(",")]
    D = max(tr.num_feature, te.num_feature)
    assert D == t["nums"]["D"]
    groups = None
    if "meta" in m:
        groups = np.loadtxt(os.path.join(GOLDEN, case.split("/")[0], m["meta"]), dtype=np.uint32)[:D]
    ovb = oc.OVB(k0, k1, k, D, m["batch"], groups)
    ovb.init(m["seed"], m["init_stdev"], tr, te)
    return t, a, ovb, tr, te


@pytest.mark.parametrize("case", ONLINE_CASES)
def test_online_vb_trace_bit_exact(case, synth_files, sa_split):
    """fm_learn_vb_online_simultaneous::_learn: epoch shuffle (std::random_shuffle on rand()),
    mini-batches in file order, natural-gradient steps, hyper-parameters, free energy of the
    first and last batch and the test RMSE -- all equal to the reference's."""
    t, a, ovb, tr, te = run_online_oracle(case, synth_files, sa_split)
    if "init_mu_w" in a:
        p = ovb.params()
        np.testing.assert_array_equal(p["mu_w"], a["init_mu_w"])
        np.testing.assert_array_equal(p["nat_mu_v"], a["init_nat_mu_v"])
    for it, ref in enumerate(t["trace"]):
        rmse, mae, fe1, fe2 = ovb.epoch()
        assert rmse == ref["rmse"], (it, rmse, ref["rmse"])
        fe = [fe1] if t["meta"]["batch"] == 1 else [fe1, fe2]
        assert fe == ref["free_energy"], (it, fe, ref["free_energy"])
    p = ovb.params()
    for key in ("mu_w", "sigma_w", "mu_v", "sigma_v", "hyp_sigma_w", "hyp_sigma_v", "nat_mu_w", "nat_sigma_w",
                "nat_mu_v", "nat_sigma_v", "steps", "scalars", "pred"):
        if "final_" + key in a:
            np.testing.assert_array_equal(p[key], a["final_" + key], err_msg=key)
    for key, (s1, s2) in t["meta"].get("array_sums", {}).items():
        if key.startswith("final_"):
            v = p[key[len("final_"):]]
            assert float(np.sum(v)) == s1 and float(np.sum(v ** 2)) == s2, key
