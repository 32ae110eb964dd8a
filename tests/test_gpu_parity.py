"""Parity of the HIP path (libvbfm.so through its C-ABI) with the oracle and the reference.

Tolerances (north star: 1e-6 relative on free energy and test RMSE at iteration parity):
  * per-row sums (q-cache, predictions, T) keep the reference's summation order: bit-exact;
  * everything downstream of a column / data-set reduction (the device sums in a fixed
    tree order, the reference sequentially) is held to REL = 1e-9 relative -- observed
    differences are ~1e-13; the 1e-6 gate of the north star is far looser.
"""
import os

import numpy as np
import pytest

import oracle_ctypes as oc
import synth
import vbfm
from conftest import GOLDEN, load_case

pytestmark = pytest.mark.gpu
REL = 1e-9


def rel_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    scale = max(1e-300, float(np.max(np.abs(b))) if b.size else 1.0)
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def close(a, b, tol=REL):
    assert rel_err(a, b) <= tol, (rel_err(a, b), a, b)


def gpu_learner(train, test, dim, seed, init_stdev, attr_group=None):
    k0, k1, k = [int(x) for x in dim.split(",")]
    D = vbfm.num_all_attribute(train, test)
    fml = vbfm.FMLearnVB(k0, k1, k, D, attr_group=attr_group, min_target=train.min_target,
                         max_target=train.max_target)
    fml.init(seed, init_stdev)
    fml.set_data(train, test)
    return fml


def oracle_learner(tr_path, te_path, dim, seed, init_stdev, attr_group=None):
    tr, te = oc.Data(tr_path), oc.Data(te_path)
    k0, k1, k = [int(x) for x in dim.split(",")]
    vb = oc.VB(k0, k1, k, oc.num_all_attribute(tr, te), attr_group)
    vb.init_params(seed, init_stdev)
    vb.attach(tr, te)
    return vb


@pytest.mark.parametrize("case,dim", [("tiny", "1,1,3"), ("tiny_dup", "1,1,3"), ("tiny", "1,0,3"),
                                      ("tiny_dup", "0,0,3")])
def test_update_all_steps_vs_oracle(case, dim):
    """update_all step by step. The q-cache of factor f is accumulated inside the previous
    sweep (w sweep for f = 0 when k1, else the row-parallel kernel): bit-exact."""
    d = os.path.join(GOLDEN, case)
    trp, tep = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
    train, test = vbfm.DataSubset.load(trp), vbfm.DataSubset.load(tep)
    g = gpu_learner(train, test, dim, 5, 0.1)
    o = oracle_learner(trp, tep, dim, 5, 0.1)
    po, pg = o.params(), g.get_params()
    for key in ("mu_w", "mu_v", "sigma_v"):
        np.testing.assert_array_equal(pg[key], po[key])
    g.init_caches()
    o.init_caches()
    rg, ro = g.rows(), o.rows()
    np.testing.assert_array_equal(rg["e"], ro["e"])       # per-row sums: bit-exact
    np.testing.assert_array_equal(rg["t"], ro["t"])
    np.testing.assert_array_equal(g.test_e(), oc.arr(o.s.e_test, o.s.n_test))
    g.step_w0()
    if int(dim.split(",")[0]):                    # update_all calls update_w0 only with k0
        o.step("update_w0")
    close(g.rows()["e"], o.rows()["e"]); close(g.rows()["t"], o.rows()["t"])
    g.step_w(); o.step("update_w_all")
    close(g.get_params()["mu_w"], o.params()["mu_w"]); close(g.rows()["e"], o.rows()["e"])
    for f in range(3):
        g.step_qcache(f); o.step("add_main_q", f)
        rg, ro = g.rows(), o.rows()
        for key in ("q", "tq", "tz"):
            np.testing.assert_array_equal(rg[key], ro[key], err_msg="f%d %s" % (f, key))
        g.step_v(f); o.step("update_v_all", f)
        rg, ro = g.rows(), o.rows()
        for key in ("e", "t", "q", "tq", "tz"):
            close(rg[key], ro[key])
        close(g.get_params()["mu_v"], o.params()["mu_v"])
        close(g.get_params()["sigma_v"], o.params()["sigma_v"])
    early = g.step_hyper()
    assert early == bool(o.step("hyper") or o.s.hyper_skipped)
    close(g.get_params()["hyp_sigma_v"], o.params()["hyp_sigma_v"])
    close([g.free_energy()], [oc.lib().or_vb_free_energy(oc.C.byref(o.s), oc.C.byref(o.train.d))])


def run_trace(train, test, meta, attr_group=None):
    fml = gpu_learner(train, test, meta["dim"], meta["seed"], meta["init_stdev"], attr_group)
    fml.init_caches()
    out = [fml.iterate() for _ in range(meta["iter"])]
    return fml, out


def check_trace(stats, trace, tol=REL):
    for it, (st, ref) in enumerate(zip(stats, trace)):
        assert st.free_energy_valid
        close([st.rmse], [ref["rmse"]], tol)
        close([st.mae], [ref["mae"]], tol)
        close([st.train_quirk], [ref["train"]], tol)
        close([st.alpha], [ref["alpha"]], tol)
        close([st.mu_0_dash], [ref["mu_0_dash"]], tol)
        close([st.free_energy], [ref["free_energy"]], tol)


@pytest.mark.parametrize("case", ["tiny/vb", "tiny_dup/vb", "tiny/vb_meta"])
def test_trace_tiny_vs_reference(case):
    t, a = load_case(case)
    d = os.path.join(GOLDEN, case.split("/")[0])
    train = vbfm.DataSubset.load(os.path.join(d, "train.libfm"))
    test = vbfm.DataSubset.load(os.path.join(d, "test.libfm"))
    groups = None
    if "meta" in t["meta"]:
        groups = vbfm.load_meta(os.path.join(d, t["meta"]["meta"]), vbfm.num_all_attribute(train, test))
    fml, stats = run_trace(train, test, t["meta"], groups)
    check_trace(stats, t["trace"])
    p = fml.get_params()
    last = len(stats) - 1
    close(p["mu_v"], a["iter%d_mu_v" % last])
    close(p["sigma_w"], a["iter%d_sigma_w" % last])
    close(fml.predict(), a["iter%d_pred" % last])


@pytest.mark.parametrize("layout", ["column", "level"])
@pytest.mark.parametrize("split", ["fused", "split"])
def test_trace_synthetic_vs_reference(synth_files, split, layout, monkeypatch):
    """split: the row-sharded kernels (stats -> all-reduce -> correct) on one rank;
    layout: row caches gathered in row order, or kept in level order and streamed."""
    if split == "split":
        monkeypatch.setenv("VBFM_FORCE_SPLIT", "1")
    monkeypatch.setenv("VBFM_LAYOUT", layout)
    t, a = load_case("synth")
    train, test = vbfm.DataSubset.load(synth_files["train"]), vbfm.DataSubset.load(synth_files["test"])
    fml, stats = run_trace(train, test, t["meta"])
    assert fml.layout() == layout
    assert stats[0].num_levels == t["meta"]["n_fields"]
    check_trace(stats, t["trace"])
    close(fml.get_params()["mu_v"], a["final_mu_v"])


@pytest.mark.parametrize("layout", ["column", "level"])
@pytest.mark.parametrize("split", ["fused", "split", "rccl", "rccl_chunks"])
def test_trace_movielens_split_vs_reference(sa_split, split, layout, monkeypatch):
    """split: the row-sharded kernels on one rank; rccl: the same through a real 1-rank RCCL
    communicator (every ncclAllReduce of the multi-GPU path runs); rccl_chunks: each level's
    statistics in 3 chunks whose all-reduces run on the communication stream while the next
    chunk computes (stats_exchange). Every ML-1M row is one (user, item) pair, so both
    dependency levels hold every row: the level layout applies."""
    if split != "fused":
        monkeypatch.setenv("VBFM_FORCE_SPLIT", "1")
    if split == "rccl_chunks":
        monkeypatch.setenv("VBFM_AR_CHUNKS", "3")
    monkeypatch.setenv("VBFM_LAYOUT", layout)
    t, a = load_case("sa_k8")
    train, test = vbfm.DataSubset.load(sa_split["train"]), vbfm.DataSubset.load(sa_split["test"])
    if split.startswith("rccl"):
        monkeypatch.setenv("VBFM_FORCE_COMM", "1")
        m = t["meta"]
        k0, k1, k = [int(x) for x in m["dim"].split(",")]
        fml = vbfm.FMLearnVB(k0, k1, k, vbfm.num_all_attribute(train, test), min_target=train.min_target,
                             max_target=train.max_target)
        fml.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
        fml.init(m["seed"], m["init_stdev"])
        fml.set_data(train, test)
        fml.init_caches()
        stats = [fml.iterate() for _ in range(m["iter"])]
    else:
        fml, stats = run_trace(train, test, t["meta"])
    assert fml.layout() == layout
    check_trace(stats, t["trace"])
    close(fml.get_params()["mu_w"], a["final_mu_w"])


@pytest.mark.parametrize("model_seed,row_offset", [(synth.MODEL_SEED, 0), (12345, 0), (synth.MODEL_SEED, 777_777)])
def test_device_generator_matches_spec(model_seed, row_offset):
    """vbfm_synth_generate (device) == tests/synth.py (numpy), CSC and targets bit-exact,
    with the default and another planted model, and as a row shard of a larger data set."""
    n, F, S, seed = 5000, 7, 300, 99
    fml = vbfm.FMLearnVB(1, 1, 2, F * S + 1)
    fml.synth(0, n, F, S, seed, xmode=1, model_seed=model_seed, row_offset=row_offset)
    cp, ent, tg = fml.get_csc(0)
    rp, f, v, y = synth.generate(n, F, S, seed, 1, model_seed=model_seed, row_offset=row_offset)
    ecp, erow, eval_ = synth.csr_to_csc(n, F * S, rp, f, v)
    np.testing.assert_array_equal(cp, ecp)
    np.testing.assert_array_equal(ent["id"], erow)
    np.testing.assert_array_equal(ent["value"], eval_)
    np.testing.assert_array_equal(tg, y)
    lv, L = fml.levels()
    assert L == F
    present = np.bincount(f, minlength=F * S) > 0
    np.testing.assert_array_equal(lv[present], (np.arange(F * S) // S + 1)[present])


@pytest.mark.parametrize("predict,layout", [("exact", "column"), ("blocked", "column"), ("wave", "column"),
                                            ("exact", "level"), ("blocked", "level"), ("wave", "level")])
def test_generated_data_vs_oracle_two_iterations(predict, layout, monkeypatch):
    """Device-generated field data (real-valued x) through 2 iterations vs the oracle, with
    every form of the prediction kernels (blocked, wave: ~1 ulp from the reference's order)
    and both row layouts."""
    monkeypatch.setenv("VBFM_PREDICT", predict)
    monkeypatch.setenv("VBFM_LAYOUT", layout)
    n, F, S, seed, k = 60000, 8, 500, 3, 11
    D = F * S + 1
    rp, f, v, y = synth.generate(n, F, S, seed, 1)
    rpt, ft, vt, yt = synth.generate(2000, F, S, seed + 1, 1)
    fml = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()))
    fml.init(7, 0.1)
    fml.synth(0, n, F, S, seed, 1)
    fml.synth(1, 2000, F, S, seed + 1, 1)
    fml.init_caches()
    tr = oc.Data(csr=(n, rp, f, v, y))
    te = oc.Data(csr=(2000, rpt, ft, vt, yt))
    o = oc.VB(1, 1, k, D)
    o.init_params(7, 0.1)
    o.attach(tr, te)
    o.init_caches()
    assert fml.layout() == layout
    rg, ro = fml.rows(), o.rows()
    if predict == "exact":
        np.testing.assert_array_equal(rg["e"], ro["e"])
        np.testing.assert_array_equal(rg["t"], ro["t"])
    else:
        close(rg["e"], ro["e"], 1e-13)
        close(rg["t"], ro["t"], 1e-13)
    for _ in range(2):
        st = fml.iterate()
        rmse, mae, trq = o.iterate()
        close([st.rmse], [rmse]); close([st.train_quirk], [trq])
        close([st.free_energy], [o.s.last_free_energy])
    close(fml.get_params()["mu_v"], o.params()["mu_v"])


def test_deterministic_run_to_run():
    def run():
        fml = vbfm.FMLearnVB(1, 1, 4, 10 * 1000 + 1, min_target=1, max_target=5)
        fml.init(3, 0.1)
        fml.synth(0, 100000, 10, 1000, 5, 1)
        fml.synth(1, 5000, 10, 1000, 6, 1)
        fml.init_caches()
        st = [fml.iterate() for _ in range(2)]
        return [s.free_energy for s in st], fml.get_params()["mu_v"]
    a, b = run(), run()
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])


def _synth_learner(n, F, S, k, seed, layout, dim=(1, 1)):
    rp, f, v, y = synth.generate(n, F, S, seed, 1)
    rpt, ft, vt, yt = synth.generate(500, F, S, seed + 1, 1)
    D = F * S + 1
    g = vbfm.FMLearnVB(dim[0], dim[1], k, D, min_target=float(y.min()), max_target=float(y.max()), layout=layout)
    g.init(5, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
    o = oc.VB(dim[0], dim[1], k, D)
    o.init_params(5, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(500, rpt, ft, vt, yt)))
    return g, o


@pytest.mark.parametrize("dim", [(1, 1), (1, 0), (0, 0)])
def test_update_all_steps_level_layout(dim):
    """update_all step by step with the level-ordered row store (every step reads the rows
    back in row order): q-caches bit-exact, everything else within REL of the oracle.
    dim (k0, k1) = (1, 0) / (0, 0): the q-cache of factor 0 comes from the row-parallel
    kernel writing through the level-0 position map."""
    g, o = _synth_learner(3000, 5, 40, 3, 21, "level", dim)
    assert g.layout() == "level"
    g.init_caches(); o.init_caches()
    rg, ro = g.rows(), o.rows()
    np.testing.assert_array_equal(rg["e"], ro["e"])
    np.testing.assert_array_equal(rg["t"], ro["t"])
    g.step_w0()
    if dim[0]:
        o.step("update_w0")
    close(g.rows()["e"], o.rows()["e"])
    g.step_w(); o.step("update_w_all")
    close(g.get_params()["mu_w"], o.params()["mu_w"]); close(g.rows()["e"], o.rows()["e"])
    for f in range(3):
        g.step_qcache(f); o.step("add_main_q", f)
        rg, ro = g.rows(), o.rows()
        for key in ("q", "tq", "tz"):
            np.testing.assert_array_equal(rg[key], ro[key], err_msg="f%d %s" % (f, key))
        g.step_v(f); o.step("update_v_all", f)
        rg, ro = g.rows(), o.rows()
        for key in ("e", "t", "q", "tq", "tz"):
            close(rg[key], ro[key])
        close(g.get_params()["mu_v"], o.params()["mu_v"])
        close(g.get_params()["sigma_v"], o.params()["sigma_v"])
    g.step_hyper(); o.step("hyper")
    close(g.get_params()["hyp_sigma_v"], o.params()["hyp_sigma_v"])


def test_layouts_agree():
    """Column-gather and level-ordered layouts compute bit-identical column statistics;
    only the data-set sums (w0, alpha, free energy) are summed in another row order."""
    res = {}
    for layout in ("column", "level"):
        g, _ = _synth_learner(40000, 6, 300, 4, 8, layout)
        assert g.layout() == layout
        g.init_caches()
        st = [g.iterate() for _ in range(3)]
        res[layout] = ([s.free_energy for s in st], [s.rmse for s in st], g.get_params()["mu_v"], g.rows()["e"])
    close(res["level"][0], res["column"][0], 1e-12)
    close(res["level"][1], res["column"][1], 1e-12)
    close(res["level"][2], res["column"][2], 1e-12)
    close(res["level"][3], res["column"][3], 1e-12)


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("method", ["vb", "als"])
def test_unit_x_store_bit_identical(method, split, monkeypatch):
    """One-hot data (every x 1.0f, libfm's categorical case and the bench shape): the level
    store keeps no x per entry and the deferred split an 8-B payload {next, previous}.
    VBFM_LX=1 keeps the x array / 16-B payload: the results are bit for bit the same (x = 1
    enters every product exactly), fused and split. VB also against the oracle."""
    monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
    n, F, S, k = 20000, 6, 200, 4
    rp, f, v, y = synth.generate(n, F, S, 13, 0)
    rpt, ft, vt, yt = synth.generate(500, F, S, 14, 0)
    assert np.all(v == 1.0)
    D = F * S + 1
    res = {}
    for lx in ("0", "1"):
        monkeypatch.setenv("VBFM_LX", lx)
        if method == "vb":
            g = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()), layout="level")
            g.init(5, 0.1)
        else:
            g = vbfm.FMLearnMCMC(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()), method="als",
                                 layout="level")
            g.init_device(5, 0.1)
        g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
        g.init_caches()
        st = [g.iterate() for _ in range(3)]
        assert g.layout() == "level"
        p = g.get_params()
        res[lx] = ([s.rmse if method == "vb" else s.rmse_all for s in st],
                   np.asarray(p["mu_v"] if method == "vb" else p["v"]), g.rows()["e"])
        g.close()
    for a, b in zip(res["0"], res["1"]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    if method == "vb":
        o = oc.VB(1, 1, k, D)
        o.init_params(5, 0.1)
        o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(500, rpt, ft, vt, yt)))
        o.init_caches()
        for it in range(3):
            ro, _, _ = o.iterate()
            assert abs(res["0"][0][it] - ro) <= REL * ro


@pytest.mark.parametrize("k1", [1, 0])
def test_long_columns_split_into_segments(k1, monkeypatch):
    """Skewed two-field data (a Zipf item field: the top items hold 10k-20k rows): columns
    longer than max(1024, 4 x the level's mean) entries are swept by segment workgroups of 1024
    entries (statistics partials, then the posterior + move / correction) on both layouts. Against the oracle (1e-9) and against one
    workgroup per column (VBFM_LONG=0) on either layout (summation order only, 1e-12)."""
    n, U, I, k = 60000, 5000, 400, 4
    rng = np.random.default_rng(11)
    u = rng.integers(0, U, n).astype(np.uint32)
    it = ((rng.zipf(1.4, n) - 1) % I).astype(np.uint32)
    assert np.bincount(it).max() > 2 * 8192
    f = np.empty(2 * n, np.uint32); f[0::2] = u; f[1::2] = U + it
    v = (0.5 + rng.random(2 * n)).astype(np.float32)
    y = rng.integers(1, 6, n).astype(np.float32)
    rp = np.arange(0, 2 * n + 1, 2, dtype=np.uint64)
    nt = 2000
    D = U + I + 1
    res = {}
    for name, env in (("seg", {}), ("noseg", {"VBFM_LONG": "0"}), ("column", {"VBFM_LAYOUT": "column"}),
                      ("column_noseg", {"VBFM_LAYOUT": "column", "VBFM_LONG": "0"})):
        for kk in ("VBFM_LONG", "VBFM_LAYOUT"):
            monkeypatch.delenv(kk, raising=False)
        for kk, vv in env.items():
            monkeypatch.setenv(kk, vv)
        g = vbfm.FMLearnVB(1, k1, k, D, min_target=1.0, max_target=5.0)
        g.init(5, 0.1)
        g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, U + I),
                   vbfm.DataSubset.from_csr(rp[:nt + 1], f[:2 * nt], v[:2 * nt], y[:nt], U + I))
        g.init_caches()
        st = [g.iterate() for _ in range(2)]
        res[name] = ([s.rmse for s in st], [s.free_energy for s in st], g.get_params()["mu_v"], g.layout())
        g.close()
    assert res["seg"][3] == "level" and res["column"][3] == "column"
    for other in ("noseg", "column", "column_noseg"):
        close(res["seg"][0], res[other][0], 1e-12)
        close(res["seg"][1], res[other][1], 1e-12)
        close(res["seg"][2], res[other][2], 1e-12)
    o = oc.VB(1, k1, k, D)
    o.init_params(5, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(nt, rp[:nt + 1], f[:2 * nt], v[:2 * nt], y[:nt])))
    o.init_caches()
    for it_ in range(2):
        ro, _, _ = o.iterate()
        assert abs(res["seg"][0][it_] - ro) <= REL * ro
    close(res["seg"][2], o.params()["mu_v"])


def _skewed_two_fields(n, U, I, seed, onehot):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, U, n).astype(np.uint32)
    it = ((rng.zipf(1.4, n) - 1) % I).astype(np.uint32)
    f = np.empty(2 * n, np.uint32); f[0::2] = u; f[1::2] = U + it
    v = np.ones(2 * n, np.float32) if onehot else (0.5 + rng.random(2 * n)).astype(np.float32)
    y = rng.integers(1, 6, n).astype(np.float32)
    return np.arange(0, 2 * n + 1, 2, dtype=np.uint64), f, v, y, it


COUNTERS = ("nan_mu_w", "nan_sigma_w", "inf_mu_w", "nan_mu_v", "nan_sigma_v", "inf_mu_v", "nan_alpha")


@pytest.mark.parametrize("case", ["onehot", "dup", "nan"])
def test_long_column_segments_edge_cases(case, monkeypatch):
    """The long-column segment kernels (k_lord_long_* / k_col_long_*) on the inputs the
    parametrised skew test does not cover, each against the oracle and against one
    workgroup per column (VBFM_LONG=0) on every layout that applies:
      * onehot: every x is 1.0f, so the level store keeps no x array (lx elided);
      * dup: rows of the popular items list the item twice (a libfm line with a repeated
        feature): the column layout keeps those columns on the sequential path;
      * nan: one row of the most popular item has a NaN target (the reference parses "nan"),
        so that column's (and the row's user column's) posterior is NaN in every sweep: the
        guard (fm_learn_vb.h:597-619) restores mu and skips the correction, the counters
        count it once per column, alpha turns NaN and the hyper step returns early."""
    n, U, I, k = 60000, 5000, 400, 3
    rp, f, v, y, it = _skewed_two_fields(n, U, I, 17, case == "onehot")
    top = int(np.argmax(np.bincount(it)))
    assert np.bincount(it).max() > 2 * 8192
    k0 = 1
    if case == "dup":
        # every 3rd row of the top item lists it twice: rows of 2 or 3 entries
        rows = [list(f[2 * r:2 * r + 2]) for r in range(n)]
        vals = [list(v[2 * r:2 * r + 2]) for r in range(n)]
        for r in np.flatnonzero(it == top)[::3]:
            rows[r].append(rows[r][1]); vals[r].append(np.float32(0.75))
        f = np.concatenate([np.asarray(x, np.uint32) for x in rows])
        v = np.concatenate([np.asarray(x, np.float32) for x in vals])
        rp = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.uint64)
    if case == "nan":
        y = y.copy()
        y[np.flatnonzero(it == top)[7]] = np.nan
        k0 = 0   # update_w0 has no guard: a NaN row would reach every row through mu_0
    nt = 2000
    rt, ftu, vtt, yt, _ = _skewed_two_fields(nt, U, I, 18, case == "onehot")
    D = U + I + 1
    variants = [("column_seg", {"VBFM_LAYOUT": "column"}), ("column_noseg", {"VBFM_LAYOUT": "column", "VBFM_LONG": "0"})]
    if case != "dup":
        variants += [("level_seg", {"VBFM_LAYOUT": "level"}), ("level_noseg", {"VBFM_LAYOUT": "level", "VBFM_LONG": "0"})]
    res = {}
    for name, env in variants:
        for kk in ("VBFM_LONG", "VBFM_LAYOUT"):
            monkeypatch.delenv(kk, raising=False)
        for kk, vv in env.items():
            monkeypatch.setenv(kk, vv)
        g = vbfm.FMLearnVB(k0, 1, k, D, min_target=1.0, max_target=5.0)
        g.init(5, 0.1)
        g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, U + I), vbfm.DataSubset.from_csr(rt, ftu, vtt, yt, U + I))
        g.init_caches()
        st = [g.iterate() for _ in range(2)]
        res[name] = dict(rmse=[s.rmse for s in st], mae=[s.mae for s in st], quirk=[s.train_quirk for s in st],
                         fe_valid=[s.free_energy_valid for s in st],
                         fe=[s.free_energy for s in st if s.free_energy_valid],
                         cnt=[[getattr(s, c) for c in COUNTERS] for s in st],
                         mu_v=g.get_params()["mu_v"], layout=g.layout())
        g.close()
    for name, env in variants:
        assert res[name]["layout"] == env["VBFM_LAYOUT"]
    o = oc.VB(k0, 1, k, D)
    o.init_params(5, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(nt, rt, ftu, vtt, yt)))
    o.init_caches()
    for i in range(2):
        ro, mo, qo = o.iterate()
        cnt = [getattr(o.s, c) for c in COUNTERS]
        for name, _ in variants:
            r = res[name]
            assert abs(r["rmse"][i] - ro) <= REL * ro, (name, i)
            assert abs(r["mae"][i] - mo) <= REL * mo, (name, i)
            assert abs(r["quirk"][i] - qo) <= REL * qo, (name, i)
            assert r["cnt"][i] == cnt, (name, i, r["cnt"][i], cnt)
            assert r["fe_valid"][i] == (0 if o.s.hyper_skipped else 1), (name, i)
            if not o.s.hyper_skipped:
                close(r["fe"][i], o.s.last_free_energy)
    if case == "nan":
        assert o.s.hyper_skipped and o.s.nan_mu_v >= 2 * k and o.s.nan_alpha == 1
    else:
        assert not o.s.hyper_skipped and o.s.nan_mu_v == 0
    for name, _ in variants:
        close(res[name]["mu_v"], o.params()["mu_v"])
        close(res[name]["mu_v"], res[variants[0][0]]["mu_v"], 1e-12)
        close(res[name]["fe"], res[variants[0][0]]["fe"], 1e-12)


def test_level_layout_refused_when_levels_incomplete():
    """tiny has rows of different lengths: a level misses rows, the level layout cannot
    apply -- auto takes the entry store, an explicit level request fails loudly."""
    d = os.path.join(GOLDEN, "tiny")
    train = vbfm.DataSubset.load(os.path.join(d, "train.libfm"))
    test = vbfm.DataSubset.load(os.path.join(d, "test.libfm"))
    g = gpu_learner(train, test, "1,1,3", 5, 0.1)
    g.init_caches()
    assert g.layout() == "entry"
    D = vbfm.num_all_attribute(train, test)
    g2 = vbfm.FMLearnVB(1, 1, 3, D, min_target=train.min_target, max_target=train.max_target, layout="level")
    g2.init(5, 0.1)
    g2.set_data(train, test)
    with pytest.raises(vbfm.VbfmError, match="level-ordered row layout not possible"):
        g2.init_caches()


@pytest.mark.parametrize("k", [70, 130])
def test_wave_prediction_many_factors(k, monkeypatch):
    """The wave-per-row prediction with two and three factor passes per lane (k > 64),
    against the oracle's initial caches (e and T of every row)."""
    monkeypatch.setenv("VBFM_PREDICT", "wave")
    g, o = _synth_learner(4000, 6, 100, k, 31, "auto")
    g.init_caches(); o.init_caches()
    rg, ro = g.rows(), o.rows()
    close(rg["e"], ro["e"], 1e-12)
    close(rg["t"], ro["t"], 1e-12)
    np.testing.assert_allclose(g.test_e(), oc.arr(o.s.e_test, o.s.n_test), rtol=1e-12, atol=1e-12)


def test_million_rows_two_iterations_vs_oracle():
    """Parity at scale: 1e6 rows x 40 one-hot fields of 25,000 ids (C3's field shape, real-valued
    x), k = 4, on the level-ordered store with the wave-form predictions, two full iterations
    against the oracle (the reference restated, bit-exact on every fixture): test RMSE, MAE,
    free energy, alpha and the final parameters within REL."""
    n, F, S, k, seed = 1_000_000, 40, 25_000, 4, 5
    n_test = 20_000
    D = F * S + 1
    rp, f, v, y = synth.generate(n, F, S, seed, 1)
    rpt, ft, vt, yt = synth.generate(n_test, F, S, seed + 1, 1)
    fml = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()))
    fml.init(3, 0.1)
    fml.synth(0, n, F, S, seed, 1)
    fml.synth(1, n_test, F, S, seed + 1, 1)
    fml.init_caches()
    assert fml.layout() == "level"
    o = oc.VB(1, 1, k, D)
    o.init_params(3, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(n_test, rpt, ft, vt, yt)))
    o.init_caches()
    for it in range(2):
        st = fml.iterate()
        rmse, mae, quirk = o.iterate()
        assert st.num_levels == F
        close(st.rmse, rmse)
        close(st.mae, mae)
        close(st.train_quirk, quirk)
        close(st.free_energy, o.s.last_free_energy)
        close(st.alpha, o.s.alpha)
    p, op = fml.get_params(), o.params()
    for key in ("mu_w", "sigma_w", "mu_v", "sigma_v"):
        close(p[key], op[key])


@pytest.mark.parametrize("k,dim", [(8, (1, 1)), (70, (1, 1)), (130, (0, 1)), (20, (1, 0))])
def test_fused_train_prediction_equals_test_prediction(k, dim, monkeypatch):
    """init_caches predicts e and T of the train rows in one pass (k_predict_et_wave); the
    test set goes through predict_e alone. With the test set = the train set, the fused
    kernel's y - yhat must equal y - (the separate kernel's yhat) bit for bit."""
    monkeypatch.setenv("VBFM_PREDICT", "wave")
    n, F, S, seed = 3000, 6, 80, 41
    rp, f, v, y = synth.generate(n, F, S, seed, 1)
    D = F * S + 1
    g = vbfm.FMLearnVB(dim[0], dim[1], k, D, min_target=float(y.min()), max_target=float(y.max()))
    g.init(9, 0.1)
    ds = vbfm.DataSubset.from_csr(rp, f, v, y, F * S)
    g.set_data(ds, vbfm.DataSubset.from_csr(rp, f, v, y, F * S))
    g.init_caches()
    yhat = g.test_e()
    rows = g.rows()
    np.testing.assert_array_equal(rows["e"], y.astype(np.float64) - yhat)
    o = oc.VB(dim[0], dim[1], k, D)
    o.init_params(9, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(n, rp, f, v, y)))
    o.init_caches()
    close(rows["t"], o.rows()["t"], 1e-12)


@pytest.mark.parametrize("P", [1, 2, 3])
def test_feature_shards_vs_oracle(P):
    """VBFM_SHARD_FEATURES (the north star's column partition) with P shards run one after
    another in this process -- the kernels, the shard chunks of every level, the zeroed
    q-cache partials and the merge of the multi-rank mode, without the all-reduce -- against
    the oracle's restatement of the same Jacobi-across-shards sweep, 2 iterations."""
    from shards import feature_shards
    n, F, S, k = 8000, 5, 60, 3
    rp, f, v, y = synth.generate(n, F, S, 41, 1)
    rpt, ft, vt, yt = synth.generate(500, F, S, 42, 1)
    D = F * S + 1
    g = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()))
    g.set_shard_mode("features", P)
    g.init(5, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
    assert g.layout() == "column"
    o = oc.VB(1, 1, k, D)
    o.init_params(5, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(500, rpt, ft, vt, yt)))
    shard = feature_shards(rp, f, F * S, P)
    g.init_caches(); o.init_caches()
    for _ in range(2):
        st = g.iterate()
        o.update_all_fsharded(shard)
        close([st.free_energy], [o.s.last_free_energy])
        close([st.alpha], [o.s.alpha])
    close(g.rows()["e"], o.rows()["e"])
    close(g.get_params()["mu_v"], o.params()["mu_v"])
    close(g.get_params()["mu_w"], o.params()["mu_w"])


def test_full_size_layouts_and_split_agree():
    """Size-independent properties at C3 shape (1e7 rows x 40 one-hot fields, 1e6 features;
    k = 4 to keep it short): the level-ordered and the column-gather layouts, fused and split
    (multi-rank: deferred one-pass, and the two-pass form) kernels, agree to summation order
    over two iterations; the deferred split equals the fused kernel bit for bit."""
    n, F, S, k = 10_000_000, 40, 25_000, 4
    res = {}
    for layout, split in (("level", "0"), ("column", "0"), ("level", "1"), ("level", "nodefer")):
        os.environ["VBFM_FORCE_SPLIT"] = "0" if split == "0" else "1"
        if split == "nodefer":
            os.environ["VBFM_DEFER"] = "0"
        try:
            g = vbfm.FMLearnVB(1, 1, k, F * S + 1, min_target=1.0, max_target=5.0, layout=layout)
            g.init_device(42)
            g.synth(0, n, F, S, 1000, 0)
            g.synth(1, 100_000, F, S, 500000, 0)
            g.init_caches()
            assert g.layout() == layout
            st = [g.iterate() for _ in range(2)]
            res[(layout, split)] = ([s.free_energy for s in st], [s.rmse for s in st], g.get_params()["mu_v"])
            g.close()
        finally:
            os.environ.pop("VBFM_FORCE_SPLIT", None)
            os.environ.pop("VBFM_DEFER", None)
    base = res[("level", "0")]
    # the deferred split applies the same per-row arithmetic in the same order: bit-identical
    assert res[("level", "1")][0] == base[0] and res[("level", "1")][1] == base[1]
    np.testing.assert_array_equal(res[("level", "1")][2], base[2])
    for key, r in res.items():
        close(r[0], base[0], 1e-11)
        close(r[1], base[1], 1e-11)
        close(r[2], base[2], 1e-11)


@pytest.mark.parametrize("case", ["tiny", "tiny_dup"])
def test_schedule_check_and_markers(case, monkeypatch):
    """VBFM_CHECK=1 verifies on the device that no level lets two columns touch one row (a
    repeated row inside one column is allowed: it is corrected sequentially); VBFM_ROCTX=2
    wraps phases and level launches in roctx ranges. Neither changes the results."""
    monkeypatch.setenv("VBFM_CHECK", "1")
    monkeypatch.setenv("VBFM_ROCTX", "2")
    d = os.path.join(GOLDEN, case)
    train = vbfm.DataSubset.load(os.path.join(d, "train.libfm"))
    test = vbfm.DataSubset.load(os.path.join(d, "test.libfm"))
    g = gpu_learner(train, test, "1,1,3", 5, 0.1)
    g.init_caches()
    a = [g.iterate().rmse for _ in range(2)]
    monkeypatch.delenv("VBFM_CHECK")
    g2 = gpu_learner(train, test, "1,1,3", 5, 0.1)
    g2.init_caches()
    assert a == [g2.iterate().rmse for _ in range(2)]


# seed 376 draws a zero u at output 820,432 of its stream (Leva redraws it: every later attempt
# shifts by one); found by a host scan of seeds 1..1300 (tools/find_zero_seed.cpp)
@pytest.mark.parametrize("seed,init_stdev", [(1, 0.1), (376, 0.1), (376, 0.0), (823, 0.05)])
def test_init_replay_equals_host_draws(seed, init_stdev):
    """vbfm_init_params_replay (the glibc stream by jump-ahead chunks on the device, Leva's
    rejection as a compaction) == vbfm_init_params_host, bit for bit, model draws included."""
    k, D = 8, 1_000_001 if seed == 823 else 100_001
    a = vbfm.FMLearnVB(1, 1, k, D)
    a.init(seed, init_stdev, keep_model_draws=True)
    b = vbfm.FMLearnVB(1, 1, k, D)
    b.init_replay(seed, init_stdev, keep_model_draws=True)
    pa, pb = a.get_params(), b.get_params()
    for key in ("mu_w", "sigma_w", "mu_v", "sigma_v", "hyp_sigma_w", "hyp_sigma_v"):
        np.testing.assert_array_equal(pa[key], pb[key], err_msg=key)
    for key in ("alpha", "sigma_0", "mu_0_dash", "sigma_0_dash"):
        assert pa[key] == pb[key]
    np.testing.assert_array_equal(a.fm_v, b.fm_v)
    np.testing.assert_array_equal(a.fm_w, b.fm_w)


def test_test_prediction_overlap_is_bit_identical(monkeypatch):
    """The per-iteration test prediction runs on its own stream under the hyper-parameter
    step (fm_learn_vb_simultaneous.h:125 after update_all): the same kernel on the same
    parameters, so RMSE / MAE / predictions equal the serial order (VBFM_TEST_OVERLAP=0) bit
    for bit, on both prediction forms."""
    n, F, S, k = 60_000, 12, 500, 6
    runs = {}
    for overlap in ("1", "0"):
        for predict in ("exact", "wave"):
            monkeypatch.setenv("VBFM_TEST_OVERLAP", overlap)
            monkeypatch.setenv("VBFM_PREDICT", predict)
            g = vbfm.FMLearnVB(1, 1, k, F * S + 1, min_target=1.0, max_target=5.0)
            g.init(4, 0.1)
            g.synth(0, n, F, S, 1000, 1)
            g.synth(1, 5000, F, S, 500000, 1)
            g.init_caches()
            st = [g.iterate() for _ in range(3)]
            assert all(s.ms_test_predict > 0 for s in st)
            runs[(overlap, predict)] = ([(s.rmse, s.mae, s.free_energy) for s in st], g.test_e())
            g.close()
    for predict in ("exact", "wave"):
        a, b = runs[("1", predict)], runs[("0", predict)]
        assert a[0] == b[0]
        np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("method", ["vb", "mcmc", "als"])
@pytest.mark.parametrize("layout", ["level", "column"])
def test_chunked_exchange_is_bit_identical(method, layout, monkeypatch):
    """The per-level exchange cut into chunks (VBFM_AR_CHUNKS=4 through a 1-rank RCCL
    communicator: chunk i's all-reduce on the communication stream while chunk i+1's
    statistics kernel runs) against the fused single-rank sweep: the same chain bit for bit
    (every chunk sums exactly its columns' entries; VB and ALS / MCMC with device RNG streams)."""
    rp, f, v, y = synth.generate(60000, 8, 1500, 17, 1)
    rpt, ft, vt, yt = synth.generate(3000, 8, 1500, 18, 1)
    nf = 8 * 1500

    def run(split, chunks):
        monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
        monkeypatch.setenv("VBFM_FORCE_COMM", split)
        if chunks:
            monkeypatch.setenv("VBFM_AR_CHUNKS", str(chunks))
        else:
            monkeypatch.delenv("VBFM_AR_CHUNKS", raising=False)
        if method == "vb":
            g = vbfm.FMLearnVB(1, 1, 3, nf + 1, min_target=float(y.min()), max_target=float(y.max()), layout=layout)
        else:
            g = vbfm.FMLearnMCMC(1, 1, 3, nf + 1, min_target=float(y.min()), max_target=float(y.max()),
                                 method=method, layout=layout)
        if split == "1":
            g.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
        if method == "vb":
            g.init(3, 0.1)
        else:
            g.init_device(3, 0.1)
        g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, nf), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, nf))
        g.init_caches()
        st = [g.iterate() for _ in range(2)]
        p = g.get_params()
        g.close()
        key = "mu_v" if method == "vb" else "v"
        return [s.rmse if method == "vb" else s.rmse_all for s in st], np.asarray(p[key])

    fused = run("0", 0)
    chunked = run("1", 4)
    assert chunked[0] == fused[0]
    np.testing.assert_array_equal(chunked[1], fused[1])


def test_shape_128x3_forms_agree(monkeypatch):
    """Field data of ~300-entry columns takes the 128 x 3 workgroup shape (dispatch_shape,
    csrc/vbfm_device.h) in every kernel family. On the level store the fused kernel, the deferred
    split and the two-pass split agree bit for bit; on the column layout the split's statistics
    kernel takes the fused kernel's BLOCK, so split == fused bit for bit there too; the two
    layouts agree within the data-set sums' row order (1e-12)."""
    n, F, S, k = 30000, 6, 100, 4
    rp, f, v, y = synth.generate(n, F, S, 23, 1)
    rpt, ft, vt, yt = synth.generate(1000, F, S, 24, 1)
    D = F * S + 1
    res = {}
    for layout, split, defer in (("level", "0", "1"), ("level", "1", "1"), ("level", "1", "0"),
                                 ("column", "0", "1"), ("column", "1", "1")):
        monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
        monkeypatch.setenv("VBFM_DEFER", defer)
        g = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()), layout=layout)
        g.init(5, 0.1)
        g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
        g.init_caches()
        assert g.layout() == layout
        st = [g.iterate() for _ in range(3)]
        res[layout, split, defer] = ([(s.rmse, s.free_energy) for s in st], np.asarray(g.get_params()["mu_v"]))
        g.close()
    base = res["level", "0", "1"]
    for key in (("level", "1", "1"), ("level", "1", "0")):
        assert res[key][0] == base[0], key
        np.testing.assert_array_equal(res[key][1], base[1], err_msg=str(key))
    col = res["column", "0", "1"]
    assert res["column", "1", "1"][0] == col[0]
    np.testing.assert_array_equal(res["column", "1", "1"][1], col[1])
    close([x for t in col[0] for x in t], [x for t in base[0] for x in t], 1e-12)
    close(col[1], base[1], 1e-12)
