"""Per-level parity: the sweeps driven one dependency level at a time (vbfm_step_w_level /
vbfm_step_v_level, include/vbfm.h) against the reference's own update_w / update_v called
level by level (oracle/_ref/ref_driver levels -> tests/golden/<case>/levels; SURVEY §8b's
per-level debug entry points, §4 item 1).

After level l the device's caches e, t, q, tq, tz and parameters mu, sigma must equal the
reference's after it has updated every feature of levels 0..l (fm_learn_vb.h:390-406 w sweep,
409-440 factor sweeps, 527-574 update_w, 577-644 update_v). Tolerance 1e-12 relative: each
column's statistics are reduced in a fixed tree order on the device and sequentially in the
reference; the q-cache a factor's sweep starts from is a per-row sum in the reference's order
and stays bit-exact. tests/test_oracle_golden.py checks that the reference's level-by-level
sweep ends bit for bit where its ascending sweep ends.
"""
import os

import numpy as np
import pytest

import synth
import vbfm
from conftest import GOLDEN, load_case

pytestmark = pytest.mark.gpu
TOL = 1e-12


def rel_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    scale = max(1e-300, float(np.max(np.abs(b))) if b.size else 1.0)
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def close(a, b, what):
    assert rel_err(a, b) <= TOL, (what, rel_err(a, b))


def _learner(case, layout):
    d = os.path.join(GOLDEN, case)
    train = vbfm.DataSubset.load(os.path.join(d, "train.libfm"))
    test = vbfm.DataSubset.load(os.path.join(d, "test.libfm"))
    g = vbfm.FMLearnVB(1, 1, 3, vbfm.num_all_attribute(train, test), min_target=train.min_target,
                       max_target=train.max_target, layout=layout)
    g.init(5, 0.1)
    g.set_data(train, test)
    return g


@pytest.mark.parametrize("case,layout,split", [("tiny", "auto", "0"), ("tiny", "column", "0"),
                                               ("tiny", "column", "1"), ("tiny_dup", "auto", "0"),
                                               ("tiny_dup", "auto", "1")])
def test_every_level_vs_reference(case, layout, split, monkeypatch):
    """split "1": the row-shard kernels on one rank in their two-pass form (statistics, then
    posterior + correction: VBFM_FORCE_SPLIT=1, VBFM_DEFER=0)."""
    monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
    monkeypatch.setenv("VBFM_DEFER", "0")
    t, a = load_case(case + "/levels")
    _, s0 = load_case(case + "/steps")
    L = t["meta"]["num_levels"]
    g = _learner(case, layout)
    lv, nl = g.levels()
    assert nl == L
    np.testing.assert_array_equal(lv, a["levels"])
    g.init_caches()
    r = g.rows()
    np.testing.assert_array_equal(r["e"], s0["s0_init_e"])
    np.testing.assert_array_equal(r["t"], s0["s0_init_t"])
    g.step_w0()
    for key in ("e", "t"):
        close(g.rows()[key], a["l_w0_" + key], "w0 " + key)
    for l in range(L):
        g.step_w_level(l)
        tag = "l_w_l%d" % l
        r, p = g.rows(), g.get_params()
        for key in ("e", "t"):
            close(r[key], a[tag + "_" + key], tag + key)
        close(p["mu_w"], a[tag + "_mu_w"], tag + "mu_w")
        close(p["sigma_w"], a[tag + "_sigma_w"], tag + "sigma_w")
    for f in range(3):
        for l in range(L):
            g.step_v_level(f, l)
            tag = "l_f%d_l%d" % (f, l)
            r, p = g.rows(), g.get_params()
            for key in ("e", "t", "q", "tq", "tz"):
                close(r[key], a[tag + "_" + key], tag + key)
            close(p["mu_v"], a[tag + "_mu_v"], tag + "mu_v")
            close(p["sigma_v"], a[tag + "_sigma_v"], tag + "sigma_v")
    g.step_hyper()          # the sweep is complete: the whole-sweep steps run again
    g.close()


def test_q_cache_entering_each_sweep_is_bit_exact():
    """The q-cache factor f's level 0 starts from (fused into the previous sweep or the row
    kernel) is the reference's add_main_q bit for bit (steps fixture s3_f<f>_q)."""
    _, s = load_case("tiny/steps")
    t, _ = load_case("tiny/levels")
    g = _learner("tiny", "auto")
    g.init_caches()
    g.step_w0()
    for l in range(t["meta"]["num_levels"]):
        g.step_w_level(l)
    for f in range(3):
        g.step_qcache(f)
        r = g.rows()
        for key in ("q", "tq", "tz"):
            np.testing.assert_array_equal(r[key], s["s3_f%d_q_%s" % (f, key)])
        for l in range(t["meta"]["num_levels"]):
            g.step_v_level(f, l)
    g.close()


@pytest.mark.parametrize("layout", ["level", "entry"])
def test_level_stores_mid_sweep_equal_column_layout(layout):
    """Half a sweep on a level-ordered store (the field store holds the records in the next
    level's order, the entry store in each row's next slot): read back in row order, every
    cache equals the column layout's after the same level, bit for bit (the i-th entry of a
    column is the same (row, x) in every layout). Field data for the field
    store, multi-hot rows for the entry store."""
    res = {}
    for lay in ("column", layout):
        if layout == "level":
            rp, f, v, y = synth.generate(3000, 5, 40, 21, 1)
            rpt, ft, vt, yt = synth.generate(300, 5, 40, 22, 1)
            nf = 200
        else:
            rp, f, v, y = synth.generate_multihot(3000, 400, 2, 9, 31, 1)
            rpt, ft, vt, yt = synth.generate_multihot(300, 400, 2, 9, 32, 1)
            nf = 400
        train = vbfm.DataSubset.from_csr(rp, f, v, y, nf)
        test = vbfm.DataSubset.from_csr(rpt, ft, vt, yt, nf)
        g = vbfm.FMLearnVB(1, 1, 2, nf + 1, min_target=float(y.min()), max_target=float(y.max()), layout=lay)
        g.init(9, 0.1)
        g.set_data(train, test)
        g.init_caches()
        assert g.layout() == lay
        _, L = g.levels()
        assert L >= 3
        g.step_w0()
        out = []
        for l in range(L):
            g.step_w_level(l)
            out.append(g.rows())
        for fk in range(2):
            for l in range(L):
                g.step_v_level(fk, l)
                out.append(g.rows())
                out.append({"mu_v": g.get_params()["mu_v"]})
        res[lay] = out
        g.close()
    for i, (a, b) in enumerate(zip(res["column"], res[layout])):
        for key in a:
            np.testing.assert_array_equal(a[key], b[key], err_msg="%d %s" % (i, key))


def test_per_level_steps_refuse_misuse(monkeypatch):
    g = _learner("tiny", "auto")
    g.init_caches()
    with pytest.raises(vbfm.VbfmError, match="in order"):
        g.step_v_level(0, 1)                       # not from level 0
    g.step_v_level(0, 0)
    with pytest.raises(vbfm.VbfmError, match="in progress"):
        g.iterate()                                # half a sweep
    with pytest.raises(vbfm.VbfmError, match="in order"):
        g.step_v_level(1, 1)                       # another factor mid-sweep
    g.close()
    # the deferred split (row shards on the field store) keeps each level's correction pending
    monkeypatch.setenv("VBFM_FORCE_SPLIT", "1")
    monkeypatch.delenv("VBFM_DEFER", raising=False)
    rp, f, v, y = synth.generate(2000, 4, 30, 3, 1)
    train = vbfm.DataSubset.from_csr(rp, f, v, y, 120)
    d = vbfm.FMLearnVB(1, 1, 2, 121, min_target=float(y.min()), max_target=float(y.max()), layout="level")
    d.init(9, 0.1)
    d.set_data(train, train)
    d.init_caches()
    with pytest.raises(vbfm.VbfmError, match="deferred"):
        d.step_v_level(0, 0)
    d.close()


def test_failed_level_refuses_every_read_until_restart(monkeypatch):
    """a level that fails mid-sweep may leave the records half moved; every entry point
    that reads or sweeps them -- vbfm_get_rows included -- refuses until vbfm_set_train or
    vbfm_load_state (VBFM_FAULT=level: the step of level 1 fails after its kernel ran)."""
    g = _learner("tiny", "auto")
    g.init_caches()
    g.step_v_level(0, 0)
    monkeypatch.setenv("VBFM_FAULT", "level")
    with pytest.raises(vbfm.VbfmError, match="VBFM_FAULT=level"):
        g.step_v_level(0, 1)
    monkeypatch.delenv("VBFM_FAULT")
    for call in (g.rows, g.iterate, g.step_w0, lambda: g.step_v_level(0, 0)):
        with pytest.raises(vbfm.VbfmError, match="failed"):
            call()
    g.close()
