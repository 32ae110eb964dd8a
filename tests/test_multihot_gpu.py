"""Data without field structure (SURVEY §7 hard part (a)): multi-hot rows of
lo..hi distinct ids (tests/synth.py generate_multihot, device vbfm_synth_multihot). The
dependency levels of such data miss rows and run long (the reference's feature order chains
features through shared rows), so the sweeps take the column-gather layout with many small
level launches. Checked: the device generator against the numpy specification (CSC and targets
bit-exact), and two VB iterations against the oracle (1e-9)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import synth
import vbfm

pytestmark = pytest.mark.gpu

REL = 1e-9


def rel_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b))) / max(float(np.max(np.abs(b))), 1e-300)


@pytest.mark.parametrize("row_offset", [0, 123_457])
def test_device_multihot_generator_matches_spec(row_offset):
    n, D, lo, hi, seed = 6000, 3000, 5, 60, 17
    g = vbfm.FMLearnVB(1, 1, 2, D + 1)
    g.synth_multihot(0, n, D, lo, hi, seed, xmode=1, row_offset=row_offset)
    cp, ent, tg = g.get_csc(0)
    rp, f, v, y = synth.generate_multihot(n, D, lo, hi, seed, 1, row_offset=row_offset)
    ecp, erow, eval_ = synth.csr_to_csc(n, D, rp, f, v)
    np.testing.assert_array_equal(cp, ecp)
    np.testing.assert_array_equal(ent["id"], erow)
    np.testing.assert_array_equal(ent["value"], eval_)
    np.testing.assert_array_equal(tg, y)


@pytest.mark.parametrize("layout", ["auto", "column"])
@pytest.mark.parametrize("k", [1, 6])
def test_multihot_two_iterations_vs_oracle(k, layout):
    """layout auto = the entry store (the levels miss rows: one slot per entry, records moved
    to their rows' next slots), column = the column-gather layout."""
    n, D, lo, hi = 30_000, 4000, 5, 60
    g = vbfm.FMLearnVB(1, 1, k, D + 1, min_target=1.0, max_target=5.0, layout=layout)
    g.init(7, 0.1)
    g.synth_multihot(0, n, D, lo, hi, 1000, 1)
    g.synth_multihot(1, 3000, D, lo, hi, 500000, 1)
    g.init_caches()
    assert g.layout() == ("entry" if layout == "auto" else "column")
    tr = synth.generate_multihot(n, D, lo, hi, 1000, 1)
    te = synth.generate_multihot(3000, D, lo, hi, 500000, 1)
    o = oc.VB(1, 1, k, D + 1)
    o.init_params(7, 0.1)
    o.attach(oc.Data(csr=(n,) + tr), oc.Data(csr=(3000,) + te))
    o.init_caches()
    for _ in range(2):
        st = g.iterate()
        rmse, mae, _ = o.iterate()
        assert abs(st.rmse - rmse) <= REL * rmse
        assert abs(st.free_energy - o.s.last_free_energy) <= REL * abs(o.s.last_free_energy)
    assert st.num_levels > 100                  # long dependency chains: many small levels
    assert rel_err(g.get_params()["mu_v"], o.params()["mu_v"]) <= REL


# rows of the small multi-hot sets: 20,000 give ~143-entry columns (the 256 x 1 workgroup shape),
# 45,000 ~320-entry columns (128 x 3, dispatch_shape in csrc/vbfm_device.h)
SHAPE_ROWS = [20_000, 45_000]


@pytest.mark.parametrize("n", SHAPE_ROWS)
@pytest.mark.parametrize("xmode", [0, 1])
def test_entry_store_equals_column_layout(xmode, n):
    """The entry store sweeps every column's entries in the column layout's order with the same
    per-thread assignment and reduction tree, and the data-set sums (w0, alpha, free energy,
    train quirk) add the rows in row order on both: the two layouts agree bit for bit over three
    iterations (x = 1 without a stored x array, and x ~ U(0.5, 1.5)), at two workgroup shapes."""
    D, lo, hi, k = 3000, 3, 40, 4
    res = {}
    for layout in ("entry", "column"):
        g = vbfm.FMLearnVB(1, 1, k, D + 1, min_target=1.0, max_target=5.0, layout=layout)
        g.init(7, 0.1)
        g.synth_multihot(0, n, D, lo, hi, 1000, xmode)
        g.synth_multihot(1, 2000, D, lo, hi, 500000, xmode)
        g.init_caches()
        assert g.layout() == layout
        st = [g.iterate() for _ in range(3)]
        res[layout] = ([(s.rmse, s.free_energy, s.alpha, s.mu_0_dash, s.train_quirk) for s in st],
                       g.get_params()["mu_v"], g.rows()["e"])
        g.close()
    assert res["entry"][0] == res["column"][0]
    np.testing.assert_array_equal(res["entry"][1], res["column"][1])
    np.testing.assert_array_equal(res["entry"][2], res["column"][2])


def test_entry_store_refused_where_it_cannot_apply(monkeypatch):
    """A row listing a feature twice puts it twice in one level: auto falls back to the column
    layout, an explicit entry request fails loudly; VBFM_ESTORE=0 keeps the column layout."""
    import os
    from conftest import GOLDEN
    d = os.path.join(GOLDEN, "tiny_dup")
    train = vbfm.DataSubset.load(os.path.join(d, "train.libfm"))
    test = vbfm.DataSubset.load(os.path.join(d, "test.libfm"))
    D = vbfm.num_all_attribute(train, test)
    for layout, expect in (("auto", "column"), ("entry", None)):
        g = vbfm.FMLearnVB(1, 1, 3, D, min_target=train.min_target, max_target=train.max_target, layout=layout)
        g.init(5, 0.1)
        g.set_data(train, test)
        if expect is None:
            with pytest.raises(vbfm.VbfmError, match="entry store not possible"):
                g.init_caches()
        else:
            g.init_caches()
            assert g.layout() == expect
        g.close()
    monkeypatch.setenv("VBFM_ESTORE", "0")
    g = vbfm.FMLearnVB(1, 1, 3, 3001, min_target=1.0, max_target=5.0)
    g.init(5, 0.1)
    g.synth_multihot(0, 5000, 3000, 3, 20, 1, 0)
    g.synth_multihot(1, 500, 3000, 3, 20, 2, 0)
    g.init_caches()
    assert g.layout() == "column"


@pytest.mark.parametrize("n", SHAPE_ROWS)
@pytest.mark.parametrize("xmode", [0, 1])
@pytest.mark.parametrize("form", ["deferred", "two_pass", "rccl_chunks"])
def test_entry_store_split_forms_equal_fused(form, xmode, n, monkeypatch):
    """The entry store under row shards (VBFM_FORCE_SPLIT=1 on one rank): deferred -- level l's
    kernel applies each record's pending correction (its row's previous entry, from any earlier
    level, through a posterior table over all level features; a row's first entry the previous
    sweep's carried one), reduces, moves; two_pass -- statistics, all-reduce, correction + move
    (VBFM_DEFER=0); rccl_chunks -- the deferred form through a 1-rank RCCL communicator with
    each level's exchange in 3 chunks. Every form equals the fused single-rank entry store bit
    for bit over three iterations (the same per-column order of every sum), at two workgroup
    shapes."""
    D, lo, hi, k = 3000, 3, 40, 4

    def run(split):
        monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
        monkeypatch.setenv("VBFM_DEFER", "0" if form == "two_pass" else "1")
        comm = split == "1" and form == "rccl_chunks"
        monkeypatch.setenv("VBFM_FORCE_COMM", "1" if comm else "0")
        monkeypatch.setenv("VBFM_AR_CHUNKS", "3")
        g = vbfm.FMLearnVB(1, 1, k, D + 1, min_target=1.0, max_target=5.0, layout="entry")
        if comm:
            g.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
        g.init(7, 0.1)
        g.synth_multihot(0, n, D, lo, hi, 1000, xmode)
        g.synth_multihot(1, 2000, D, lo, hi, 500000, xmode)
        g.init_caches()
        assert g.layout() == "entry"
        st = [g.iterate() for _ in range(3)]
        out = ([(s.rmse, s.free_energy, s.alpha, s.mu_0_dash, s.train_quirk) for s in st],
               g.get_params()["mu_v"], g.rows()["e"])
        g.close()
        return out

    fused, split = run("0"), run("1")
    assert split[0] == fused[0]
    np.testing.assert_array_equal(split[1], fused[1])
    np.testing.assert_array_equal(split[2], fused[2])


@pytest.mark.parametrize("n", [15_000, 45_000])
@pytest.mark.parametrize("method", ["als", "mcmc"])
def test_entry_store_split_mcmc_equals_fused(method, n, monkeypatch):
    """MCMC / ALS on the entry store under row shards (the two-pass split: statistics, all-reduce,
    draw + move) with the device RNG streams: the fused single-rank chain bit for bit, at two
    workgroup shapes (~100- and ~300-entry columns: 64 x 2 and 128 x 3)."""
    D, lo, hi, k = 2500, 3, 30, 3

    def run(split):
        monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
        g = vbfm.FMLearnMCMC(1, 1, k, D + 1, min_target=1.0, max_target=5.0, method=method, layout="entry")
        g.init_device(7, 0.1)
        g.synth_multihot(0, n, D, lo, hi, 1000, 1)
        g.synth_multihot(1, 1500, D, lo, hi, 500000, 1)
        g.init_caches()
        assert g.layout() == "entry"
        st = [g.iterate() for _ in range(3)]
        out = ([s.rmse_all for s in st], g.get_params()["v"])
        g.close()
        return out

    fused, split = run("0"), run("1")
    assert split[0] == fused[0]
    np.testing.assert_array_equal(split[1], fused[1])


def test_next_level_prefetch_changes_nothing(monkeypatch):
    """The level kernel's touch of the next level's column bounds (VBFM_PREFETCH, default on) is a
    load whose value is never used: the entry store and the field store run bit for bit as
    without it."""
    res = {}
    for pf in ("1", "0"):
        monkeypatch.setenv("VBFM_PREFETCH", pf)
        g = vbfm.FMLearnVB(1, 1, 3, 3001, min_target=1.0, max_target=5.0, layout="entry")
        g.init(7, 0.1)
        g.synth_multihot(0, 45_000, 3000, 3, 40, 1000, 0)
        g.synth_multihot(1, 2000, 3000, 3, 40, 500000, 0)
        g.init_caches()
        st = [g.iterate() for _ in range(2)]
        res["entry", pf] = ([(s.rmse, s.free_energy) for s in st], g.get_params()["mu_v"])
        g.close()
        rp, f, v, y = synth.generate(30_000, 6, 100, 3, 0)
        te = synth.generate(1000, 6, 100, 4, 0)
        g = vbfm.FMLearnVB(1, 1, 3, 601, min_target=float(y.min()), max_target=float(y.max()), layout="level")
        g.init(7, 0.1)
        g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, 600), vbfm.DataSubset.from_csr(*te, 600))
        g.init_caches()
        assert g.layout() == "level"
        st = [g.iterate() for _ in range(2)]
        res["level", pf] = ([(s.rmse, s.free_energy) for s in st], g.get_params()["mu_v"])
        g.close()
    for lay in ("entry", "level"):
        assert res[lay, "1"][0] == res[lay, "0"][0]
        np.testing.assert_array_equal(res[lay, "1"][1], res[lay, "0"][1])
