"""Dependency levels of the train features (vbfm_capi.hip build_schedule): the relaxation's fixed
point (k_level_relax, one round per row switch on the longest path) and Kahn's order (k_kahn_*,
one pass over the edges, the default once three relaxation rounds have not converged) give the
same levels, equal to the numpy restatement (tests/shards.py levels): on multi-hot rows
(hundreds of levels), and on ragged rows with empty rows, ids listed twice in a row, a column
listing a row twice and unused features."""
import numpy as np
import pytest

import shards
import synth
import vbfm

pytestmark = pytest.mark.gpu


def _ragged(seed=5, n=5000, nf=800):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 12, n)                       # empty rows included
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    f = rng.integers(0, nf - 50, int(rp[-1]))           # repeats inside rows; 50 unused features
    v = rng.uniform(0.5, 1.5, int(rp[-1]))
    y = rng.normal(size=n)
    return rp, f, v, y, nf


@pytest.mark.parametrize("case", ["multihot", "ragged"])
def test_schedule_modes_agree(case, monkeypatch):
    if case == "multihot":
        n, D, lo, hi = 20_000, 3000, 5, 60
        rp, f, _, _ = synth.generate_multihot(n, D, lo, hi, 17, 1)
        nf = D

        def setup(g):
            g.synth_multihot(0, n, D, lo, hi, 17, 1)
    else:
        rp, f, v, y, nf = _ragged()
        ds = vbfm.DataSubset.from_csr(rp, f, v, y, num_feature=nf)

        def setup(g):
            g.set_data(ds, ds)
    expect = shards.levels(rp, f, nf)
    got = {}
    for mode in ("relax", "kahn", "auto"):
        monkeypatch.setenv("VBFM_SCHEDULE", mode)
        g = vbfm.FMLearnVB(1, 1, 2, nf + 1)
        setup(g)
        lv, L = g.levels()
        g.close()
        exp = np.ones(len(lv), dtype=np.int64)
        exp[:nf] = expect
        np.testing.assert_array_equal(lv.astype(np.int64), exp)
        assert L == int(exp.max())
        got[mode] = L
    assert got["relax"] > 50                              # long chains: the case Kahn's order is for


def test_kahn_schedule_trains_like_relaxation(monkeypatch):
    """The whole learner on both schedules: the same levels give bit-identical iterations."""
    rp, f, v, y, nf = _ragged(seed=9, n=8000, nf=600)
    ds = vbfm.DataSubset.from_csr(rp, f, v, y, num_feature=nf)
    res = {}
    for mode in ("relax", "kahn"):
        monkeypatch.setenv("VBFM_SCHEDULE", mode)
        g = vbfm.FMLearnVB(1, 1, 3, nf, min_target=float(y.min()), max_target=float(y.max()))
        g.init(3, 0.1)
        g.set_data(ds, ds)
        g.init_caches()
        st = [g.iterate() for _ in range(2)]
        res[mode] = ([(s.rmse, s.free_energy) for s in st], g.get_params()["mu_v"])
        g.close()
    assert res["relax"][0] == res["kahn"][0]
    np.testing.assert_array_equal(res["relax"][1], res["kahn"][1])


@pytest.mark.parametrize("stride", [1, 7])
def test_sampled_launch_events(stride):
    """vbfm_set_profiling(ctx, stride): an event pair around every stride-th v-level launch (bench.py
    samples the launches of many-level data so that the timing does not slow the sweep); the
    sampled launches are counted, their summed time averages like the full set."""
    n, D, lo, hi, k = 20_000, 3000, 5, 60, 4
    g = vbfm.FMLearnVB(1, 1, k, D + 1, min_target=1.0, max_target=5.0)
    g.init(7, 0.1)
    g.synth_multihot(0, n, D, lo, hi, 1000, 1)
    g.synth_multihot(1, 2000, D, lo, hi, 500000, 1)
    g.init_caches()
    g.set_profiling(True)
    full = g.iterate()
    g.set_profiling(True, stride)
    st = g.iterate()
    g.close()
    assert full.n_vlevel_launches == full.num_levels * k
    assert st.n_vlevel_launches == -(-full.n_vlevel_launches // stride)
    a_full = full.ms_vlevel_kernels / full.n_vlevel_launches
    a = st.ms_vlevel_kernels / st.n_vlevel_launches
    assert 0.5 * a_full < a < 2.0 * a_full


@pytest.mark.parametrize("shape", ["c3_fields", "multihot_bench"])
def test_kahn_equals_relaxation_at_bench_size(shape, monkeypatch):
    """At the bench sizes: C3's 1e7 rows x 40 fields (level = field + 1, 25k columns of ~400
    entries per frontier) and the multi-hot bench's 1e7 rows x U(5,60) ids of 1e6 features
    (785 levels): Kahn's order gives the relaxation's levels."""
    got = {}
    for mode in ("relax", "kahn"):
        monkeypatch.setenv("VBFM_SCHEDULE", mode)
        if shape == "c3_fields":
            F, S = 40, 25_000
            g = vbfm.FMLearnVB(1, 1, 2, F * S + 1)
            g.synth(0, 10_000_000, F, S, 1000, 0)
        else:
            g = vbfm.FMLearnVB(1, 1, 2, 1_000_001)
            g.synth_multihot(0, 10_000_000, 1_000_000, 5, 60, 1000, 0)
        got[mode] = g.levels()
        g.close()
    np.testing.assert_array_equal(got["relax"][0], got["kahn"][0])
    assert got["relax"][1] == got["kahn"][1]
    if shape == "c3_fields":
        assert got["kahn"][1] == 40
        np.testing.assert_array_equal(got["kahn"][0][:40 * 25_000], np.arange(40 * 25_000) // 25_000 + 1)
    else:
        assert got["kahn"][1] == 785
