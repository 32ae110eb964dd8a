"""Deterministic guard for the read-old / write-new race class.

In the split forms' posterior / draw kernels every wave of a column's workgroup reads the column's
old parameter, and one thread then writes the new value; a barrier must separate the two
(the reference's update_v / update_w use the old value in the correction after computing the new
one: /root/reference/src/libfm/src/fm_learn_vb.h:597-643, fm_learn_mcmc.h:780-835). Without it a
late wave reads the new value as "old" -- which round 5 saw once, at C4 size, in one of several
runs. VBFM_DEBUG_SKEW=1 makes every wave but the first sleep ~50 us before that read
(csrc/vbfm_device.h debug_skew), so the late waves always come after the write: with the barrier
the results stay bit-identical to the fused sweep, without it they differ on every run.
tools/build_nobarrier.sh builds the library without those barriers; this test fails against it.

Columns are ~600 entries (workgroups of 4 waves or more) so every kernel runs multi-wave.
"""
import numpy as np
import pytest

import synth
import vbfm

pytestmark = pytest.mark.gpu

N, F, S, K = 48000, 6, 80, 3


@pytest.fixture(scope="module")
def data():
    tr = synth.generate(N, F, S, 41, 1)
    te = synth.generate(2000, F, S, 42, 1)
    return tr, te


def _run(data, method, layout, split, defer, monkeypatch):
    (rp, f, v, y), (rpt, ft, vt, yt) = data
    monkeypatch.setenv("VBFM_DEBUG_SKEW", "1")
    monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
    monkeypatch.setenv("VBFM_DEFER", defer)
    nf = F * S
    if method == "vb":
        g = vbfm.FMLearnVB(1, 1, K, nf + 1, min_target=float(y.min()), max_target=float(y.max()), layout=layout)
        g.init(5, 0.1)
    else:
        g = vbfm.FMLearnMCMC(1, 1, K, nf + 1, min_target=float(y.min()), max_target=float(y.max()), method=method,
                             layout=layout)
        g.init_device(5, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, nf), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, nf))
    g.init_caches()
    assert g.layout() == layout
    st = [g.iterate() for _ in range(2)]
    p = g.get_params()
    g.close()
    if method == "vb":
        return [(s.rmse, s.free_energy) for s in st], np.asarray(p["mu_v"]), np.asarray(p["mu_w"])
    return [s.rmse_all for s in st], np.asarray(p["v"]), np.asarray(p["w"])


# (method, layout, split forms that run the skewed kernels): VB's two-pass split on the level store
# (k_level_lord_move) and the column layout's correction kernels (k_v/w_level_correct); MCMC / ALS
# MODE 2 draws on both layouts (k_mc_level_lord, k_mc_v/w_level)
@pytest.mark.parametrize("method,layout", [("vb", "level"), ("vb", "column"), ("als", "level"),
                                           ("als", "column"), ("mcmc", "column")])
def test_split_forms_equal_fused_under_skew(data, method, layout, monkeypatch):
    fused = _run(data, method, layout, "0", "1", monkeypatch)
    split = _run(data, method, layout, "1", "0", monkeypatch)
    assert split[0] == fused[0]
    np.testing.assert_array_equal(split[1], fused[1])
    np.testing.assert_array_equal(split[2], fused[2])
