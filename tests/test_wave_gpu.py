"""The one-wave-per-column level kernel (k_level_wave, vbfm_lorder.hip) against the workgroup
kernel it replaces on 256-thread levels (k_level_lord<256, R>, VBFM_WAVE=0): bit for bit.

The wave kernel keeps a column's run in registers and reproduces k_level_lord's reduction tree
(virtual thread i mod 256, virtual waves added in order) on permuted lanes, so the column
statistics, posteriors, corrections and moves must be identical, not merely close. Cases cover
the register-resident path (G = 4 groups for ~160-entry columns, G = 8 for ~400; columns of up to
128 entries take the 64 x 2 workgroup shape, shape_small_max), runs longer than the registers hold
(~600 entries: statistics and move chunk by chunk), x stored or not (one-hot), both workgroup
packings (VBFM_WAVE_WPB 1 / 4), the deferred split (VBFM_FORCE_SPLIT with VBFM_WAVE=1 runs its
wave form, k_defer_wave, against the fused workgroup kernel), the two-pass split (VBFM_DEFER=0:
the workgroup statistics / move kernels against the fused wave kernel), and the oracle at 1e-9
(fm_learn_vb.h:577-644)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import synth
import vbfm

pytestmark = pytest.mark.gpu


def _run(n, F, S, k, xmode, seed, env, monkeypatch, iters=2):
    for kk in ("VBFM_WAVE", "VBFM_WAVE_WPB", "VBFM_FORCE_SPLIT", "VBFM_LAYOUT", "VBFM_DEFER"):
        monkeypatch.delenv(kk, raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    rp, f, v, y = synth.generate(n, F, S, seed, xmode)
    rpt, ft, vt, yt = synth.generate(500, F, S, seed + 1, xmode)
    D = F * S + 1
    g = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()), layout="level")
    g.init(5, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
    g.init_caches()
    st = [g.iterate() for _ in range(iters)]
    assert g.layout() == "level"
    p = g.get_params()
    rows = g.rows()
    out = {"rmse": [s.rmse for s in st], "fe": [s.free_energy for s in st], "mu_v": np.asarray(p["mu_v"]),
           "sigma_v": np.asarray(p["sigma_v"]), "mu_w": np.asarray(p["mu_w"]), "e": rows["e"], "t": rows["t"]}
    g.close()
    return out, (rp, f, v, y, rpt, ft, vt, yt, D)


def _same(a, b):
    for key in a:
        np.testing.assert_array_equal(np.asarray(a[key]), np.asarray(b[key]), err_msg=key)


# (rows, fields, ids per field): mean column length rows / ids
SHAPES = [(64000, 4, 400), (80000, 4, 200), (120000, 3, 200)]


@pytest.mark.parametrize("xmode", [0, 1])
@pytest.mark.parametrize("shape", SHAPES, ids=["len160", "len400", "len600"])
def test_wave_kernel_equals_workgroup_kernel(shape, xmode, monkeypatch):
    n, F, S = shape
    k = 3
    ref, _ = _run(n, F, S, k, xmode, 31, {"VBFM_WAVE": "0"}, monkeypatch)
    for env in ({"VBFM_WAVE": "1"}, {"VBFM_WAVE": "1", "VBFM_WAVE_WPB": "1"},
                {"VBFM_WAVE": "1", "VBFM_FORCE_SPLIT": "1"},
                {"VBFM_WAVE": "1", "VBFM_FORCE_SPLIT": "1", "VBFM_DEFER": "0"}):
        got, _ = _run(n, F, S, k, xmode, 31, env, monkeypatch)
        _same(got, ref)


def test_wave_kernel_vs_oracle(monkeypatch):
    """~400-entry columns with stored x, against the oracle's sequential update_v."""
    n, F, S, k = 40000, 3, 100, 2
    got, (rp, f, v, y, rpt, ft, vt, yt, D) = _run(n, F, S, k, 1, 7, {"VBFM_WAVE": "1"}, monkeypatch)
    o = oc.VB(1, 1, k, D)
    o.init_params(5, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(500, rpt, ft, vt, yt)))
    o.init_caches()
    for it in range(2):
        ro, _, _ = o.iterate()
        assert abs(got["rmse"][it] - ro) <= 1e-9 * ro
    mv = np.asarray(o.params()["mu_v"])
    assert float(np.max(np.abs(got["mu_v"] - mv))) <= 1e-9 * float(np.max(np.abs(mv)))
