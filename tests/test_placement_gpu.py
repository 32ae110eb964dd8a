"""Record-buffer placement tuning of the level store (tune_placement, csrc/vbfm_capi.hip; DESIGN
§5b): which physical buffers hold the records changes the level kernel's speed only, so a learner
that tuned its placement must match one that did not, bit for bit, and the report
(vbfm_placement_info) must name the two best-scored candidates."""
import numpy as np
import pytest

import synth
import vbfm

pytestmark = pytest.mark.gpu


def _run(env, monkeypatch, n=2_100_000, F=3, S=2100, k=2, seed=41):
    for kk in ("VBFM_PLACE", "VBFM_PLACE_TRIES", "VBFM_LAYOUT", "VBFM_WAVE"):
        monkeypatch.delenv(kk, raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    rp, f, v, y = synth.generate(n, F, S, seed, 0)
    rpt, ft, vt, yt = synth.generate(500, F, S, seed + 1, 0)
    D = F * S + 1
    g = vbfm.FMLearnVB(1, 1, k, D, min_target=float(y.min()), max_target=float(y.max()), layout="level")
    g.init(5, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
    g.init_caches()
    st = g.iterate()
    assert g.layout() == "level"
    place = g.placement()
    p = g.get_params()
    rows = g.rows()
    out = {"rmse": st.rmse, "mu_v": np.asarray(p["mu_v"]), "sigma_v": np.asarray(p["sigma_v"]),
           "mu_w": np.asarray(p["mu_w"]), "e": rows["e"], "t": rows["t"]}
    g.close()
    return out, place


def test_placement_is_bit_identical_and_reported(monkeypatch):
    ref, p0 = _run({"VBFM_PLACE": "0"}, monkeypatch)
    assert p0 == ([], [-1, -1])
    got, (ms, kept) = _run({"VBFM_PLACE_TRIES": "6"}, monkeypatch)
    for key in ref:
        np.testing.assert_array_equal(np.asarray(got[key]), np.asarray(ref[key]), err_msg=key)
    assert len(ms) == 6 and all(m > 0 for m in ms)
    assert kept[0] != kept[1] and all(0 <= i < 6 for i in kept)
    order = sorted(range(6), key=lambda i: ms[i])
    assert ms[kept[0]] == ms[order[0]] and ms[kept[1]] == ms[order[1]]
