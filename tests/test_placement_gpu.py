"""Record-buffer placement tuning of the level store (tune_placement, csrc/vbfm_capi.hip; DESIGN
§5b): which physical buffers hold the records changes the level kernel's speed only, so a learner
that tuned its placement must match one that did not, bit for bit, and the report
(vbfm_placement_info) must name the kept pair: the best pair among the best-scored candidates
(the store ping-pongs between two buffers, so the best few singles are scored again as pairs),
or the best two singles with VBFM_PLACE_PAIRS=0. The search stays inside the
caller's budget (vbfm_config place_candidates / place_budget_bytes) and half of the free device
memory, degrades to fewer candidates (or none) when memory is short, and a failure inside it
leaves no candidate allocated and the next call rebuilding the store (VBFM_FAULT=placement)."""
import numpy as np
import pytest

import synth
import vbfm

pytestmark = pytest.mark.gpu


N_ROWS = 2_100_000           # >= 2e6: the search runs
REC_BYTES = N_ROWS * 64      # one record buffer


def _data(n=N_ROWS, F=3, S=2100, seed=41):
    rp, f, v, y = synth.generate(n, F, S, seed, 0)
    rpt, ft, vt, yt = synth.generate(500, F, S, seed + 1, 0)
    return (vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S),
            F * S + 1, float(y.min()), float(y.max()))


def _run(env, monkeypatch, k=2, cfg=None, data=None, fail_first=None):
    for kk in ("VBFM_PLACE", "VBFM_PLACE_TRIES", "VBFM_PLACE_BUDGET_GB", "VBFM_PLACE_PAIRS", "VBFM_LAYOUT",
               "VBFM_FAULT"):
        monkeypatch.delenv(kk, raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    train, test, D, lo, hi = data or _data()
    g = vbfm.FMLearnVB(1, 1, k, D, min_target=lo, max_target=hi, layout="level", **(cfg or {}))
    g.init(5, 0.1)
    g.set_data(train, test)
    if fail_first:   # the first store build fails inside the search; the next call builds it again
        monkeypatch.setenv("VBFM_FAULT", fail_first)
        with pytest.raises(vbfm.VbfmError, match="VBFM_FAULT=" + fail_first):
            g.init_caches()
        monkeypatch.delenv("VBFM_FAULT")
    g.init_caches()
    st = g.iterate()
    assert g.layout() == "level"
    place = g.placement()
    setup = g.setup_info()
    p = g.get_params()
    rows = g.rows()
    out = {"rmse": st.rmse, "mu_v": np.asarray(p["mu_v"]), "sigma_v": np.asarray(p["sigma_v"]),
           "mu_w": np.asarray(p["mu_w"]), "e": rows["e"], "t": rows["t"]}
    g.close()
    return out, place, setup


def _same(got, ref):
    for key in ref:
        np.testing.assert_array_equal(np.asarray(got[key]), np.asarray(ref[key]), err_msg=key)


def test_placement_is_bit_identical_and_reported(monkeypatch):
    ref, p0, s0 = _run({"VBFM_PLACE": "0"}, monkeypatch)
    assert p0 == ([], [-1, -1])
    assert s0["place_candidates"] == 0 and s0["place_bytes"] == 0 and s0["s_placement"] == 0
    assert s0["s_schedule"] > 0 and s0["s_store"] > 0 and s0["s_set_train"] > 0
    got, (ms, kept), su = _run({"VBFM_PLACE_TRIES": "6", "VBFM_PLACE_PAIRS": "3"}, monkeypatch)
    _same(got, ref)
    assert su["place_candidates"] == 6 and su["place_kept"] == kept
    assert su["place_bytes"] == 6 * REC_BYTES            # 4 fresh candidates + the stash + the reference
    assert 0 < su["s_placement"] <= su["s_store"]
    assert len(ms) == 6 and all(m > 0 for m in ms)
    assert kept[0] != kept[1] and all(0 <= i < 6 for i in kept)
    order = sorted(range(6), key=lambda i: ms[i])
    assert set(kept) <= set(order[:3])                   # a pair among the best three singles
    got2, (ms2, kept2), _ = _run({"VBFM_PLACE_TRIES": "6", "VBFM_PLACE_PAIRS": "0"}, monkeypatch)
    _same(got2, ref)
    order2 = sorted(range(6), key=lambda i: ms2[i])
    assert ms2[kept2[0]] == ms2[order2[0]] and ms2[kept2[1]] == ms2[order2[1]]   # the best two singles


def test_placement_budget_from_config(monkeypatch):
    """vbfm_config: place_budget_bytes bounds what the search holds (stash + reference + fresh
    candidates), place_candidates the buffers scored, 1 turns the search off; bit for bit either way."""
    data = _data()
    ref, _, _ = _run({"VBFM_PLACE": "0"}, monkeypatch, data=data)
    got, (ms, kept), su = _run({}, monkeypatch, data=data,
                               cfg={"place_budget_bytes": 3 * REC_BYTES + (1 << 20)})
    _same(got, ref)
    assert len(ms) == 3 and su["place_candidates"] == 3 and su["place_bytes"] == 3 * REC_BYTES
    got, (ms, _), su = _run({}, monkeypatch, data=data, cfg={"place_candidates": 5})
    _same(got, ref)
    assert len(ms) == 5 and su["place_bytes"] == 5 * REC_BYTES
    got, (ms, _), su = _run({}, monkeypatch, data=data, cfg={"place_candidates": 1})
    _same(got, ref)
    assert ms == [] and su["place_candidates"] == 0
    # the environment overrides the configuration
    got, (ms, _), _ = _run({"VBFM_PLACE_TRIES": "4"}, monkeypatch, data=data, cfg={"place_candidates": 9})
    assert len(ms) == 4


def test_placement_with_little_free_memory(monkeypatch):
    """A co-resident allocation (torch's, here) leaves little device memory: the search scores no
    more candidates than half of what is left can hold beside the stash and the reference (none
    when it cannot hold those), and the store still builds, bit for bit the same learner."""
    import torch
    data = _data()
    ref, _, _ = _run({"VBFM_PLACE": "0"}, monkeypatch, data=data)
    for leave in (2 << 30, 2 * REC_BYTES + (550 << 20)):
        torch.cuda.empty_cache()
        free, _ = torch.cuda.mem_get_info()
        hog = torch.empty(max(free - leave, 0), dtype=torch.uint8, device="cuda")
        try:
            got, (ms, _), su = _run({}, monkeypatch, data=data)
        finally:
            del hog
            torch.cuda.empty_cache()
        _same(got, ref)
        bound = 2 + max(0, (leave // 2 - 2 * REC_BYTES) // REC_BYTES)   # free at the search <= leave
        assert su["place_candidates"] == len(ms) and len(ms) in [0] + list(range(3, bound + 1)), (leave, len(ms))
        assert su["place_bytes"] <= leave // 2


def test_placement_failure_frees_candidates_and_rebuilds(monkeypatch):
    """A failure inside the search (VBFM_FAULT=placement: after the third candidate's score) puts
    the records back, frees every fresh candidate, the stash and the reference, and leaves the
    schedule to be rebuilt: the next call builds the store again and the learner matches a clean
    one bit for bit."""
    import torch
    data = _data()
    ref, _, _ = _run({"VBFM_PLACE": "0"}, monkeypatch, data=data)
    for kk in ("VBFM_PLACE", "VBFM_LAYOUT"):
        monkeypatch.delenv(kk, raising=False)
    monkeypatch.setenv("VBFM_PLACE_TRIES", "24")
    train, test, D, lo, hi = data
    g = vbfm.FMLearnVB(1, 1, 2, D, min_target=lo, max_target=hi, layout="level")
    g.init(5, 0.1)
    g.set_data(train, test)
    torch.cuda.empty_cache()
    free0, _ = torch.cuda.mem_get_info()
    monkeypatch.setenv("VBFM_FAULT", "placement")
    with pytest.raises(vbfm.VbfmError, match="VBFM_FAULT=placement"):
        g.init_caches()
    monkeypatch.delenv("VBFM_FAULT")
    free1, _ = torch.cuda.mem_get_info()
    # the half-built store goes with the failure (second record buffer 134 MB, next positions 25 MB,
    # maps); the store build's scratch position map is n * 4 = 8.4 MB: a leak of it, of any
    # candidate (134 MB) or of the stash / reference shows. What stays is the schedule's (KB)
    assert free1 >= free0 - (6 << 20), ("device memory not returned after the failed search (MB)",
                                        (free0 - free1) / 2**20)
    assert g.placement() == ([], [-1, -1])
    g.init_caches()
    st = g.iterate()
    ms, kept = g.placement()
    assert len(ms) == 24
    p = g.get_params()
    rows = g.rows()
    got = {"rmse": st.rmse, "mu_v": np.asarray(p["mu_v"]), "sigma_v": np.asarray(p["sigma_v"]),
           "mu_w": np.asarray(p["mu_w"]), "e": rows["e"], "t": rows["t"]}
    g.close()
    _same(got, ref)
