"""Edge cases of the data against the oracle (the C restatement pinned to the reference's
fixtures): train rows without entries, a single train row, a feature space far larger than the
data (ids never seen: the +1 / empty-column quirks, fm_learn_vb.h), k = 0, and an empty test set
(the reference's test RMSE is sqrt(0 / 0) = NaN: libfm.cpp prints nan; the sweep itself runs).
Tolerance as test_gpu_parity: REL = 1e-9."""
import math

import numpy as np
import pytest

import oracle_ctypes as oc
import vbfm

pytestmark = pytest.mark.gpu
REL = 1e-9

ROWS = [([(0, 1.0), (3, 1.0)], 4.0), ([(1, 1.0), (2, 0.5)], 2.0), ([(0, 1.0), (2, 1.0)], 3.0),
        ([(3, 2.0), (4, 1.0)], 5.0), ([(1, 1.0)], 1.0)]


def csr(rows):
    rp = np.zeros(len(rows) + 1, dtype=np.uint64)
    f, v, y = [], [], []
    for i, (ents, t) in enumerate(rows):
        rp[i + 1] = rp[i] + len(ents)
        for j, x in ents:
            f.append(j)
            v.append(x)
        y.append(t)
    return rp, np.array(f, dtype=np.uint32), np.array(v, dtype=np.float32), np.array(y, dtype=np.float32)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


# test ids far beyond the train ids: num_all_attribute covers them (libfm.cpp:215), VB never
# updates them, but they enter the sigma sums and the free energy
FAR = [([(0, 1.0), (999, 1.0)], 4.0), ([(1, 1.0), (640, 0.5)], 2.0)]

CASES = {
    "rows_without_entries": ([([], 3.0), ([], 4.0), ([(1, 1.0)], 2.0), ([], 1.0)], ROWS, 2),
    "one_train_row": ([([(0, 1.0), (2, 0.5)], 3.0)], ROWS, 2),
    "test_ids_beyond_train": (ROWS, FAR, 3),
    "k_zero": (ROWS, ROWS, 0),
    "empty_test_set": (ROWS, [], 2),
}


def num_feature(rows):
    return max([j for ents, _ in rows for j, _ in ents], default=-1) + 1


@pytest.mark.parametrize("case", list(CASES))
def test_edge_case_vs_oracle(case):
    train_rows, test_rows, k = CASES[case]
    tr, te = csr(train_rows), csr(test_rows)
    nf_tr, nf_te = num_feature(train_rows), num_feature(test_rows)
    D = max(nf_tr, nf_te) + 1                  # num_all_attribute: the reference's +1
    g = vbfm.FMLearnVB(1, 1, k, D, min_target=float(tr[3].min()), max_target=float(tr[3].max()))
    g.init(11, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(*tr, nf_tr), vbfm.DataSubset.from_csr(*te, nf_te))
    g.init_caches()
    o = oc.VB(1, 1, k, D)
    o.init_params(11, 0.1)
    o.attach(oc.Data(csr=(len(train_rows),) + tr), oc.Data(csr=(len(test_rows),) + te))
    o.init_caches()
    for it in range(3):
        st = g.iterate()
        rmse, mae, quirk = o.iterate()
        if not test_rows:
            assert math.isnan(st.rmse) and math.isnan(rmse), (st.rmse, rmse)
        else:
            assert rel(st.rmse, rmse) <= REL, (it, st.rmse, rmse)
            assert rel(st.mae, mae) <= REL, (it, st.mae, mae)
        assert rel(st.free_energy, o.s.last_free_energy) <= REL, (it, st.free_energy, o.s.last_free_energy)
        assert rel(st.alpha, o.s.alpha) <= REL, (it, st.alpha, o.s.alpha)
    p, op = g.get_params(), o.params()
    for key in ("mu_w", "sigma_w") + (("mu_v", "sigma_v") if k else ()):
        a, b = np.asarray(p[key], dtype=np.float64), np.asarray(op[key], dtype=np.float64)
        assert np.max(np.abs(a - b)) <= REL * max(np.max(np.abs(b)), 1e-300), key
    g.close()
