"""CPU checks of libvbfm.so: it loads, exports every entry point include/vbfm.h declares,
and its host side (loader, RNG init) matches the oracle / the reference fixtures bit for
bit. No GPU: nothing here launches a kernel."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_ctypes as oc
import synth
import vbfm
from conftest import GOLDEN, ROOT, load_case


def header_functions():
    src = open(os.path.join(ROOT, "include", "vbfm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vbfm_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    L = vbfm.lib()
    declared = header_functions()
    assert declared, "no functions parsed from include/vbfm.h"
    assert sorted(vbfm.EXPORTS) == declared
    for name in declared:
        assert hasattr(L, name), name
    assert L.vbfm_abi_version() == vbfm.ABI_VERSION == 4


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(vbfm.VbfmError):
        vbfm.FMLearnVB(1, 1, 2, 10)


@pytest.mark.parametrize("case", ["tiny", "tiny_dup"])
def test_host_loader_matches_oracle(case):
    for part in ("train", "test"):
        path = os.path.join(GOLDEN, case, part + ".libfm")
        ds = vbfm.DataSubset.load(path)
        od = oc.Data(path)
        cp, cr, cv = od.csc()
        assert ds.num_feature == od.num_feature and ds.num_cases == od.num_rows
        np.testing.assert_array_equal(ds.col_ptr, cp)
        np.testing.assert_array_equal(ds.col_ent["id"], cr)
        np.testing.assert_array_equal(ds.col_ent["value"], cv)
        rp, rf, rv, tg = od.csr()
        np.testing.assert_array_equal(ds.row_ptr, rp)
        np.testing.assert_array_equal(ds.row_ent["id"], rf)
        np.testing.assert_array_equal(ds.target, tg)
        assert ds.min_target == od.d.min_target and ds.max_target == od.d.max_target


def test_host_loader_movielens_split(sa_split):
    ds = vbfm.DataSubset.load(sa_split["train"])
    t, _ = load_case("sa_k8")
    assert ds.num_cases == t["nums"]["train_rows"] and ds.num_feature == t["nums"]["train_nf"]
    od = oc.Data(sa_split["train"])
    np.testing.assert_array_equal(ds.col_ptr, od.csc()[0])
    np.testing.assert_array_equal(ds.col_ent["id"], od.csc()[1])


def test_loader_rejects_garbage(tmp_path):
    p = tmp_path / "bad.libfm"
    p.write_text("3 1:1.0 2:0.5\n4 1:1 junk\n")
    with pytest.raises(vbfm.VbfmError, match="cannot parse line"):
        vbfm.DataSubset.load(str(p))
    with pytest.raises(vbfm.VbfmError, match="unable to open"):
        vbfm.DataSubset.load(str(tmp_path / "missing.libfm"))


def test_loader_text_edge_cases(tmp_path):
    # blank lines, comments, tabs, a row without features, no trailing newline
    p = tmp_path / "e.libfm"
    p.write_text("# comment\n\n5\t 0:1.5  3:-7.9 \n2 1:1e-5 3:2\n-1 1:0.01 6:1 # trailing\n4")
    ds = vbfm.DataSubset.load(str(p))
    od = oc.Data(str(p))
    assert ds.num_cases == od.num_rows == 4
    assert ds.num_feature == od.num_feature == 7
    np.testing.assert_array_equal(ds.col_ent["value"], od.csc()[2])
    np.testing.assert_array_equal(ds.target, np.array([5, 2, -1, 4], dtype=np.float32))


def test_binary_loader_matches_text(tmp_path):
    rp, f, v, y = synth.generate(3000, 6, 50, 11, 1)
    base = str(tmp_path / "d")
    synth.write_libfm(base + ".libfm", rp, f, v, y)
    synth.write_binary(base, 300, rp, f, v, y)
    dt = vbfm.DataSubset.load(base + ".libfm")
    db = vbfm.DataSubset.load(base)            # picks base.x / base.xt / base.y
    assert dt.num_feature == db.num_feature == 300
    np.testing.assert_array_equal(dt.col_ptr, db.col_ptr)
    np.testing.assert_array_equal(dt.col_ent, db.col_ent)
    np.testing.assert_array_equal(dt.target, db.target)
    np.testing.assert_array_equal(dt.row_ent, db.row_ent)


def _host_init(seed, init_stdev, k, D, G=1):
    p = {"mu_w": np.zeros(D), "sigma_w": np.zeros(D), "mu_v": np.zeros(k * D), "sigma_v": np.zeros(k * D),
         "hyp_sigma_w": np.zeros(G), "hyp_sigma_v": np.zeros(G * k)}
    P = vbfm.Params(*[p[n].ctypes.data_as(vbfm.P_f64) for n in
                      ("mu_w", "sigma_w", "mu_v", "sigma_v", "hyp_sigma_w", "hyp_sigma_v")], 0, 0, 0, 0)
    fm_v, fm_w = np.zeros(k * D), np.zeros(D)
    rc = vbfm.lib().vbfm_init_params_host(seed, init_stdev, k, D, G, ctypes.byref(P),
                                          fm_v.ctypes.data_as(vbfm.P_f64), fm_w.ctypes.data_as(vbfm.P_f64))
    assert rc == 0
    return p, fm_v, fm_w, P


@pytest.mark.parametrize("case", ["tiny/steps", "tiny/vb_meta"])
def test_init_params_host_bit_exact_vs_reference(case):
    """srand + fm.v + fm.w + mu_w' + mu_v' draws in the reference's order (libfm.cpp:123-366)."""
    t, a = load_case(case)
    m = t["meta"]
    k = int(m["dim"].split(",")[2])
    D = int(t["nums"]["D"])
    p, fm_v, fm_w, P = _host_init(m["seed"], m["init_stdev"], k, D)
    np.testing.assert_array_equal(fm_v, a["init_fm_v"])
    np.testing.assert_array_equal(fm_w, a["init_fm_w"])
    pref = "s0" if "s0_mu_w" in a else "init"
    np.testing.assert_array_equal(p["mu_w"], a[pref + "_mu_w"])
    np.testing.assert_array_equal(p["mu_v"], a[pref + "_mu_v"])
    np.testing.assert_array_equal(p["sigma_v"], a[pref + "_sigma_v"])
    assert (P.alpha, P.sigma_0, P.mu_0_dash, P.sigma_0_dash) == tuple(a[pref + "_scalars"][:4])


def test_init_params_host_movielens_draws():
    t, a = load_case("sa_k8")
    p, _, _, _ = _host_init(42, 0.1, 8, int(t["nums"]["D"]))
    np.testing.assert_array_equal(p["mu_w"], a["init_mu_w"])


WEIRD_LINES = ["3 1: 2.5", "+3 +1:+2", "4 2:1e-3\t", "  \t5 0:1 1:2#c", "1 7:1 7:2", "2", "2 \t # only target",
               "1.5e1 3:.5 4:5.", "-0 1:-0", "3 1:1\r", "\r", "3 1:1 junk", "3 0x1p3:1", "3 1:x", "3 1:1:2",
               "3 -1:1", "0x1p2 1:1", "3 1:1e", "inf 1:1", "3 70000:1"]


@pytest.mark.parametrize("line", WEIRD_LINES)
def test_loader_line_semantics_vs_oracle(line, tmp_path):
    """Each odd line on its own, against the oracle's sscanf-based Data::load restatement:
    both accept it with the same entries, or both reject it."""
    p = tmp_path / "l.libfm"
    p.write_text("1 0:1\n" + line + "\n")
    try:
        od = oc.Data(str(p))
    except ValueError:
        od = None
    if od is None:
        with pytest.raises(vbfm.VbfmError, match="cannot parse line"):
            vbfm.DataSubset.load(str(p))
        return
    ds = vbfm.DataSubset.load(str(p))
    assert ds.num_cases == od.num_rows and ds.num_feature == od.num_feature
    np.testing.assert_array_equal(ds.target, od.csr()[3])
    np.testing.assert_array_equal(ds.col_ptr, od.csc()[0])
    np.testing.assert_array_equal(ds.col_ent["id"], od.csc()[1])
    np.testing.assert_array_equal(ds.col_ent["value"], od.csc()[2])


def test_loader_threads_agree(tmp_path, monkeypatch):
    """The parallel parse and transpose (several MB, split at line boundaries) give the
    single-threaded result exactly."""
    rp, f, v, y = synth.generate(60000, 12, 400, 21, 1)
    path = str(tmp_path / "big.libfm")
    synth.write_libfm(path, rp, f, v, y)
    out = {}
    for t in ("1", "7"):
        monkeypatch.setenv("VBFM_LOADER_THREADS", t)
        out[t] = vbfm.DataSubset.load(path)
    a, b = out["1"], out["7"]
    for key in ("col_ptr", "col_ent", "target", "row_ptr", "row_ent"):
        np.testing.assert_array_equal(getattr(a, key), getattr(b, key), err_msg=key)
    np.testing.assert_array_equal(b.col_ent["id"], oc.Data(path).csc()[1])


def test_save_binary_round_trip(tmp_path):
    """vbfm_save_data writes the reference's .x/.xt/.y; loading it gives the text data set."""
    rp, f, v, y = synth.generate(5000, 7, 60, 5, 1)
    path = str(tmp_path / "d.libfm")
    synth.write_libfm(path, rp, f, v, y)
    dt = vbfm.DataSubset.load(path)
    base = str(tmp_path / "bin")
    dt.save_binary(base)
    ref = str(tmp_path / "ref")
    synth.write_binary(ref, dt.num_feature, rp, f, v, y)   # tests/synth.py's independent writer
    for ext in (".x", ".xt", ".y"):
        assert open(base + ext, "rb").read() == open(ref + ext, "rb").read(), ext
    db = vbfm.DataSubset.load(base)
    for key in ("col_ptr", "col_ent", "target", "row_ptr", "row_ent"):
        np.testing.assert_array_equal(getattr(dt, key), getattr(db, key), err_msg=key)
