"""The libFM-compatible CLI (bin/libFM) against the reference's own outputs.

The reference CLI writes test_rmse_<k0><k1><k>_vb / free_energy_<k0><k1><k>_vb with the
default 6-significant-digit stream format and prints "#Iter=  i\\tTrain=..\\tTest=.." lines
(fm_learn_vb_simultaneous.h:58-73,221-222; fm_learn_vb.h:646-681). The golden traces hold
the reference's values at 17 digits for the same seed; formatted like the reference prints
them they must match digit for digit (differences below 1e-9 relative cannot reach the 6th
significant digit except at a rounding boundary, which the check tolerates by one unit).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, load_case

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd", "bin", "libFM")


def g6(x):
    return "%g" % x


def same6(a, b):
    if a == b:
        return True
    fa, fb = float(a), float(b)
    return abs(fa - fb) <= 1.01 * 10 ** (np.floor(np.log10(abs(fb))) - 5)


def run_cli(tmp_path, train, test, dim, iters, seed, extra=(), method="vb"):
    out = subprocess.run([CLI, "-task", "r", "-train", train, "-test", test, "-method", method, "-dim", dim,
                          "-iter", str(iters), "-seed", str(seed)] + list(extra),
                         cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert "ERROR" not in out.stderr, out.stderr
    return out.stdout


@pytest.mark.parametrize("init", ["host", "replay"])
@pytest.mark.parametrize("case", ["tiny/vb", "tiny/vb_meta"])
def test_cli_tiny_files_match_reference(case, init, tmp_path, monkeypatch):
    """init: the initial draws on the host or generated on the device (vbfm_init_params_replay,
    the CLI's choice for large models)."""
    monkeypatch.setenv("VBFM_INIT", init)
    t, a = load_case(case)
    m = t["meta"]
    d = os.path.join(GOLDEN, case.split("/")[0])
    extra = ["-init_stdev", str(m["init_stdev"]), "-rlog", "log.tsv", "-out", "pred.txt"]
    if "meta" in m:
        extra += ["-meta", os.path.join(d, m["meta"])]
    stdout = run_cli(tmp_path, os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm"), m["dim"],
                     m["iter"], m["seed"], extra)
    tag = m["dim"].replace(",", "")
    rmse = open(tmp_path / ("test_rmse_%s_vb" % tag)).read().split()
    fe = open(tmp_path / ("free_energy_%s_vb" % tag)).read().split()
    assert len(rmse) == len(fe) == m["iter"]
    for it, ref in enumerate(t["trace"]):
        assert same6(rmse[it], g6(ref["rmse"])), (it, rmse[it], ref["rmse"])
        assert same6(fe[it], g6(-ref["free_energy"])), (it, fe[it], ref["free_energy"])
    iters = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", stdout)
    assert len(iters) == m["iter"]
    for (i, tr, te), ref in zip(iters, t["trace"]):
        assert same6(tr, g6(ref["train"])) and same6(te, g6(ref["rmse"]))
    # v_file.txt: fm.v draws (fm_model.h:98), tab-separated, 6 digits
    k = int(m["dim"].split(",")[2])
    vf = np.loadtxt(tmp_path / "v_file.txt", ndmin=2)
    np.testing.assert_allclose(vf.ravel(), a["init_fm_v"], rtol=1e-5, atol=1e-7)
    assert vf.shape[0] == k
    # -out: the clipped predictions of the last iteration
    pred = np.loadtxt(tmp_path / "pred.txt")
    np.testing.assert_allclose(pred, a["iter%d_pred" % (m["iter"] - 1)], rtol=1e-5)
    hdr = open(tmp_path / "log.tsv").readline().rstrip("\n").split("\t")
    assert hdr[:9] == ["rmse", "mae", "time_pred", "time_learn", "time_learn2", "time_learn4", "alpha",
                       "rmse_mcmc_this", "rmse_mcmc_all"]


def test_cli_movielens_split(sa_split, tmp_path):
    t, _ = load_case("sa_k8")
    stdout = run_cli(tmp_path, sa_split["train"], sa_split["test"], "1,1,8", 20, 42, ["-vfile", "0"])
    iters = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", stdout)
    assert len(iters) == 20
    for (i, tr, te), ref in zip(iters, t["trace"]):
        assert same6(te, g6(ref["rmse"])), (i, te, ref["rmse"])
        assert same6(tr, g6(ref["train"])), (i, tr, ref["train"])


def test_cli_binary_input(tmp_path):
    """The .x/.xt/.y triple (Data.h:112-171) gives the same run as the text file."""
    import synth
    rp, f, v, y = synth.generate(3000, 5, 40, 21, 1)
    rpt, ft, vt, yt = synth.generate(300, 5, 40, 22, 1)
    synth.write_libfm(str(tmp_path / "tr.libfm"), rp, f, v, y)
    synth.write_libfm(str(tmp_path / "te.libfm"), rpt, ft, vt, yt)
    synth.write_binary(str(tmp_path / "trb"), 200, rp, f, v, y)
    synth.write_binary(str(tmp_path / "teb"), 200, rpt, ft, vt, yt)
    a = run_cli(tmp_path, str(tmp_path / "tr.libfm"), str(tmp_path / "te.libfm"), "1,1,3", 3, 9, ["-vfile", "0"])
    b = run_cli(tmp_path, str(tmp_path / "trb"), str(tmp_path / "teb"), "1,1,3", 3, 9, ["-vfile", "0"])
    ia = re.findall(r"#Iter=.*", a)
    assert len(ia) == 3 and ia == re.findall(r"#Iter=.*", b)


@pytest.mark.parametrize("case", ["tiny/mcmc", "tiny/mcmc_meta", "tiny/als", "tiny/als_meta_reg"])
def test_cli_mcmc_als_match_reference(case, tmp_path):
    """-method mcmc | als: #Iter lines, test_rmse_<dim>_mcmc, v_file.txt and -out
    (pred_sum_all / num_iter for mcmc, the last predictions for als; clipped)."""
    t, a = load_case(case)
    m = t["meta"]
    d = os.path.join(GOLDEN, case.split("/")[0])
    extra = ["-init_stdev", str(m["init_stdev"]), "-out", "pred.txt", "-rlog", "log.tsv"]
    if "meta" in m:
        extra += ["-meta", os.path.join(d, m["meta"])]
    if "regular" in m:
        extra += ["-regular", ",".join(repr(r) for r in m["regular"])]
    method = "mcmc" if "mcmc" in case else "als"
    stdout = run_cli(tmp_path, os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm"), m["dim"],
                     m["iter"], m["seed"], extra, method=method)
    iters = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", stdout)
    assert len(iters) == m["iter"]
    for (i, tr, te), ref in zip(iters, t["trace"]):
        assert same6(tr, g6(ref["train"])) and same6(te, g6(ref["rmse_all"])), (i, tr, te, ref)
    tag = m["dim"].replace(",", "")
    rmse = open(tmp_path / ("test_rmse_%s_mcmc" % tag)).read().split()
    assert [same6(r, g6(ref["rmse_all"])) for r, ref in zip(rmse, t["trace"])] == [True] * m["iter"]
    assert "Final" not in stdout
    k = int(m["dim"].split(",")[2])
    vf = np.loadtxt(tmp_path / "v_file.txt", ndmin=2)
    np.testing.assert_allclose(vf.ravel(), a["init_fm_v"], rtol=1e-5, atol=1e-7)
    assert vf.shape[0] == k
    pred = np.loadtxt(tmp_path / "pred.txt")
    tg = np.array([float(l.split()[0]) for l in open(os.path.join(d, "test.libfm"))])
    ytr = np.array([float(l.split()[0]) for l in open(os.path.join(d, "train.libfm"))])
    assert np.all(pred >= ytr.min()) and np.all(pred <= ytr.max())
    if method == "mcmc":   # pred_sum_all / num_iter: its RMSE is the last Test= value
        assert abs(np.sqrt(np.mean((pred - tg) ** 2)) - t["trace"][-1]["rmse_all"]) < 1e-5
    hdr = open(tmp_path / "log.tsv").readline().rstrip("\n").split("\t")
    assert "rmse_mcmc_all" in hdr and "alpha" in hdr


@pytest.mark.parametrize("init", ["host", "replay"])
@pytest.mark.parametrize("case", ["tiny/online_b3", "tiny/online_meta", "tiny/online_b1"])
def test_cli_online_matches_reference(case, init, tmp_path, monkeypatch):
    """-method vb_online: "#Iter=  i\\tTest=.." lines, test_rmse_<tag>_vb_online, the free
    energies of the first and last batch appended (as -F) to free_energy_<tag>_vb and printed as
    "free energy F", an empty free_energy_<tag>_vb_online, v_file.txt
    (fm_learn_vb_online_simultaneous.h:37-52, 143-146, 243-244; fm_learn_vb_online.h:636-662)."""
    monkeypatch.setenv("VBFM_INIT", init)
    t, a = load_case(case)
    m = t["meta"]
    d = os.path.join(GOLDEN, case.split("/")[0])
    extra = ["-init_stdev", str(m["init_stdev"]), "-batch", str(m["batch"]), "-out", "pred.txt"]
    if "meta" in m:
        extra += ["-meta", os.path.join(d, m["meta"])]
    stdout = run_cli(tmp_path, os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm"), m["dim"],
                     m["iter"], m["seed"], extra, method="vb_online")
    tag = m["dim"].replace(",", "")
    rmse = open(tmp_path / ("test_rmse_%s_vb_online" % tag)).read().split()
    fe = open(tmp_path / ("free_energy_%s_vb" % tag)).read().split()
    assert open(tmp_path / ("free_energy_%s_vb_online" % tag)).read() == ""
    ref_fe = [x for r in t["trace"] for x in r["free_energy"]]
    assert len(rmse) == m["iter"] and len(fe) == len(ref_fe)
    for it, ref in enumerate(t["trace"]):
        assert same6(rmse[it], g6(ref["rmse"])), (it, rmse[it], ref["rmse"])
    for got, ref in zip(fe, ref_fe):
        assert same6(got, g6(-ref)), (got, ref)
    iters = re.findall(r"#Iter=\s*(\d+)\tTest=(\S+)", stdout)
    assert [int(i) for i, _ in iters] == list(range(m["iter"]))
    for (_, te), ref in zip(iters, t["trace"]):
        assert same6(te, g6(ref["rmse"]))
    printed = [float(x) for x in re.findall(r"^free energy (\S+)$", stdout, re.M)]
    np.testing.assert_allclose(printed, ref_fe, rtol=1e-5)
    k = int(m["dim"].split(",")[2])
    vf = np.loadtxt(tmp_path / "v_file.txt", ndmin=2)
    assert vf.shape[0] == k
    np.testing.assert_allclose(vf.ravel(), a["init_fm_v"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(np.loadtxt(tmp_path / "pred.txt"), a["final_pred"], rtol=1e-5)
    assert "Final\tTrain=nan\tTest=nan" in stdout


@pytest.mark.parametrize("case", ["tiny/vb", "tiny/mcmc", "tiny/als"])
def test_cli_parity_log_17_digits(case, tmp_path):
    """-parity_log: one JSON line per iteration with the values the reference prints at 17
    digits, against the compiled reference's trace at 1e-9 (the 6-digit files cannot carry that),
    plus the sweep's throughput fields."""
    import json
    t, _ = load_case(case)
    m = t["meta"]
    d = os.path.join(GOLDEN, case.split("/")[0])
    method = case.split("/")[1]
    run_cli(tmp_path, os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm"), m["dim"], m["iter"], m["seed"],
            ["-init_stdev", str(m["init_stdev"]), "-parity_log", "parity.jsonl", "-vfile", "0"], method=method)
    lines = [json.loads(x) for x in open(tmp_path / "parity.jsonl")]
    setup, lines = lines[0], lines[1:]            # the first line: what the set-up cost (vbfm_setup_info)
    assert setup["method"] == "setup" and setup["learner"] == method and setup["schedule_s"] > 0
    assert setup["placement_candidates"] == 0     # tiny data: no placement search
    assert len(lines) == m["iter"]
    for it, (got, ref) in enumerate(zip(lines, t["trace"])):
        assert got["iter"] == it and got["method"] == method
        pairs = [("train", "train")]
        if method == "vb":
            pairs += [("test_rmse", "rmse"), ("test_mae", "mae"), ("alpha", "alpha"), ("mu_0_dash", "mu_0_dash"),
                      ("sigma_0_dash", "sigma_0_dash"), ("free_energy", "free_energy")]
        else:
            pairs += [("test_rmse", "rmse_all")]
        for gk, rk in pairs:
            assert abs(got[gk] - ref[rk]) <= 1e-9 * max(abs(ref[rk]), 1e-300), (it, gk, got[gk], ref[rk])
        assert got["ms_v"] > 0 and got["sweep_nnz_k_per_s"] > 0 and 0 < got["hbm_frac_per_gpu"] < 1
        # one rank: no communicator, no exchange
        assert got["exchange_calls"] == 0 and got["exchange_bytes"] == 0


def test_cli_parity_log_online(tmp_path):
    """-parity_log with -method vb_online: test RMSE and the first / last batch's free energy of
    every epoch at 1e-9 against the compiled reference's trace (tiny/online_b3)."""
    import json
    t, _ = load_case("tiny/online_b3")
    m = t["meta"]
    d = os.path.join(GOLDEN, "tiny")
    run_cli(tmp_path, os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm"), m["dim"], m["iter"], m["seed"],
            ["-init_stdev", str(m["init_stdev"]), "-batch", str(m["batch"]), "-parity_log", "p.jsonl", "-vfile", "0"],
            method="vb_online")
    lines = [json.loads(x) for x in open(tmp_path / "p.jsonl")]
    setup, lines = lines[0], lines[1:]            # the set-up line, as for the other methods
    assert setup["method"] == "setup" and setup["learner"] == "vb_online"
    assert len(lines) == m["iter"]
    for it, (got, ref) in enumerate(zip(lines, t["trace"])):
        assert got["iter"] == it and got["method"] == "vb_online"
        pairs = [(got["test_rmse"], ref["rmse"]), (got["free_energy_first"], ref["free_energy"][0]),
                 (got["free_energy_last"], ref["free_energy"][-1])]
        for a, b in pairs:
            assert abs(a - b) <= 1e-9 * abs(b), (it, a, b)
        assert got["ms_v"] > 0 and got["sweep_nnz_k_per_s"] > 0


def write_synth_binary(base, which_rows, F, S, seed, xmode, model_seed):
    """One data set of the BASELINE configs' generator (tests/synth.py, generated on the device,
    copied back) in the reference's binary format (<base>.x/.xt/.y, fmatrix.h:46-52), as the
    reference's own Data::load reads it (Data.h:112-171)."""
    import synth
    import vbfm
    g = vbfm.FMLearnVB(1, 1, 1, F * S + 1, min_target=1.0, max_target=5.0)
    g.synth(0, which_rows, F, S, seed, xmode, model_seed)
    cp, ent, y = g.get_csc(0)
    g.close()
    crow, cval = ent["id"], ent["value"]
    del ent
    rp, feat, val = synth.field_csr_from_csc(which_rows, F, S, cp, crow, cval)
    synth.write_binary_csc(base, F * S, rp, feat, val, y, cp, crow, cval)


def test_cli_c3_k50_binary_files_vs_reference(tmp_path):
    """The drop-in CLI at a BASELINE configuration's own size: C3 -- 1e7 rows x
    40 fields x 25,000 ids (nnz 4e8, real-valued x), k = 50 -- written in the reference's binary
    format and run through bin/libFM -method vb -dim 1,1,50 -iter 2 -seed 3 exactly as the
    reference's CLI would be (libfm.cpp:149-171 load, 215 num_all_attribute, 306-311 method; the
    fixture tests/golden/c3_k50 is the reference's fm_learn_vb_simultaneous run on the same data and
    seed). The -parity_log lines (17 digits) match the reference's trace within 1e-9 relative; the
    reference-format files test_rmse_1150_vb / free_energy_1150_vb and the #Iter= lines match its
    6-digit output; the setup line reports the load, hand-over, schedule and store times."""
    import json
    t, _ = load_case("c3_k50")
    m = t["meta"]
    n, F, S = m["n_rows"], m["n_fields"], m["ids_per_field"]
    write_synth_binary(str(tmp_path / "c3_train"), n, F, S, m["seed"], m["xmode"], m["model_seed"])
    write_synth_binary(str(tmp_path / "c3_test"), m["test_rows"], F, S, m["test_seed"], m["xmode"], m["model_seed"])
    stdout = run_cli(tmp_path, str(tmp_path / "c3_train"), str(tmp_path / "c3_test"), m["dim"], m["iter"],
                     m["ref_seed"], ["-init_stdev", str(m["init_stdev"]), "-parity_log", "parity.jsonl"])
    assert "num_rows=%d\tnum_values=%d\tnum_features=%d" % (n, n * F, F * S) in stdout
    lines = [json.loads(x) for x in open(tmp_path / "parity.jsonl")]
    setup, its = lines[0], lines[1:]
    assert setup["method"] == "setup" and setup["learner"] == "vb"
    assert all(setup[kk] > 0 for kk in ("load_s", "set_train_s", "schedule_s", "store_s"))
    print("C3 via bin/libFM: load %.2f s, hand-over %.2f s, schedule %.2f s, store %.2f s (placement %.2f s, %d "
          "buffers); iterations %s ms" % (setup["load_s"], setup["set_train_s"], setup["schedule_s"],
                                          setup["store_s"], setup["placement_s"], setup["placement_candidates"],
                                          [round(x["ms_total"], 1) for x in its]))
    assert len(its) == m["iter"]
    for x, ref in zip(its, t["trace"]):
        for got, key in (("train", "train"), ("test_rmse", "rmse"), ("test_mae", "mae"), ("alpha", "alpha"),
                         ("sigma_0", "sigma_0"), ("mu_0_dash", "mu_0_dash"), ("sigma_0_dash", "sigma_0_dash"),
                         ("free_energy", "free_energy")):
            assert abs(x[got] - ref[key]) <= 1e-9 * abs(ref[key]), (x["iter"], got, x[got], ref[key])
    rmse = open(tmp_path / "test_rmse_1150_vb").read().split()
    fe = open(tmp_path / "free_energy_1150_vb").read().split()
    iters = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", stdout)
    assert len(rmse) == len(fe) == len(iters) == m["iter"]
    for it, ref in enumerate(t["trace"]):
        assert same6(rmse[it], g6(ref["rmse"])) and same6(fe[it], g6(-ref["free_energy"])), it
        assert same6(iters[it][1], g6(ref["train"])) and same6(iters[it][2], g6(ref["rmse"])), it
    vf = tmp_path / "v_file.txt"     # fm.v's k x D draws, as the reference always writes them
    with open(vf) as fh:
        assert len(fh.readline().split("\t")) == F * S + 1
