"""Checkpoint / resume of the VB and MCMC / ALS learners (include/vbfm.h vbfm_save_state / vbfm_load_state).

The reference has no counterpart (it always starts from its initial draws,
fm_learn_vb_simultaneous.h:20): the contract is that a run stopped after i iterations and
resumed from its file in a fresh context continues bit for bit -- every later iteration's
RMSE, free energy, alpha and the final parameters equal the uninterrupted run's -- and that a
file is refused for another model configuration or another train data set.
"""
import os
import re

import numpy as np
import pytest

import synth
import vbfm
from conftest import GOLDEN, ROOT, load_case

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd", "bin", "libFM")


def _data(n=30000, F=6, S=300, seed=41):
    tr = synth.generate(n, F, S, seed, 1)
    te = synth.generate(1000, F, S, seed + 1, 1)
    return tr, te, F * S


def _learner(tr, te, nf, k, layout, dim=(1, 1)):
    rp, f, v, y = tr
    g = vbfm.FMLearnVB(dim[0], dim[1], k, nf + 1, min_target=float(y.min()), max_target=float(y.max()),
                       layout=layout)
    g.init(7, 0.1)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, nf), vbfm.DataSubset.from_csr(*te, nf))
    return g


def _trace(stats):
    return [(s.rmse, s.mae, s.train_quirk, s.free_energy, s.alpha, s.mu_0_dash) for s in stats]


@pytest.mark.parametrize("split,layout", [("0", "level"), ("0", "column"), ("1", "level"), ("1", "column"),
                                          ("0", "entry")])
def test_resume_continues_bit_for_bit(layout, split, tmp_path, monkeypatch):
    """4 iterations in one go against 2 + save, then load into a fresh context + 2: equal
    bit for bit (level-ordered store, column layout and entry store; fused and deferred-split
    sweeps). The entry store runs on multi-hot rows (its levels miss rows)."""
    monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
    if layout == "entry":
        tr = synth.generate_multihot(8000, 1500, 3, 30, 41, 1)
        te = synth.generate_multihot(800, 1500, 3, 30, 42, 1)
        nf = 1500
    else:
        tr, te, nf = _data()
    k = 5
    a = _learner(tr, te, nf, k, layout)
    a.init_caches()
    full = [a.iterate() for _ in range(4)]
    pa = a.get_params()
    a.close()

    b = _learner(tr, te, nf, k, layout)
    b.init_caches()
    first = [b.iterate() for _ in range(2)]
    path = str(tmp_path / "vb.state")
    b.save_state(path)
    cont = [b.iterate() for _ in range(2)]   # the saving context goes on as if nothing happened
    b.close()
    assert _trace(first + cont) == _trace(full)

    c = _learner(tr, te, nf, k, layout)
    assert c.load_state(path) == 2
    assert c.layout() == layout
    rest = [c.iterate() for _ in range(2)]
    pc = c.get_params()
    c.close()
    assert _trace(first + rest) == _trace(full)
    for key in ("mu_w", "sigma_w", "mu_v", "sigma_v", "hyp_sigma_w", "hyp_sigma_v"):
        np.testing.assert_array_equal(np.asarray(pc[key]), np.asarray(pa[key]), err_msg=key)


def test_load_refuses_other_model_or_data(tmp_path):
    tr, te, nf = _data(n=5000)
    g = _learner(tr, te, nf, 3, "auto")
    g.init_caches()
    g.iterate()
    path = str(tmp_path / "vb.state")
    g.save_state(path)
    g.close()
    # another factor count
    h = _learner(tr, te, nf, 4, "auto")
    with pytest.raises(vbfm.VbfmError, match="another model configuration"):
        h.load_state(path)
    h.close()
    # the same shape, one target changed
    rp, f, v, y = tr
    y2 = y.copy()
    y2[123] += 0.5
    h = _learner((rp, f, v, y2), te, nf, 3, "auto")
    with pytest.raises(vbfm.VbfmError, match="another train data set"):
        h.load_state(path)
    h.close()
    # not a checkpoint
    bad = tmp_path / "bad.state"
    bad.write_bytes(b"\0" * 200)
    h = _learner(tr, te, nf, 3, "auto")
    with pytest.raises(vbfm.VbfmError, match="not a libvbfm checkpoint"):
        h.load_state(str(bad))
    h.close()


def test_load_refuses_other_shape_table(tmp_path):
    """a column's reduction tree follows its workgroup shape and long-column segments, so
    a checkpoint records the tables it ran with (StateHeader::shapes: revision << 48 | segment override
    id << 32 | VBFM_SMALL_MAX) and a file of other tables -- another revision, another cutoff, a
    segment override, or an older libvbfm that did not record it -- is refused instead of resuming
    off by the sums' order."""
    tr, te, nf = _data(n=5000)
    g = _learner(tr, te, nf, 3, "auto")
    g.init_caches()
    g.iterate()
    path = str(tmp_path / "vb.state")
    g.save_state(path)
    g.close()
    raw = bytearray(open(path, "rb").read())
    assert raw[88:96] == (4 << 48 | 128).to_bytes(8, "little")   # revision 4, no segment override, cutoff 128
    for word, origin in ((0, "before round 6"), (3 << 48 | 128, "revision 3"), (4 << 48 | 64, "VBFM_SMALL_MAX 64"),
                         (4 << 48 | 0x1235 << 32 | 128, "segment override 4661")):
        raw[88:96] = word.to_bytes(8, "little")
        other = str(tmp_path / ("other_%x.state" % word))
        open(other, "wb").write(bytes(raw))
        h = _learner(tr, te, nf, 3, "auto")
        with pytest.raises(vbfm.VbfmError, match="another workgroup shape table") as ei:
            h.load_state(other)
        assert origin in str(ei.value)
        assert h.load_state(path) == 1
        h.close()


def test_cli_save_state_and_resume(tmp_path):
    """bin/libFM -save_state after 3 iterations, then -resume for 3 more: the appended
    test_rmse / free_energy files and the #Iter lines continue the 6-iteration run's."""
    d = os.path.join(GOLDEN, "tiny")
    t, _ = load_case("tiny/vb")
    m = t["meta"]
    import subprocess

    def run(cwd, iters, extra):
        os.makedirs(cwd, exist_ok=True)
        out = subprocess.run([CLI, "-task", "r", "-train", os.path.join(d, "train.libfm"), "-test",
                              os.path.join(d, "test.libfm"), "-method", "vb", "-dim", m["dim"], "-iter", str(iters),
                              "-seed", str(m["seed"]), "-init_stdev", str(m["init_stdev"])] + extra,
                             cwd=str(cwd), capture_output=True, text=True, timeout=300)
        assert "ERROR" not in out.stderr, out.stderr
        return out.stdout

    one = tmp_path / "one"
    s_one = run(one, 6, [])
    two = tmp_path / "two"
    run(two, 3, ["-save_state", "vb.state"])
    s_two = run(two, 3, ["-resume", "vb.state"])
    tag = m["dim"].replace(",", "")
    for fn in ("test_rmse_%s_vb" % tag, "free_energy_%s_vb" % tag):
        assert open(one / fn).read() == open(two / fn).read(), fn
    it_one = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", s_one)
    it_two = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", s_two)
    assert it_two == it_one[3:]


def test_load_refuses_truncated_file_and_other_layout_without_touching_state(tmp_path):
    """A truncated checkpoint is refused before anything is replaced (the context then runs on
    exactly as if the load had not been tried); a checkpoint of the level-ordered store is
    refused by a column-layout context (the data-set sums would add the rows in another order)."""
    tr, te, nf = _data(n=5000)
    g = _learner(tr, te, nf, 3, "level")
    g.init_caches()
    g.iterate()
    path = str(tmp_path / "vb.state")
    g.save_state(path)
    assert not os.path.exists(path + ".tmp")
    g.close()
    raw = open(path, "rb").read()
    cut = tmp_path / "cut.state"
    cut.write_bytes(raw[:-64])
    ref = _learner(tr, te, nf, 3, "level")
    ref.init_caches()
    want = _trace([ref.iterate()])
    ref.close()
    h = _learner(tr, te, nf, 3, "level")
    h.init_caches()
    with pytest.raises(vbfm.VbfmError, match="truncated"):
        h.load_state(str(cut))
    assert _trace([h.iterate()]) == want
    h.close()
    h = _learner(tr, te, nf, 3, "column")
    with pytest.raises(vbfm.VbfmError, match="another row layout"):
        h.load_state(path)
    h.close()


def test_failed_save_keeps_the_previous_checkpoint(tmp_path):
    """The file is written beside the target and renamed over it: a save that cannot be
    written (here: the temporary name is a directory) leaves the old checkpoint intact."""
    tr, te, nf = _data(n=5000)
    g = _learner(tr, te, nf, 3, "auto")
    g.init_caches()
    g.iterate()
    path = str(tmp_path / "vb.state")
    g.save_state(path)
    before = open(path, "rb").read()
    os.mkdir(path + ".tmp")
    g.iterate()
    with pytest.raises(vbfm.VbfmError, match="cannot open checkpoint file"):
        g.save_state(path)
    assert open(path, "rb").read() == before
    g.close()


def _mc_learner(tr, te, nf, k, method, rng, layout):
    rp, f, v, y = tr
    g = vbfm.FMLearnMCMC(1, 1, k, nf + 1, min_target=float(y.min()), max_target=float(y.max()), method=method,
                         layout=layout)
    g.init(7, 0.1, rng=rng)
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, nf), vbfm.DataSubset.from_csr(*te, nf))
    return g


def _mc_trace(stats):
    return [(s.rmse_all, s.mae_all, s.rmse_this, s.train_rmse, s.alpha, s.w0, s.rng_skipped) for s in stats]


MC_CASES = [("mcmc", "reference", "level", "0"), ("mcmc", "device", "level", "0"), ("mcmc", "reference", "level", "1"),
            ("mcmc", "device", "column", "0"), ("als", "reference", "level", "0"), ("mcmc", "reference", "entry", "0")]


@pytest.mark.parametrize("method,rng,layout,split", MC_CASES)
def test_mcmc_resume_continues_bit_for_bit(method, rng, layout, split, tmp_path, monkeypatch):
    """The MCMC / ALS chain: 4 iterations in one go against 2 + save, then load into a fresh
    context + 2. Test= is the running mean over all iterations (fm_learn_mcmc_simultaneous.h:
    152-175) and the reference stream continues where it stopped, so every later value, the
    final parameters, the hyper-priors and the averaged test prediction are equal bit for bit
    (reference glibc stream and device streams; level store, column layout, entry store;
    fused and split sweeps)."""
    monkeypatch.setenv("VBFM_FORCE_SPLIT", split)
    if layout == "entry":
        tr = synth.generate_multihot(8000, 1500, 3, 30, 41, 1)
        te = synth.generate_multihot(800, 1500, 3, 30, 42, 1)
        nf = 1500
    else:
        tr, te, nf = _data()
    r = vbfm.RNG_REFERENCE if rng == "reference" else vbfm.RNG_DEVICE
    k = 4
    a = _mc_learner(tr, te, nf, k, method, r, layout)
    a.init_caches()
    full = [a.iterate() for _ in range(4)]
    pa, preda = a.get_params(), a.predict()
    a.close()

    b = _mc_learner(tr, te, nf, k, method, r, layout)
    b.init_caches()
    first = [b.iterate() for _ in range(2)]
    path = str(tmp_path / "mc.state")
    b.save_state(path)
    cont = [b.iterate() for _ in range(2)]   # the saving context goes on as if nothing happened
    b.close()
    assert _mc_trace(first + cont) == _mc_trace(full)

    c = _mc_learner(tr, te, nf, k, method, r, layout)
    assert c.load_state(path) == 2
    assert c.layout() == layout
    rest = [c.iterate() for _ in range(2)]
    pc, predc = c.get_params(), c.predict()
    c.close()
    assert _mc_trace(first + rest) == _mc_trace(full)
    for key in ("w", "v", "w_mu", "w_lambda", "v_mu", "v_lambda", "w0", "alpha"):
        np.testing.assert_array_equal(np.asarray(pc[key]), np.asarray(pa[key]), err_msg=key)
    np.testing.assert_array_equal(predc, preda)


def test_mcmc_load_refuses_other_learner_method_or_rng(tmp_path):
    tr, te, nf = _data(n=5000)
    g = _mc_learner(tr, te, nf, 3, "mcmc", vbfm.RNG_REFERENCE, "auto")
    g.init_caches()
    g.iterate()
    path = str(tmp_path / "mc.state")
    g.save_state(path)
    g.close()
    h = _learner(tr, te, nf, 3, "auto")   # a VB context
    with pytest.raises(vbfm.VbfmError, match="MCMC / ALS checkpoint"):
        h.load_state(path)
    h.close()
    h = _mc_learner(tr, te, nf, 3, "als", vbfm.RNG_REFERENCE, "auto")
    with pytest.raises(vbfm.VbfmError, match="another method"):
        h.load_state(path)
    h.close()
    h = _mc_learner(tr, te, nf, 3, "mcmc", vbfm.RNG_DEVICE, "auto")
    with pytest.raises(vbfm.VbfmError, match="another RNG mode"):
        h.load_state(path)
    h.close()
    v = _learner(tr, te, nf, 3, "auto")
    v.init_caches()
    v.iterate()
    vpath = str(tmp_path / "vb.state")
    v.save_state(vpath)
    v.close()
    h = _mc_learner(tr, te, nf, 3, "mcmc", vbfm.RNG_REFERENCE, "auto")
    with pytest.raises(vbfm.VbfmError, match="a VB checkpoint"):
        h.load_state(vpath)
    h.close()


@pytest.mark.parametrize("method", ["mcmc", "als"])
def test_cli_mcmc_save_state_and_resume(method, tmp_path):
    """bin/libFM -method mcmc | als: 3 iterations + -save_state, then -resume for 3 more: the
    appended test_rmse file, the #Iter lines and -out (the mean of the clipped draws over all 6
    iterations) equal the 6-iteration run's."""
    d = os.path.join(GOLDEN, "tiny")
    import subprocess

    def run(cwd, iters, extra):
        os.makedirs(cwd, exist_ok=True)
        out = subprocess.run([CLI, "-task", "r", "-train", os.path.join(d, "train.libfm"), "-test",
                              os.path.join(d, "test.libfm"), "-method", method, "-dim", "1,1,3", "-iter", str(iters),
                              "-seed", "5", "-init_stdev", "0.1", "-regular", "0.5,1,2"] + extra,
                             cwd=str(cwd), capture_output=True, text=True, timeout=300)
        assert "ERROR" not in out.stderr, out.stderr
        return out.stdout

    one = tmp_path / "one"
    s_one = run(one, 6, ["-out", "pred.txt"])
    two = tmp_path / "two"
    run(two, 3, ["-save_state", "mc.state"])
    s_two = run(two, 3, ["-resume", "mc.state", "-out", "pred.txt"])
    fn = "test_rmse_113_mcmc"
    assert open(one / fn).read() == open(two / fn).read()
    assert open(one / "pred.txt").read() == open(two / "pred.txt").read()
    it_one = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", s_one)
    it_two = re.findall(r"#Iter=\s*(\d+)\tTrain=(\S+)\tTest=(\S+)", s_two)
    assert len(it_one) == 6 and it_two == it_one[3:]


def _ov_learner(tr, te, nf, k, num_batch=7):
    rp, f, v, y = tr
    g = vbfm.FMLearnVBOnline(1, 1, k, nf, min_target=float(y.min()), max_target=float(y.max()))
    g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, nf), vbfm.DataSubset.from_csr(*te, nf))
    g.init(7, 0.1, num_batch)
    return g


def _ov_trace(stats):
    return [(s.rmse, s.mae, s.free_energy_first, s.free_energy_last, s.alpha, s.mu_0_dash, s.sigma_0_dash)
            for s in stats]


@pytest.mark.parametrize("layout", ["auto", "column"])
def test_online_resume_continues_bit_for_bit(layout, tmp_path, monkeypatch):
    """The online learner: 4 epochs against 2 + save, then load into a fresh context + 2. The
    epoch permutations continue from the saved rand() stream and last permutation (the one the
    first context drew ahead on its host thread is not saved), the natural parameters and step
    sizes from the file: every later epoch and the final natural parameters equal bit for bit
    (per-batch level store and column kernels)."""
    monkeypatch.setenv("VBFM_LAYOUT", layout)
    tr, te, nf = _data(n=20000)
    k = 4
    a = _ov_learner(tr, te, nf, k)
    full = [a.epoch() for _ in range(4)]
    sa, pa = a.online_state(), a.get_params()
    a.close()
    b = _ov_learner(tr, te, nf, k)
    first = [b.epoch() for _ in range(2)]
    path = str(tmp_path / "ov.state")
    b.save_state(path)
    cont = [b.epoch() for _ in range(2)]   # the saving context goes on as if nothing happened
    b.close()
    assert _ov_trace(first + cont) == _ov_trace(full)
    c = _ov_learner(tr, te, nf, k)
    assert c.load_state(path) == 2
    rest = [c.epoch() for _ in range(2)]
    sc, pc = c.online_state(), c.get_params()
    c.close()
    assert _ov_trace(first + rest) == _ov_trace(full)
    assert (full[-1].n_lord_batches > 0) == (layout == "auto")
    for key in sa:
        np.testing.assert_array_equal(sc[key], sa[key], err_msg=key)
    for key in ("mu_w", "sigma_w", "mu_v", "sigma_v"):
        np.testing.assert_array_equal(np.asarray(pc[key]), np.asarray(pa[key]), err_msg=key)
    # another mini-batch split is refused
    h = _ov_learner(tr, te, nf, k, num_batch=5)
    with pytest.raises(vbfm.VbfmError, match="another mini-batch split"):
        h.load_state(path)
    h.close()


def test_cli_online_save_state_and_resume(tmp_path):
    """bin/libFM -method vb_online: 3 epochs + -save_state, then -resume for 3 more: the test_rmse
    file, the free energies and the #Iter lines continue the 6-epoch run's."""
    d = os.path.join(GOLDEN, "tiny")
    import subprocess

    def run(cwd, iters, extra):
        os.makedirs(cwd, exist_ok=True)
        out = subprocess.run([CLI, "-task", "r", "-train", os.path.join(d, "train.libfm"), "-test",
                              os.path.join(d, "test.libfm"), "-method", "vb_online", "-dim", "1,1,3", "-iter",
                              str(iters), "-seed", "5", "-init_stdev", "0.1", "-batch", "3"] + extra,
                             cwd=str(cwd), capture_output=True, text=True, timeout=300)
        assert "ERROR" not in out.stderr, out.stderr
        return out.stdout

    one = tmp_path / "one"
    s_one = run(one, 6, [])
    two = tmp_path / "two"
    run(two, 3, ["-save_state", "ov.state"])
    s_two = run(two, 3, ["-resume", "ov.state"])
    for fn in ("test_rmse_113_vb_online", "free_energy_113_vb"):
        assert open(one / fn).read() == open(two / fn).read(), fn
    it_one = re.findall(r"#Iter=\s*(\d+)\tTest=(\S+)", s_one)
    it_two = re.findall(r"#Iter=\s*(\d+)\tTest=(\S+)", s_two)
    assert len(it_one) == 6 and it_two == it_one[3:]


def test_online_checkpoint_refuses_other_store(tmp_path, monkeypatch):
    """the online learner records whether its batches ran on the per-batch level
    store in the checkpoint's layout word; resuming under the other layout (whose data-set sums add
    a batch's rows in another order) is refused before any state is replaced."""
    tr, te, nf = _data(n=20000)
    paths = {}
    for layout in ("auto", "column"):
        monkeypatch.setenv("VBFM_LAYOUT", layout)
        a = _ov_learner(tr, te, nf, 4)
        a.epoch()
        paths[layout] = str(tmp_path / ("ov_%s.state" % layout))
        a.save_state(paths[layout])
        a.close()
    for layout, other in (("auto", "column"), ("column", "auto")):
        monkeypatch.setenv("VBFM_LAYOUT", layout)
        c = _ov_learner(tr, te, nf, 4)
        with pytest.raises(vbfm.VbfmError, match="another row layout"):
            c.load_state(paths[other])
        assert c.load_state(paths[layout]) == 1
        c.close()


def test_online_checkpoint_of_older_library_refused(tmp_path, monkeypatch):
    """online checkpoints written before the layout word recorded the per-batch store
    carry COLUMN whichever store ran; such a file (header flags word 0, as every older libvbfm
    wrote it) is refused with a message naming its origin, not as "another row layout"."""
    monkeypatch.delenv("VBFM_LAYOUT", raising=False)
    tr, te, nf = _data(n=20000)
    a = _ov_learner(tr, te, nf, 4)
    a.epoch()
    path = str(tmp_path / "ov.state")
    a.save_state(path)
    a.close()
    raw = bytearray(open(path, "rb").read())
    assert raw[80:88] == (1).to_bytes(8, "little")        # StateHeader::flags = STATE_FLAG_OV_LAYOUT
    raw[80:88] = bytes(8)                                   # an older library's header
    legacy = str(tmp_path / "ov_legacy.state")
    open(legacy, "wb").write(bytes(raw))
    c = _ov_learner(tr, te, nf, 4)
    with pytest.raises(vbfm.VbfmError, match="older libvbfm"):
        c.load_state(legacy)
    assert c.load_state(path) == 1
    c.close()
