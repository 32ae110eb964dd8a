"""The reference-side binding, compiled and run: oracle/_ref/ref_binding is the learner class a
maintainer would add to the reference: a subclass of the reference's own
fm_learn_vb_simultaneous, built against the unmodified reference headers, whose learn() hands
the reference's DataSubset (data_t, targets, loaded by the reference's own Data::load) and the
parameters its own fm_learn_vb::init drew to libvbfm.so through include/vbfm.h, and iterates on
the GPU. Its per-iteration test RMSE, MAE, "Train=" value, free energy and alpha must match
the reference's own run of the same flow (tests/golden/sa_k8, produced by oracle/_ref/ref_driver
from the same reference code) within 1e-9 relative (north star gate: 1e-6).
"""
import os
import subprocess

import pytest

from conftest import load_case

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BINDING = os.path.join(ROOT, "oracle", "_ref", "ref_binding")
REL = 1e-9


def test_reference_learner_subclass_drives_libvbfm(sa_split, tmp_path):
    if not os.path.exists(BINDING):
        pytest.skip("oracle/_ref/ref_binding not built (make -C oracle ref needs the reference sources)")
    t, _ = load_case("sa_k8")
    m = t["meta"]
    out = subprocess.run([BINDING, "--train", sa_split["train"], "--test", sa_split["test"], "--dim", m["dim"],
                          "--iter", str(m["iter"]), "--seed", str(m["seed"]), "--init_stdev", str(m["init_stdev"])],
                         cwd=str(tmp_path), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = []
    for line in out.stdout.splitlines():
        if line.startswith("BIND "):
            tok = line.split()
            rows.append({tok[i]: float(tok[i + 1]) for i in range(2, len(tok) - 1, 2)})
    assert len(rows) == m["iter"] == len(t["trace"])
    assert "#Iter=  0\tTrain=" in out.stdout                    # the reference's own progress lines
    for it, (got, ref) in enumerate(zip(rows, t["trace"])):
        for key in ("rmse", "mae", "train", "free_energy", "alpha"):
            assert abs(got[key] - ref[key]) <= REL * abs(ref[key]), (it, key, got[key], ref[key])
