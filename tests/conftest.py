import gzip
import json
import os
import shutil
import sys

import numpy as np
import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
sys.path.insert(0, TESTS)
sys.path.insert(0, os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def pytest_sessionstart(session):
    """torch's HIP runtime initialised before libvbfm's (tests that size memory with torch.cuda):
    torch initialising second, in a process where libvbfm already created contexts, can find no
    device (a test file run on its own, profiles/r06_*). A no-op without a GPU."""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def load_case(name):
    d = os.path.join(GOLDEN, name)
    with open(os.path.join(d, "trace.json")) as fh:
        t = json.load(fh)
    arrays = {}
    p = os.path.join(d, "arrays.npz")
    if os.path.exists(p):
        with np.load(p) as z:
            arrays = {k: z[k] for k in z.files}
    return t, arrays


@pytest.fixture(scope="session")
def golden():
    return load_case


@pytest.fixture(scope="session")
def sa_split(tmp_path_factory):
    """The bundled ML-1M test file split 90k/10k, unpacked once."""
    d = tmp_path_factory.mktemp("sa")
    out = {}
    for part in ("train", "test"):
        p = str(d / (part + ".libfm"))
        with gzip.open(os.path.join(GOLDEN, "sa_split", part + ".libfm.gz"), "rb") as fi, open(p, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        out[part] = p
    return out


@pytest.fixture(scope="session")
def synth_files(tmp_path_factory):
    """The synthetic golden case's inputs, regenerated from tests/synth.py."""
    import synth
    t, _ = load_case("synth")
    m = t["meta"]
    d = tmp_path_factory.mktemp("synth")
    out = {}
    for part, n, seed in (("train", m["n_rows"], m["seed"]), ("test", m["test_rows"], m["test_seed"])):
        rp, f, v, y = synth.generate(n, m["n_fields"], m["ids_per_field"], seed, m["xmode"])
        p = str(d / (part + ".libfm"))
        synth.write_libfm(p, rp, f, v, y)
        out[part] = p
    return out
