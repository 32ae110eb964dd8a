"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer (a host
ASan/UBSan build of the C restatement; GPU sanitizers are not available on the pool).

tests/host_sanitize.cpp is compiled with -fsanitize=address,undefined together with the
product's host code (csrc/vbfm_host.cpp: the libfm loader, the transpose, the binary reader /
writer, the reference's initial draws) and the oracle (oracle/vbfm_oracle.c), and run on
edge-case, malformed, truncated and multi-threaded inputs; any sanitizer report (out-of-bounds
access, use after free, leak, signed overflow, misaligned access ...) fails the test. CPU only.
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT, TESTS

PKG = os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd")
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off", "-fsanitize=address,undefined",
       "-fno-sanitize-recover=all"]


@pytest.mark.skipif(not (shutil.which("gcc") and shutil.which("g++")), reason="needs gcc / g++")
def test_host_code_under_asan_ubsan(tmp_path):
    obj = str(tmp_path / "oracle.o")
    exe = str(tmp_path / "host_sanitize")
    subprocess.run(["gcc", "-std=c11", *SAN, "-c", os.path.join(ROOT, "oracle", "vbfm_oracle.c"), "-o", obj],
                   check=True, capture_output=True, text=True)
    # the sanitizer runtimes linked statically: the executable's own runtime comes first
    # whatever the environment preloads
    subprocess.run(["g++", "-std=c++17", *SAN, "-static-libasan", "-static-libubsan", "-pthread",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
                    os.path.join(TESTS, "host_sanitize.cpp"), os.path.join(PKG, "csrc", "vbfm_host.cpp"), obj,
                    "-o", exe, "-lm"], check=True, capture_output=True, text=True)
    work = tmp_path / "work"
    work.mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", VBFM_LOADER_THREADS="4")
    r = subprocess.run([exe, str(work)], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-8000:]
    assert "host sanitizer run ok" in r.stdout


@pytest.mark.skipif(not shutil.which("g++"), reason="needs g++")
def test_cli_launcher_under_asan_ubsan(tmp_path):
    """bin/libFM's host logic -- the rank processes it forks (-devices), their row slices, the
    shared-memory exchange (a buffer larger than one slot included), rank 0's files, the -out
    gather across ranks, per-rank checkpoints and the failure path -- built from
    host/libfm_main.cpp with the product's host code and tests/cli_stub.cpp in place of the GPU
    entry points, under ASan + UBSan."""
    exe = str(tmp_path / "libfm_san")
    subprocess.run(["g++", "-std=c++17", *SAN, "-static-libasan", "-static-libubsan", "-pthread",
                    "-I", os.path.join(ROOT, "include"), os.path.join(PKG, "host", "libfm_main.cpp"),
                    os.path.join(PKG, "csrc", "vbfm_host.cpp"), os.path.join(TESTS, "cli_stub.cpp"), "-o", exe],
                   check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    d = os.path.join(TESTS, "golden", "tiny")
    tr, te = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
    ys = [float(l.split()[0]) for l in open(te)]

    def run(cwd, *flags):
        os.makedirs(cwd, exist_ok=True)
        return subprocess.run([exe, "-task", "r", "-train", tr, "-test", te, "-method", "vb", "-dim", "1,1,2",
                               "-seed", "3"] + list(flags), cwd=str(cwd), env=env, capture_output=True, text=True,
                              timeout=300)

    for P in (1, 3):
        r = run(tmp_path / ("p%d" % P), "-iter", "2", "-devices", str(P), "-transport", "host", "-out", "pred.txt",
                "-rlog", "log.tsv", "-save_state", "st")
        assert r.returncode == 0 and "ERROR" not in r.stderr, r.stdout[-3000:] + r.stderr[-6000:]
        rm = open(tmp_path / ("p%d" % P) / "test_rmse_112_vb").read().split()
        assert [float(x) for x in rm] == pytest.approx([sum(ys) / len(ys)] * 2, rel=1e-5)
        fe = open(tmp_path / ("p%d" % P) / "free_energy_112_vb").read().split()
        assert [float(x) for x in fe] == [24.0, 24.0]          # -F = the train rows of all ranks
        assert [float(x) for x in open(tmp_path / ("p%d" % P) / "pred.txt").read().split()] == ys
        assert r.stdout.count("#Iter=") == 2
        files = sorted(os.listdir(tmp_path / ("p%d" % P)))
        assert ("st" in files) if P == 1 else all("st.%d" % q in files for q in range(P))
        r2 = run(tmp_path / ("p%d" % P), "-iter", "1", "-devices", str(P), "-transport", "host", "-resume", "st")
        assert r2.returncode == 0 and "ERROR" not in r2.stderr, r2.stderr[-6000:]
        assert "resuming from st after 2 iterations" in r2.stdout
    # a failing rank (the stub has no RCCL): the launcher reports it and stops the others
    r = run(tmp_path / "fail", "-iter", "2", "-devices", "2")
    assert "no RCCL in the sanitizer build" in r.stderr and "of 2 failed" in r.stderr, r.stderr[-6000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
