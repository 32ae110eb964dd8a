"""The multi-GPU launch of bin/libFM without a GPU: -plan 1 makes every forked rank print its
launch and shard plan (rank, device, row slice, its nnz) and, with -transport host, all-reduce
its rank number and nnz through the shared-memory exchange before exiting. Checks the shard
plan (contiguous near-equal row slices covering the data, the entries of each slice, all rows
per rank for feature shards), the exchange (sum / max identical on every rank) and the flag
validation of the reference-style CLI (errors print "ERROR:" and exit 0 like libfm.cpp:521-525).
No HIP call is made on any of these paths."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

CLI = os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd", "bin", "libFM")
TINY = os.path.join(GOLDEN, "tiny")

pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="bin/libFM not built (make -C ...amd)")


def plan(tmp_path, *flags, method="vb", train=None, test=None):
    out = subprocess.run([CLI, "-task", "r", "-train", train or os.path.join(TINY, "train.libfm"),
                          "-test", test or os.path.join(TINY, "test.libfm"), "-method", method, "-dim", "1,1,2",
                          "-plan", "1"] + list(flags), cwd=str(tmp_path), capture_output=True, text=True,
                         timeout=120)
    lines = sorted((json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")), key=lambda r: r["rank"])
    return out, lines


def tiny_counts():
    rows = [l.split()[1:] for l in open(os.path.join(TINY, "train.libfm"))]
    trows = [l.split()[1:] for l in open(os.path.join(TINY, "test.libfm"))]
    return [len(r) for r in rows], [len(r) for r in trows]


@pytest.mark.parametrize("P", [2, 3, 5])
def test_row_shard_plan_and_host_exchange(P, tmp_path):
    out, ranks = plan(tmp_path, "-devices", str(P), "-transport", "host")
    assert out.returncode == 0 and "ERROR" not in out.stderr, out.stderr
    assert [r["rank"] for r in ranks] == list(range(P))
    cnt, tcnt = tiny_counts()
    N, NT = len(cnt), len(tcnt)
    for r in ranks:
        assert r["nranks"] == P and r["transport"] == "host" and r["shard"] == "rows"
        assert r["device"] == -1                           # r % visible devices, resolved in the rank
        lo, hi = r["train_rows"]
        assert (lo, hi) == (N * r["rank"] // P, N * (r["rank"] + 1) // P)
        assert r["train_nnz"] == sum(cnt[lo:hi])
        assert r["train_features"] == 12                  # the feature count stays global
        tlo, thi = r["test_rows"]
        assert (tlo, thi) == (NT * r["rank"] // P, NT * (r["rank"] + 1) // P)
        assert r["test_nnz"] == sum(tcnt[tlo:thi])
        # the shared-memory all-reduce: every rank holds the same sums and max
        assert r["xchg_rank_sum"] == P * (P - 1) / 2
        assert r["xchg_nnz_sum"] == sum(cnt)
        assert r["xchg_rank_max"] == P - 1


def test_rccl_plan_one_device_per_rank(tmp_path):
    out, ranks = plan(tmp_path, "-devices", "4")
    assert [r["device"] for r in ranks] == [0, 1, 2, 3]
    assert all(r["transport"] == "rccl" for r in ranks)
    out, ranks = plan(tmp_path, "-devices", "3,1,6")
    assert [r["device"] for r in ranks] == [3, 1, 6]


def test_feature_shard_plan_holds_every_row(tmp_path):
    out, ranks = plan(tmp_path, "-devices", "2", "-shard", "features", "-transport", "host")
    cnt, tcnt = tiny_counts()
    for r in ranks:
        assert r["shard"] == "features"
        assert r["train_rows"] == [0, len(cnt)] and r["train_nnz"] == sum(cnt)
        assert r["test_rows"] == [0, len(tcnt)]
        assert r["xchg_nnz_sum"] == 2 * sum(cnt)


def test_one_rank_plan(tmp_path):
    out, ranks = plan(tmp_path, "-device", "5")
    assert len(ranks) == 1 and ranks[0]["device"] == 5 and ranks[0]["transport"] == "none"


def test_large_row_shard_plan_covers_the_data(tmp_path):
    """A synthetic binary data set with 8 ranks: slices are contiguous, cover every row once,
    and their entries add up to the data set's."""
    import synth
    rp, f, v, y = synth.generate(10007, 4, 50, 3, 1)
    synth.write_binary(str(tmp_path / "tr"), 200, rp, f, v, y)
    rpt, ft, vt, yt = synth.generate(997, 4, 50, 4, 1)
    synth.write_binary(str(tmp_path / "te"), 200, rpt, ft, vt, yt)
    out, ranks = plan(tmp_path, "-devices", "8", "-transport", "host", train=str(tmp_path / "tr"),
                      test=str(tmp_path / "te"))
    assert len(ranks) == 8
    bounds = [tuple(r["train_rows"]) for r in ranks]
    assert bounds[0][0] == 0 and bounds[-1][1] == 10007
    assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    assert all(abs((hi - lo) - 10007 / 8) <= 1 for lo, hi in bounds)
    assert sum(r["train_nnz"] for r in ranks) == 4 * 10007
    assert all(r["xchg_nnz_sum"] == 4 * 10007 for r in ranks)


@pytest.mark.parametrize("flags,msg", [
    (["-devices", "0,0"], "RCCL needs one GPU per rank"),
    (["-devices", "0"], "-devices: expected a rank count"),
    (["-devices", "2", "-transport", "xgmi"], "-transport: rccl or host"),
    (["-devices", "2", "-shard", "cols"], "-shard: rows or features"),
])
def test_flag_errors(flags, msg, tmp_path):
    out, ranks = plan(tmp_path, *flags)
    assert ranks == [] and msg in out.stderr and out.returncode == 0


def test_method_restrictions(tmp_path):
    out, _ = plan(tmp_path, "-devices", "2", method="vb_online")
    assert "vb_online runs on one GPU" in out.stderr
    out, _ = plan(tmp_path, "-devices", "2", "-shard", "features", method="mcmc")
    assert "-shard features is a -method vb mode" in out.stderr
    out, ranks = plan(tmp_path, "-devices", "2", "-transport", "host", method="als")
    assert len(ranks) == 2 and ranks[0]["method"] == "als"


def test_fewer_rows_than_ranks(tmp_path):
    out, ranks = plan(tmp_path, "-devices", "30", "-transport", "host")
    assert ranks == [] and "fewer train rows than ranks" in out.stderr
