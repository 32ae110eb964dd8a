"""Several ranks on the GPU: the multi-GPU kernels and exchange pattern with real ranks.

RCCL refuses two ranks on one GPU ("invalid usage"), and the test box has one GPU. The library's
host exchange (vbfm_comm_init_host) stages every all-reduce of the path in host memory and hands
it to the caller -- here a torch.distributed gloo all_reduce -- so 2 or 3 rank processes sharing
cuda:0 run exactly the code the 8-GPU run executes per rank (row-sharded split kernels, the
max-all-reduced level schedule, the padded feature count, every data-set sum; or the feature
shards' pass exchange), with only the collective itself replaced. Rank 0 then runs the un-sharded
data set in the same process and the results must agree to summation order (1e-9 relative; the
per-level sums change order only). RCCL itself is covered by the 1-rank communicator tests
(test_gpu_parity.py / test_mcmc_gpu.py, VBFM_FORCE_COMM=1).
"""
import os
import queue
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REL = 1e-9


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(kind):
    sys.path.insert(0, HERE)
    import synth
    if kind == "ragged":
        # rows missing fields (the levels no longer hold every row: column-gather layout) and
        # different train feature counts per shard (the padded global feature count)
        N, F, S = 12000, 6, 200
        rp, f, v, y = synth.generate(N, F, S, 21, 1)
        keep = (np.arange(N * F) * 2654435761 % 7) != 3
        keep[:F] = True
        cnt = np.add.reduceat(keep.astype(np.int64), rp[:-1].astype(np.int64))
        rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
        f, v = f[keep], v[keep]
        # the last rows only use low ids: the last shard's own feature count is smaller
        last = N - 800
        lo = int(rp[last])
        f = f.copy()
        f[lo:] = np.minimum(f[lo:], np.uint32(3 * S))
        # keep ids ascending within a row (libfm rows may repeat ids: the reference then
        # updates them sequentially, as the duplicate path does)
        for r in range(last, N):
            a, b = int(rp[r]), int(rp[r + 1])
            order = np.argsort(f[a:b], kind="stable")
            f[a:b], v[a:b] = f[a:b][order], v[a:b][order]
        rpt, ft, vt, yt = synth.generate(1500, F, S, 22, 1)
        return (rp, f, v, y), (rpt, ft, vt, yt), F * S
    if kind == "multihot":   # rows of 3..30 distinct ids, no fields: the entry store's levels miss rows
        tr = synth.generate_multihot(12000, 1500, 3, 30, 5, 1)
        te = synth.generate_multihot(1500, 1500, 3, 30, 6, 1)
        return tr, te, 1500
    N, F, S = 16000, 6, 250
    xmode = 0 if kind == "onehot" else 1   # onehot: every x 1 (no x array, 8-B deferred payloads)
    tr = synth.generate(N, F, S, 5, xmode)
    te = synth.generate(1500, F, S, 6, xmode)
    return tr, te, F * S


def _subset(csr, lo, hi, nf):
    import vbfm
    rp, f, v, y = csr
    sl = slice(int(rp[lo]), int(rp[hi]))
    return vbfm.DataSubset.from_csr(rp[lo:hi + 1] - rp[lo], f[sl], v[sl], y[lo:hi], nf)


def _learner(method, K, D, ymin, ymax, layout):
    import vbfm
    if method == "vb":
        return vbfm.FMLearnVB(1, 1, K, D, min_target=ymin, max_target=ymax, device=0, layout=layout)
    return vbfm.FMLearnMCMC(1, 1, K, D, min_target=ymin, max_target=ymax, device=0, method=method, layout=layout)


def _run(fml, method, train, test, iters, shard=None):
    if shard is not None:
        fml.set_shard_mode("features", shard)
    if method == "vb":
        fml.init(7, 0.1)
    else:
        fml.init_device(7, 0.1)
    fml.set_data(train, test)
    fml.init_caches()
    st = [fml.iterate() for _ in range(iters)]
    p = fml.get_params()
    out = {"layout": fml.layout(), "levels": st[-1].num_levels}
    if method == "vb":
        out.update(rmse=[s.rmse for s in st], fe=[s.free_energy for s in st], alpha=[s.alpha for s in st],
                   mu_v=np.asarray(p["mu_v"]), mu_w=np.asarray(p["mu_w"]))
    else:
        out.update(rmse=[s.rmse_all for s in st], mu_v=np.asarray(p["v"]), mu_w=np.asarray(p["w"]))
    return out


def _worker(rank, world, port, kind, method, layout, mode, out_q):
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scalable-variational-bayesian-factorization-machine_amd"))
        import torch
        import torch.distributed as dist
        import vbfm
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)

        def allreduce(arr, op):
            t = torch.from_numpy(arr.astype(np.float64) if arr.dtype == np.uint32 else arr.copy())
            if arr.dtype == np.uint8:
                t = t.to(torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
            arr[:] = t.numpy().astype(arr.dtype)

        (tr, te, nf) = _data(kind)
        N, Nt = len(tr[3]), len(te[3])
        ymin, ymax = float(tr[3].min()), float(tr[3].max())
        D = nf + 1
        K = 4
        if mode == "features":   # every rank all rows, its chunk of every level's columns
            train, test = _subset(tr, 0, N, nf), _subset(te, 0, Nt, nf)
        else:
            train = _subset(tr, rank * N // world, (rank + 1) * N // world, nf)
            test = _subset(te, rank * Nt // world, (rank + 1) * Nt // world, nf)
        fml = _learner(method, K, D, ymin, ymax, layout)
        fml.comm_init_host(world, rank, allreduce)
        res = _run(fml, method, train, test, 3, shard=0 if mode == "features" else None)
        fml.close()
        if rank == 0:
            ref = _learner(method, K, D, ymin, ymax, layout)
            # feature shards: the same Jacobi arithmetic with the shards one after another in
            # one process; row shards: the un-sharded data set
            res_ref = _run(ref, method, _subset(tr, 0, N, nf), _subset(te, 0, Nt, nf), 3,
                           shard=world if mode == "features" else None)
            ref.close()
            out_q.put({"sharded": res, "single": res_ref})
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as exc:   # reported to the parent instead of a silent hang
        import traceback
        out_q.put({"error": "rank %d: %r\n%s" % (rank, exc, traceback.format_exc())})


def _launch(world, kind, method, layout, mode="rows"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, method, layout, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        msg = q.get(timeout=300)
    except queue.Empty:
        msg = {"error": "no result within 300 s"}
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join()
    assert "error" not in msg, msg["error"]
    return msg["sharded"], msg["single"]


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("world,kind,layout,chunks", [(2, "field", "level", 0), (3, "field", "level", 0),
                                                      (2, "onehot", "level", 0), (2, "field", "column", 0),
                                                      (2, "ragged", "auto", 0), (3, "field", "level", 3),
                                                      (2, "field", "column", 2), (2, "multihot", "entry", 0),
                                                      (3, "multihot", "entry", 2)])
def test_vb_row_shards_match_one_rank(world, kind, layout, chunks, monkeypatch):
    """VB row shards (deferred split kernels on the level-ordered store, stats / correct on the
    column layout) vs the un-sharded data set: RMSE, free energy, alpha per iteration and the
    final parameters within 1e-9. chunks: each level's exchange cut into that many chunks
    (VBFM_AR_CHUNKS, inherited by the rank processes)."""
    if chunks:
        monkeypatch.setenv("VBFM_AR_CHUNKS", str(chunks))
    s, r = _launch(world, kind, "vb", layout)
    # ragged rows: the levels miss rows (the entry store, or the column layout where a row repeats
    # an id); every rank decides like the one-rank run (the repeat flags are all-reduced)
    assert s["layout"] == r["layout"]
    assert s["levels"] == r["levels"]
    for key in ("rmse", "fe", "alpha"):
        for a, b in zip(s[key], r[key]):
            assert abs(a - b) <= REL * abs(b), (key, a, b)
    assert _rel(s["mu_v"], r["mu_v"]) <= REL
    assert _rel(s["mu_w"], r["mu_w"]) <= REL


@pytest.mark.parametrize("method,layout,kind", [("als", "level", "field"), ("als", "level", "onehot"),
                                              ("als", "column", "field"), ("mcmc", "level", "field"),
                                              ("als", "entry", "multihot"), ("mcmc", "entry", "multihot")])
def test_mcmc_row_shards_match_one_rank(method, layout, kind):
    """MCMC / ALS row shards with the device RNG streams (keyed by seed, iteration, factor and
    attribute, so every rank draws the same numbers) vs one rank: ALS is deterministic
    (1e-9); the Gibbs chain only sees the summation order of the statistics change (1e-7)."""
    s, r = _launch(2, kind, method, layout)
    assert s["layout"] == r["layout"] == layout
    tol = REL if method == "als" else 1e-7
    for a, b in zip(s["rmse"], r["rmse"]):
        assert abs(a - b) <= tol * abs(b), (a, b)
    assert _rel(s["mu_v"], r["mu_v"]) <= tol
    assert _rel(s["mu_w"], r["mu_w"]) <= tol


def test_vb_feature_shards_match_in_process_shards():
    """The north star's feature-column partition over 2 ranks == the same 2 shards run one
    after another in one process (vbfm_set_shard_mode), which the oracle's Jacobi restatement
    pins (test_gpu_parity.py::test_feature_shards_vs_oracle)."""
    s, r = _launch(2, "field", "vb", "column", mode="features")
    for key in ("rmse", "fe", "alpha"):
        for a, b in zip(s[key], r[key]):
            assert abs(a - b) <= 1e-12 * abs(b), (key, a, b)
    assert _rel(s["mu_v"], r["mu_v"]) <= 1e-12
