"""The row-sharded exchange pattern of the multi-GPU path, on CPU with gloo (world_size 2).

libvbfm's multi-rank mode splits the train rows over ranks and, per dependency level,
all-reduces each feature's sufficient statistics (and every whole-data-set sum) so that all
ranks compute identical posteriors (vbfm_capi.hip: sweep_level / allreduce_host). Here the
same decomposition runs through the oracle's sharded update_all
(or_vb_update_all_sharded) with a torch.distributed gloo all-reduce as the exchange, and
must reproduce the single-process update_all to summation-order accuracy.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, F, S, K, SEED, ITERS = 6000, 6, 120, 3, 17, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import oracle_ctypes as oc
    import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rp, f, v, y = synth.generate(N, F, S, SEED, 1)
    rpt, ft, vt, yt = synth.generate(500, F, S, SEED + 1, 1)
    lo, hi = rank * N // world, (rank + 1) * N // world
    srp = (rp[lo:hi + 1] - rp[lo]).astype(np.uint64)
    sl = slice(int(rp[lo]), int(rp[hi]))
    shard = oc.Data(csr=(hi - lo, srp, f[sl], v[sl], y[lo:hi]))
    test = oc.Data(csr=(500, rpt, ft, vt, yt))
    D = F * S + 1
    vb = oc.VB(1, 1, K, D)
    vb.init_params(3, 0.1)
    vb.attach(shard, test)
    vb.s.min_target, vb.s.max_target = float(y.min()), float(y.max())
    vb.init_caches()

    @oc.ALLREDUCE_FN
    def allreduce(buf, n, user):
        arr = np.ctypeslib.as_array(buf, shape=(n,))
        t = torch.from_numpy(arr.copy())
        dist.all_reduce(t)
        arr[:] = t.numpy()

    for _ in range(ITERS):
        oc.lib().or_vb_update_all_sharded(ctypes.byref(vb.s), ctypes.byref(shard.d), N, F * S, allreduce, None)
    p = vb.params()
    out_q.put((rank, p["mu_v"], p["mu_w"], vb.s.alpha, vb.s.last_free_energy))
    dist.barrier()
    dist.destroy_process_group()


def test_row_sharded_world2_matches_single_process():
    import oracle_ctypes as oc
    import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(2):
        r, mu_v, mu_w, alpha, fe = q.get(timeout=300)
        res[r] = (mu_v, mu_w, alpha, fe)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # both ranks hold identical parameters
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][2] == res[1][2]
    # and they equal the un-sharded update_all up to summation order
    rp, f, v, y = synth.generate(N, F, S, SEED, 1)
    rpt, ft, vt, yt = synth.generate(500, F, S, SEED + 1, 1)
    tr, te = oc.Data(csr=(N, rp, f, v, y)), oc.Data(csr=(500, rpt, ft, vt, yt))
    vb = oc.VB(1, 1, K, F * S + 1)
    vb.init_params(3, 0.1)
    vb.attach(tr, te)
    vb.init_caches()
    for _ in range(ITERS):
        vb.step("update_all")
    p = vb.params()
    scale = np.max(np.abs(p["mu_v"]))
    assert np.max(np.abs(res[0][0] - p["mu_v"])) <= 1e-12 * scale
    assert np.max(np.abs(res[0][1] - p["mu_w"])) <= 1e-12 * np.max(np.abs(p["mu_w"]))
    assert abs(res[0][2] - vb.s.alpha) <= 1e-12 * abs(vb.s.alpha)
    assert abs(res[0][3] - vb.s.last_free_energy) <= 1e-12 * abs(vb.s.last_free_energy)
