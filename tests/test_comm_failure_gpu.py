"""A rank that fails or stops must not hang the others (include/vbfm.h, "Failure handling of the
exchange"). The sweep whose levels are exchanged is the reference's update_all
(/root/reference/src/libfm/src/fm_learn_vb.h:409-440); the reference itself is one process and has
no counterpart, so these tests pin behaviour, not numbers:

* host-exchange ranks sharing the GPU: one rank takes an injected fault at its first exchange
  inside a sweep (VBFM_FAULT=comm) and leaves; the other rank's exchange fails and its call
  returns an error naming its rank and level instead of waiting;
* RCCL, set-up: rank 0 of a two-rank communicator whose peer never arrives fails at the deadline
  (VBFM_COMM_TIMEOUT_S) with the communicator aborted, and the context refuses later exchanges;
* RCCL, in flight (one GPU, a one-rank communicator): a kernel queued ahead of the first
  all-reduce of a sweep spins like a collective whose peer never arrives (VBFM_FAULT=comm_stall);
  the wait for the stream polls the deadline, releases it, aborts and names the exchange.
"""
import os
import queue
import socket
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "scalable-variational-bayesian-factorization-machine_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(N=16000, F=6, S=250):
    sys.path.insert(0, HERE)
    import synth
    return synth.generate(N, F, S, 5, 1), synth.generate(1500, F, S, 6, 1), F * S


def _subset(csr, lo, hi, nf):
    import vbfm
    rp, f, v, y = csr
    sl = slice(int(rp[lo]), int(rp[hi]))
    return vbfm.DataSubset.from_csr(rp[lo:hi + 1] - rp[lo], f[sl], v[sl], y[lo:hi], nf)


def _fault_worker(rank, world, port, out_q):
    t0 = time.time()
    try:
        sys.path.insert(0, PKG)
        import datetime
        import torch
        import torch.distributed as dist
        import vbfm
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["VBFM_FAULT"] = "comm"
        os.environ["VBFM_FAULT_RANK"] = str(world - 1)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))

        def allreduce(arr, op):
            t = torch.from_numpy(arr.astype(np.float64) if arr.dtype == np.uint32 else arr.copy())
            if arr.dtype == np.uint8:
                t = t.to(torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
            arr[:] = t.numpy().astype(arr.dtype)

        tr, te, nf = _data()
        N, Nt = len(tr[3]), len(te[3])
        fml = vbfm.FMLearnVB(1, 1, 4, nf + 1, min_target=float(tr[3].min()), max_target=float(tr[3].max()),
                             device=0)
        fml.comm_init_host(world, rank, allreduce)
        fml.init(7, 0.1)
        fml.set_data(_subset(tr, rank * N // world, (rank + 1) * N // world, nf),
                     _subset(te, rank * Nt // world, (rank + 1) * Nt // world, nf))
        fml.init_caches()      # the set-up exchanges run (the fault fires inside a sweep only)
        t1 = time.time()
        try:
            fml.iterate()
            out_q.put({"rank": rank, "error": None})
        except vbfm.VbfmError as exc:
            out_q.put({"rank": rank, "error": str(exc), "s": time.time() - t1})
        # the faulting rank leaves here (its connections close); no barrier: a peer is gone
    except BaseException as exc:
        import traceback
        out_q.put({"rank": rank, "error": "unexpected: %r\n%s" % (exc, traceback.format_exc()),
                   "s": time.time() - t0})


def test_host_exchange_rank_fault_fails_the_others():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_fault_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            m = q.get(timeout=180)
            got[m["rank"]] = m
    except queue.Empty:
        pass
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join()
    assert sorted(got) == [0, 1], got
    bad = got[1]["error"]
    assert bad and "VBFM_FAULT=comm" in bad and "rank 1/2" in bad and "level 0" in bad, bad
    other = got[0]["error"]
    # the survivor's exchange failed when the peer left: an error naming it, well before any
    # transport deadline
    assert other and "rank 0/2" in other and "host exchange failed" in other and "sweep" in other, other
    assert got[0]["s"] < 50, got[0]


def test_rccl_setup_deadline_when_peer_never_arrives(monkeypatch):
    sys.path.insert(0, PKG)
    import vbfm
    monkeypatch.setenv("VBFM_COMM_TIMEOUT_S", "4")
    fml = vbfm.FMLearnVB(1, 1, 2, 101, min_target=1.0, max_target=5.0, device=0)
    t0 = time.time()
    with pytest.raises(vbfm.VbfmError) as ei:
        fml.comm_init(2, 0, vbfm.FMLearnVB.comm_unique_id())
    dt = time.time() - t0
    msg = str(ei.value)
    assert "rank 0/2: communicator set-up" in msg and "within 4 s" in msg and "aborted" in msg, msg
    assert 3.5 < dt < 60, dt
    with pytest.raises(vbfm.VbfmError) as e2:     # the context refuses every later exchange
        fml.comm_info()
    assert str(e2.value) == msg
    fml.close()


def test_rccl_stalled_collective_hits_the_deadline(monkeypatch):
    sys.path.insert(0, PKG)
    import vbfm
    for k, v in (("VBFM_FORCE_COMM", "1"), ("VBFM_FORCE_SPLIT", "1"), ("VBFM_COMM_TIMEOUT_S", "3"),
                 ("VBFM_FAULT", "comm_stall"), ("VBFM_FAULT_RANK", "0")):
        monkeypatch.setenv(k, v)
    tr, te, nf = _data(8000)
    fml = vbfm.FMLearnVB(1, 1, 4, nf + 1, min_target=float(tr[3].min()), max_target=float(tr[3].max()), device=0)
    fml.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
    assert fml.comm_info() == (1, 0, "rccl")
    fml.init(7, 0.1)
    fml.set_data(_subset(tr, 0, len(tr[3]), nf), _subset(te, 0, len(te[3]), nf))
    fml.init_caches()
    t0 = time.time()
    with pytest.raises(vbfm.VbfmError) as ei:
        fml.iterate()
    dt = time.time() - t0
    msg = str(ei.value)
    assert "rank 0/1" in msg and "within 3 s" in msg and "aborted" in msg, msg
    assert "the first of them: rank 0/1: w sweep, level 0" in msg, msg
    assert 2.5 < dt < 60, dt
    with pytest.raises(vbfm.VbfmError) as e2:
        fml.iterate()
    assert str(e2.value) == msg
    fml.close()


def test_exchange_info_counts_every_level(monkeypatch):
    """One rank through a real one-rank communicator and the split kernels: every level of the w
    sweep and of each factor's sweep exchanges its statistics once (2 doubles per column), plus
    the data-set sums; the sampled all-reduces carry a time."""
    sys.path.insert(0, PKG)
    import vbfm
    monkeypatch.setenv("VBFM_FORCE_COMM", "1")
    monkeypatch.setenv("VBFM_FORCE_SPLIT", "1")
    tr, te, nf = _data(8000)
    K = 3
    fml = vbfm.FMLearnVB(1, 1, K, nf + 1, min_target=float(tr[3].min()), max_target=float(tr[3].max()), device=0)
    fml.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
    fml.init(7, 0.1)
    fml.set_data(_subset(tr, 0, len(tr[3]), nf), _subset(te, 0, len(te[3]), nf))
    fml.init_caches()
    fml.set_profiling(True, 1)
    fml.iterate()
    x = fml.exchange_info()
    L = fml.levels()[1]
    assert x["transport"] == 1 and x["timeout_s"] == 300.0
    assert x["n_calls"] >= (K + 1) * L
    assert x["bytes"] >= (K + 1) * 16 * nf
    assert x["n_timed"] == x["n_calls"] and x["ms_timed"] > 0 and x["ms_estimated"] == pytest.approx(x["ms_timed"])
    fml.close()


def test_second_communicator_refused(monkeypatch):
    """A context takes one communicator: a second vbfm_comm_init (or one after a host exchange) is
    refused instead of leaking the first."""
    sys.path.insert(0, PKG)
    import vbfm
    monkeypatch.setenv("VBFM_FORCE_COMM", "1")
    fml = vbfm.FMLearnVB(1, 1, 2, 101, min_target=1.0, max_target=5.0, device=0)
    fml.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
    with pytest.raises(vbfm.VbfmError, match="already has a communicator"):
        fml.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
    assert fml.comm_info() == (1, 0, "rccl")
    fml.close()
