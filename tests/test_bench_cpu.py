"""bench.py's launch contract and its synthetic data (no GPU).

* `--gpus N` without WORLD_SIZE starts N rank processes with the torchrun environment;
* strong scaling slices the config's rows into contiguous shards that cover it exactly;
* every shard and the test set come from one planted model, so a fitted model predicts the
  test set better than the constant predictor (tests/synth.py; the oracle is the learner).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_ctypes as oc
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _dry(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, BENCH, "--dry-run"] + args, env=env, capture_output=True, text=True,
                         timeout=120)
    return out


@pytest.mark.parametrize("n,scaling", [(2, "strong"), (4, "strong"), (3, "weak")])
def test_gpus_flag_spawns_configured_ranks(n, scaling):
    out = _dry(["--gpus", str(n), "--scaling", scaling])
    assert out.returncode == 0, out.stderr
    plans = sorted((json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")), key=lambda p: p["rank"])
    assert [p["rank"] for p in plans] == list(range(n))
    assert all(p["world_size"] == n and p["local_rank"] == p["rank"] for p in plans)
    assert len({p["master"] for p in plans}) == 1 and plans[0]["master"].startswith("127.0.0.1:")
    rows = 100_000_000
    for part, total in (("train", rows), ("test", rows // 100)):
        off = 0
        for p in plans:
            sh = p[part]
            assert sh["row_offset"] == off
            off += sh["rows"]
            assert sh["rows_total"] == (total if scaling == "strong" else total * n)
        assert off == plans[0][part]["rows_total"]


def test_one_gpu_runs_in_process_and_mismatch_fails():
    out = _dry([])
    plans = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(plans) == 1 and plans[0]["world_size"] == 1 and plans[0]["train"]["rows"] == 100_000_000
    bad = _dry(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr


@pytest.mark.parametrize("bad_rank", [0, 2])
def test_dead_rank_stops_the_run(bad_rank):
    """A rank that exits non-zero at start (VBFM_BENCH_FAULT=exit:R) while the others hang, as they
    would in a collective waiting for it: the launcher stops the survivors (SIGTERM to each rank's
    process group) and returns that rank's status within seconds, not at a deadline."""
    import time
    t0 = time.time()
    out = _dry(["--gpus", "4"], {"VBFM_BENCH_FAULT": "exit:%d" % bad_rank})
    dt = time.time() - t0
    assert out.returncode == 3, out.stderr
    assert dt < 30, dt
    assert "rank %d of 4 exited with status 3" % bad_rank in out.stderr
    codes = json.loads(out.stderr.split("rank exit codes ")[1].splitlines()[0])
    assert codes[bad_rank] == 3 and sorted(codes)[:3] == [-15, -15, -15], codes


def test_features_shard_holds_every_row():
    out = _dry(["--gpus", "2", "--shard", "features"])
    for l in out.stdout.splitlines():
        p = json.loads(l)
        assert p["train"] == {"rows": 100_000_000, "row_offset": 0, "rows_total": 100_000_000}


def test_row_shards_are_slices_of_one_data_set():
    n, F, S = 3001, 6, 50
    full = synth.generate(n, F, S, 1000, 1)
    parts = [synth.generate(hi - lo, F, S, 1000, 1, row_offset=lo)
             for lo, hi in ((0, 1000), (1000, 2500), (2500, 3001))]
    np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), full[1])
    np.testing.assert_array_equal(np.concatenate([p[2] for p in parts]), full[2])
    np.testing.assert_array_equal(np.concatenate([p[3] for p in parts]), full[3])


def test_planted_model_is_learnable_on_held_out_rows():
    """The bench's train/test pairing: different row seeds, one model seed. VB (the oracle)
    beats the constant predictor on the test rows and its test RMSE falls over iterations."""
    n, F, S, k = 20000, 8, 100, 4
    rp, f, v, y = synth.generate(n, F, S, 1000, 0)
    rpt, ft, vt, yt = synth.generate(4000, F, S, 500000, 0)
    o = oc.VB(1, 1, k, F * S + 1)
    o.init_params(3, 0.1)
    o.attach(oc.Data(csr=(n, rp, f, v, y)), oc.Data(csr=(4000, rpt, ft, vt, yt)))
    o.init_caches()
    trace = [o.iterate()[0] for _ in range(12)]
    const = float(np.sqrt(np.mean((yt - y.mean()) ** 2)))
    assert trace[-1] < 0.85 * const, (trace, const)
    assert trace[-1] < trace[2] < trace[0]


def test_launch_event_stride_samples_every_level():
    """Level launches are timed on a sample of ~500 per iteration (an event pair costs ~5 us of
    device time): the stride is coprime with the level count, so over k factors every level is
    timed equally often; few launches are all timed."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.launch_event_stride(40, 100) == 9            # C4: 4000 launches, 445 timed
    assert bench.launch_event_stride(785, 50) == 79           # multi-hot: 39,250 launches
    assert bench.launch_event_stride(800, 50) == 81           # 80 shares a factor with 800
    assert bench.launch_event_stride(40, 8) == 1              # few launches: each timed
    for levels, k in ((40, 100), (785, 50), (800, 50), (1024, 10), (255, 64)):
        s = bench.launch_event_stride(levels, k)
        timed = np.zeros(levels, dtype=int)
        for i in range(0, levels * k, s):
            timed[i % levels] += 1
        assert timed.max() - timed.min() <= 1


def test_cpu_baseline_extrapolates_one_iteration():
    """the reference's C4 iteration is extrapolated from the timed sample, the
    k = 0 overhead plus k factors, scaled by rows, and labelled as such."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cfg = dict(bench.CONFIGS["c4"])
    r = bench.extrapolate_iteration(cfg, 2_000_000, 2, sweep_s=4.0, k0_s=0.5)
    assert r["extrapolated_iteration_s"] == pytest.approx(50 * (0.5 + 2.0 * cfg["k"]))
    assert r["extrapolation"].startswith("extrapolated")
    assert bench.extrapolate_iteration(cfg, 2_000_000, 2, sweep_s=4.0, k0_s=None) == {}


def test_cpu_sample_files_and_reference_sweep(tmp_path):
    """The CPU leg's sample in the reference's binary format (sort-free writer, CSR rebuilt from
    the field CSC) is what the reference's own loader reads, and its sweep reports throughput."""
    import os
    import synth
    import bench
    rp, f, v, y = synth.generate(5000, 6, 50, 1000, 0)
    cp, cr, cv = synth.csr_to_csc(5000, 300, rp, f, v)
    rp2, f2, v2 = synth.field_csr_from_csc(5000, 6, 50, cp, cr, cv)
    np.testing.assert_array_equal(f2, f)
    base = str(tmp_path / "s0")
    synth.write_binary_csc(base + "_train", 300, rp2, f2, v2, y, cp, cr, cv)
    synth.write_binary(base + "_ref", 300, rp, f, v, y)
    for ext in (".x", ".xt", ".y"):
        assert open(base + "_train" + ext, "rb").read() == open(base + "_ref" + ext, "rb").read()
    rpt, ft, vt, yt = synth.generate(64, 6, 50, 1001, 0)
    synth.write_binary(base + "_test", 300, rpt, ft, vt, yt)
    model, llc = bench.host_cpu_info()
    assert model
    if not os.path.exists(os.path.join(bench.ROOT, "oracle", "_ref", "ref_driver")):
        pytest.skip("oracle/_ref/ref_driver not built")
    r = bench.ref_sweep(base, 2)
    assert r["nnz"] == 30000 and r["factors"] == 2 and r["nnz_k_per_s"] > 0


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_cpu_leg_runs_on_rank_zero_at_every_n(world):
    """the reference's sweep (the CPU baseline) runs in the same run at
    every N, on rank 0 only; MCMC / online / multi-hot and --no-cpu-baseline skip it, and so does
    a run under a profiler (the reference would inherit its preloaded library)."""
    bench = _bench_module()

    class A:
        no_cpu_baseline = False
    clean = {"PATH": "/usr/bin"}
    runs = [bench.cpu_leg_plan(r, world, A, False, False, False, clean)[0] for r in range(world)]
    assert runs == [True] + [False] * (world - 1)
    for mc, online, multihot in ((True, False, False), (False, True, False), (False, False, True)):
        assert not bench.cpu_leg_plan(0, world, A, mc, online, multihot, clean)[0]
    prof = dict(clean, LD_PRELOAD="/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so")
    run, why = bench.cpu_leg_plan(0, world, A, False, False, False, prof)
    assert not run and "profiler" in why
    assert not bench.cpu_leg_plan(0, world, A, False, False, False, dict(clean, ROCPROF_KERNEL_TRACE="1"))[0]
    A.no_cpu_baseline = True
    assert not bench.cpu_leg_plan(0, world, A, False, False, False, clean)[0]


def test_cpu_leg_core_and_pinning():
    """The CPU leg's core is one this process may use, and pin_away_from leaves every thread
    of the process on the other cores (when there are any)."""
    bench = _bench_module()
    before = os.sched_getaffinity(0)
    core = bench.cpu_leg_core()
    assert core in before
    try:
        bench.pin_away_from(core)
        if len(before) > 1:
            for tid in os.listdir("/proc/self/task"):
                assert core not in os.sched_getaffinity(int(tid))
    finally:
        for tid in os.listdir("/proc/self/task"):
            try:
                os.sched_setaffinity(int(tid), before)
            except OSError:
                pass


def _exchange_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    f = np.array([0.1 * (rank + 1), -2.5, 1e300 / (rank + 1)], dtype=np.float64)
    u = np.array([rank, 7, 4294967295 - rank], dtype=np.uint32)
    b = np.array([rank % 2, 0, 1], dtype=np.uint8)
    bench.host_allreduce(f, "sum")
    bench.host_allreduce(u, "max")
    bench.host_allreduce(b, "max")
    q.put((rank, f.tolist(), u.tolist(), b.tolist()))
    dist.destroy_process_group()


def test_host_exchange_reduces_every_dtype_over_gloo():
    """bench.py's host transport (the exchange behind vbfm_comm_init_host on an N-rank run sharing
    GPUs) over gloo with 3 CPU ranks: fp64 sums, uint32 maxima up to 2^32 - 1, uint8 flags, in place
    and in the caller's dtype."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=30)
    want_f = [0.1 + 0.2 + 0.30000000000000004, -7.5, 1e300 + 1e300 / 2 + 1e300 / 3]
    for rank, f, u, b in got:
        assert abs(f[0] - 0.6) < 1e-15 and f[1] == -7.5 and abs(f[2] - want_f[2]) <= 1e-15 * want_f[2]
        assert u == [2, 7, 4294967295]
        assert b == [1, 0, 1]
