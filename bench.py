#!/usr/bin/env python3
"""VB factor-sweep benchmark (BASELINE.json metric) on MI355X.

One step = one full VB iteration of fm_learn_vb_simultaneous (update_all: w0, w sweep,
k factor sweeps, hyper-parameters, free energy; then test prediction + RMSE) on synthetic
field-structured data resident in HBM. value = nnz_train * k * steps / wall time of the
timed steps for the WHOLE data set (all ranks), wall time = max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c3|c2|multihot|tiny]
                    [--scaling strong|weak] [--shard rows|features]

Default workload: BASELINE configs[3] / the metric's "k=100 100M rows": 1e8 rows x 40
one-hot fields x 125000 ids (D = 5e6), nnz = 4e9, k = 100.

Multi-GPU: `--gpus N` with no WORLD_SIZE in the environment starts N rank processes itself
(before this process touches a GPU), each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*;
under torchrun the ranks come from the environment and must equal --gpus. One process per
GPU; the per-level statistics are all-reduced over RCCL (xGMI). --scaling strong (default):
the data set is the config's rows in total, rank r generating rows [r N/P, (r+1) N/P) of it,
so every N describes the same problem. --scaling weak: every rank owns the config's rows
(rows [r N, (r+1) N) of one larger data set). Train, test and every shard share one planted
model (tests/synth.py), so test RMSE falls as the model fits.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd")
sys.path.insert(0, PKG)

METRIC = "factor-sweep throughput (nnz·k/s) + test RMSE at iter parity, k=100 100M rows"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: rows per GPU, fields, ids per field, k
    "c4": dict(rows=100_000_000, fields=40, ids=125_000, k=100,
               desc="C4: 100M rows x 40 one-hot fields (5M features), nnz 4e9, k=100, -method vb"),
    "c3": dict(rows=10_000_000, fields=40, ids=25_000, k=50,
               desc="C3: 10M rows x 40 one-hot fields (1M features), nnz 4e8, k=50, -method vb"),
    # BASELINE configs[1]: MovieLens-1M in libfm format (no network: the ML-1M shape, tests/synth.py
    # generate_movielens -- 6,040 users, 3,952 items with popularity ~ u^3, 900,209 train / 100,000
    # test rows, generated on the host and handed over through vbfm_set_train / vbfm_set_test)
    "c2": dict(rows=900_209, test_rows=100_000, movielens=True, k=20,
               desc="C2: MovieLens-1M-shaped 900,209 train / 100,000 test rows, 6,040 users + 3,952 items "
                    "(item popularity ~u^3), k=20, -method vb"),
    "tiny": dict(rows=200_000, fields=10, ids=2_000, k=8, desc="smoke-sized synthetic"),
    # no field structure: rows of 5..60 distinct ids out of 1e6 (tests/synth.py generate_multihot);
    # the dependency levels miss rows, so the sweeps run on the column-gather layout
    "multihot": dict(rows=10_000_000, features=1_000_000, lo=5, hi=60, k=50,
                     desc="multi-hot: 10M rows x U(5,60) distinct ids of 1M features (no fields), nnz ~3.25e8, "
                          "k=50, -method vb"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu_info():
    """CPU model and the last-level cache one core sees (the sample must not fit in it)."""
    model, llc = "?", None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
        for idx in range(8):
            d = "/sys/devices/system/cpu/cpu0/cache/index%d" % idx
            if not os.path.exists(d):
                break
            if open(d + "/level").read().strip() == "3":
                llc = open(d + "/size").read().strip()
    except OSError:
        pass
    return model, llc


def write_cpu_sample(vbfm, cfg, rows, base, device):
    """Rows [0, rows) of the bench's train set (tests/synth.py, seed 1000, x = 1) generated on
    the device like the bench's own, copied back and written in the reference's binary format
    (<base>.x/.xt/.y, fmatrix.h:46-52), plus a 64-row test set: the reference loads it with its
    own Data::load (Data.h:112-171). C2: the ML-1M-shaped rows themselves (host generator)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    if cfg.get("movielens"):
        nf = synth.ML_USERS + synth.ML_ITEMS
        synth.write_binary(base + "_train", nf, *synth.generate_movielens(rows, 1000))
        synth.write_binary(base + "_test", nf, *synth.generate_movielens(64, 500000))
        return
    F, S = cfg["fields"], cfg["ids"]
    g = vbfm.FMLearnVB(1, 1, 1, F * S + 1, min_target=1.0, max_target=5.0, device=device)
    g.synth(0, rows, F, S, seed=1000, xmode=0)
    cp, ent, y = g.get_csc(0)
    g.close()
    crow, cval = ent["id"], ent["value"]
    del ent
    rp, feat, val = synth.field_csr_from_csc(rows, F, S, cp, crow, cval)
    synth.write_binary_csc(base + "_train", F * S, rp, feat, val, y, cp, crow, cval)
    del rp, feat, val, cp, crow, cval, y
    rpt, ft, vt, yt = synth.generate(64, F, S, 1001, 0)
    synth.write_binary(base + "_test", F * S, rpt, ft, vt, yt)


PROFILER_ENV = ("ROCPROF", "ROCP_", "ROCPROFILER")


def profiler_attached(env=None):
    """True under rocprofv3 (its preloaded library, or its ROCPROF* / ROCP_* variables): a child
    process would start under the profiler's preload, which the GPU pool forbids."""
    env = os.environ if env is None else env
    if "rocprof" in env.get("LD_PRELOAD", ""):
        return True
    return any(k.startswith(PROFILER_ENV) for k in env)


def cpu_leg_plan(rank, world, args, mc, online, multihot, env=None):
    """Whether this rank runs the CPU baseline: rank 0 only, at every N (the north star's
    "alongside ... in the same run" at 1/2/4/8 GPUs), not for MCMC / online / multi-hot (the
    reference sweep timed is fm_learn_vb's), never under a profiler (the child would inherit its
    preload) or with --no-cpu-baseline. Returns (run, reason)."""
    if args.no_cpu_baseline:
        return False, "--no-cpu-baseline"
    if mc or online or multihot:
        return False, "the CPU leg times fm_learn_vb's sweep on field-structured data"
    if profiler_attached(env):
        return False, "skipped under a profiler (its preloaded library would be inherited by the reference)"
    return rank == 0, "rank 0 of %d" % world


def cpu_leg_core():
    """The host core the reference's sweep runs on: the last core this process may use. Every
    rank keeps its own threads off it (pin_away_from), so the CPU leg and the GPU-driving
    threads do not share a core."""
    try:
        return max(os.sched_getaffinity(0))
    except (AttributeError, OSError, ValueError):
        return None


def pin_away_from(core):
    """Move every thread of this process off `core` (no-op when it is the only core allowed)."""
    if core is None:
        return
    try:
        allowed = os.sched_getaffinity(0) - {core}
        if not allowed:
            return
        for tid in os.listdir("/proc/self/task"):
            try:
                os.sched_setaffinity(int(tid), allowed)
            except OSError:
                pass
    except (AttributeError, OSError):
        pass


def ref_sweep(base, factors, core=None):
    """The reference's own factor sweep (oracle/_ref/ref_driver sweep: fm_learn_vb.h:409-440,
    add_main_q + update_v over all features, plus the k = 0 overhead update_w0 + the w sweep)
    on one core: the child pins itself (sched_setaffinity before exec: no launcher process) and
    starts without any profiler preload in its environment."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    env = {k: v for k, v in os.environ.items() if k != "LD_PRELOAD" and not k.startswith(PROFILER_ENV)}
    pre = (lambda: os.sched_setaffinity(0, {core})) if core is not None else None
    out = subprocess.run([ref, "sweep", "--train", base + "_train", "--test", base + "_test",
                          "--dim", "1,1,%d" % factors, "--seed", "1", "--sweep_factors", str(factors)],
                         cwd=os.path.dirname(base), capture_output=True, text=True, check=True, timeout=1200,
                         env=env, preexec_fn=pre).stdout
    return json.loads([l for l in out.splitlines() if l.startswith("{")][0])


def cpu_baseline_start(vbfm, cfg, device, samples, core=None, world=1):
    """Write the samples (device generator, before the timed region) and start the reference's
    sweep on them in a background thread, so that the CPU leg runs while the GPU steps are
    timed (one host core; the GPU bench thread uses another). samples: [(rows, factors), ...],
    the last one reported as `value` -- large enough that its row caches (40 B per row) and
    per-entry streams exceed the host's last-level cache, as C4's do -- the others beside it.
    Returns a function that waits and returns the cpu_baseline object."""
    import threading
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if not os.path.exists(ref):
        return lambda: cpu_baseline_port(cfg, min(samples[0][0], 2_000_000), samples[0][1])
    tmp = tempfile.mkdtemp(prefix="vbfm_cpu_", dir=os.environ.get("TMPDIR"))
    bases = []
    for i, (rows, _) in enumerate(samples):
        b = os.path.join(tmp, "s%d" % i)
        write_cpu_sample(vbfm, cfg, rows, b, device)
        bases.append(b)
    res = {}

    def work():
        try:
            res["runs"] = [ref_sweep(b, f, core) for b, (_, f) in zip(bases, samples)]
        except Exception as exc:   # the GPU number stands on its own; report why the CPU leg failed
            res["error"] = str(exc)
        finally:
            subprocess.run(["rm", "-rf", tmp])

    th = threading.Thread(target=work, daemon=True)
    th.start()

    def finish():
        th.join()
        if "error" in res:
            return {"value": None, "error": res["error"]}
        model, llc = host_cpu_info()
        F, S = (2, 0) if cfg.get("movielens") else (cfg["fields"], cfg["ids"])
        out = []
        for (rows, f), r in zip(samples, res["runs"]):
            o = {"rows": rows, "factors": f, "nnz": r["nnz"], "value": r["nnz_k_per_s"], "seconds": r["sweep_s"],
                 "k0_seconds": r.get("k0_s"), "row_cache_bytes": 40 * rows}
            o.update(extrapolate_iteration(cfg, rows, f, r["sweep_s"], r.get("k0_s")))
            out.append(o)
        big = out[-1]
        return {"value": big["value"], "unit": "nnz*k/s", "cores": 1, "kind": "reference",
                "sample": "%d rows x %d fields x %d ids (D=%d), %d factor(s) of the sweep, x=1 (rows 0.. of the "
                          "bench's data set%s); oracle/_ref/ref_driver = the "
                          "reference's fm_learn_vb compiled from its "
                          "sources, pinned to host core %s (1 of %d host cores: %s, last-level cache %s per core "
                          "complex; the sample's row caches alone are %.1f GB); run by rank 0 of %d during the timed "
                          "GPU steps, every rank's threads kept off that core" % (
                              big["rows"], F, S, F * S or 6040 + 3952, big["factors"],
                              "; S = 0: the ML-1M shape, users + items" if cfg.get("movielens") else "",
                              core, os.cpu_count(), model, llc,
                              big["row_cache_bytes"] / 1e9, world),
                "seconds": big["seconds"], "k0_seconds": big["k0_seconds"],
                "extrapolated_iteration_s": big.get("extrapolated_iteration_s"),
                "extrapolation": big.get("extrapolation"), "cpu_model": model, "llc": llc,
                "samples": out}

    return finish


def cpu_baseline_port(cfg, sample_rows, sample_factors, seed=1):
    """No reference build on this host: time the oracle restatement (bit-exact port) instead."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    import oracle_ctypes as oc
    if cfg.get("movielens"):
        F, S, D = 2, 0, synth.ML_USERS + synth.ML_ITEMS + 1
        rp, f, v, y = synth.generate_movielens(sample_rows, seed)
    else:
        F, S = cfg["fields"], cfg["ids"]
        D = F * S + 1
        rp, f, v, y = synth.generate(sample_rows, F, S, seed, 0)
    tr = oc.Data(csr=(sample_rows, rp, f, v, y))
    vb = oc.VB(1, 1, sample_factors, D)
    vb.init_params(1, 0.1)
    vb.attach(tr, tr)
    vb.init_caches()
    t0 = time.perf_counter()
    for fk in range(sample_factors):
        vb.step("add_main_q", fk)
        vb.step("update_v_all", fk)
    dt = time.perf_counter() - t0
    return {"value": len(f) * sample_factors / dt, "unit": "nnz*k/s", "cores": 1, "kind": "port",
            "sample": "%d rows x %d fields x %d ids, %d factors; oracle/liboracle.so (C restatement, single thread)"
                      % (sample_rows, F, S, sample_factors), "seconds": dt}


def extrapolate_iteration(cfg, sample_rows, sample_factors, sweep_s, k0_s):
    """one reference iteration of the full configuration, extrapolated linearly
    from the timed sample -- the k = 0 overhead (update_w0 + the w sweep) plus k factors of the
    sweep, both scaled by rows (the per-row work is the same at every row count)."""
    if k0_s is None or sweep_s <= 0:
        return {}
    scale = cfg["rows"] / float(sample_rows)
    it = scale * (k0_s + sweep_s / sample_factors * cfg["k"])
    return {"extrapolated_iteration_s": it,
            "extrapolation": "extrapolated: (k0 + %d x one factor) x %d/%d rows" % (
                cfg["k"], cfg["rows"], sample_rows)}


def shard_plan(rows, world, rank, mode):
    """This rank's slice of the data set: strong = `rows` in total split into contiguous
    near-equal slices, weak = `rows` per rank, features = every rank all rows."""
    if mode == "features" or world == 1:
        return {"rows": rows, "row_offset": 0, "rows_total": rows}
    if mode == "weak":
        return {"rows": rows, "row_offset": rank * rows, "rows_total": rows * world}
    lo, hi = rows * rank // world, rows * (rank + 1) // world
    return {"rows": hi - lo, "row_offset": lo, "rows_total": rows}


def launch_event_stride(levels, k, samples=500):
    """Time every stride-th level launch, about `samples` launches per iteration: the smallest
    stride >= launches / samples that is coprime with the level count (every level sampled
    alike). An event pair opens a gap of ~5 us of device time between two launches (kernel
    trace of the multi-hot bench, profiles/r05_multihot/events/): timing every 16th of its 39,250
    launches per iteration cost 59 ms of a 644-ms iteration, every 79th costs ~0.1 %."""
    stride = max(1, -(-levels * k // samples))
    while math.gcd(stride, levels) != 1:
        stride += 1
    return stride


def spawn_ranks(n, grace_s=10.0):
    """Start n rank processes of this script (one per GPU) and watch them. This process never
    touches a GPU; each child gets the torchrun environment and a process group of its own. The
    first rank that exits non-zero stops the run: the others -- which would otherwise wait in a
    collective for it until the deadline -- get SIGTERM (their whole group: the CPU leg's
    reference process with them), SIGKILL after grace_s, and that rank's status is returned."""
    import signal
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    failed = None
    while failed is None:
        codes = [p.poll() for p in procs]
        failed = next(((r, c) for r, c in enumerate(codes) if c not in (None, 0)), None)
        if failed is None and all(c == 0 for c in codes):
            return 0
        if failed is None:
            time.sleep(0.1)
    rank, code = failed
    log("bench.py: rank %d of %d exited with status %d; stopping the other ranks" % (rank, n, code))

    def signal_all(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except OSError:
                    pass

    signal_all(signal.SIGTERM)
    end = time.time() + grace_s
    while time.time() < end and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    signal_all(signal.SIGKILL)
    for p in procs:
        p.wait()
    log("bench.py: rank exit codes %s" % [p.returncode for p in procs])
    return code if code > 0 else 128 - code     # a signal -s as the shell reports it (128 + s)


def bench_fault_hook(rank):
    """Test hook (tests/test_bench_cpu.py): VBFM_BENCH_FAULT=exit:R makes rank R exit with status
    3 at start while every other rank hangs (sleeps) as it would in a collective waiting for R."""
    spec = os.environ.get("VBFM_BENCH_FAULT", "")
    if not spec.startswith("exit:"):
        return
    if rank == int(spec.split(":", 1)[1]):
        log("rank %d: VBFM_BENCH_FAULT: exiting with status 3" % rank)
        sys.exit(3)
    time.sleep(600)


def host_allreduce(arr, op):
    """The host transport's exchange (vbfm_comm_init_host): reduce the staged buffer in place over
    the ranks with a gloo all_reduce -- fp64 sums, uint32 level maxima (through fp64: exact below
    2^53), uint8 flags (through int32)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(arr.astype(np.float64) if arr.dtype == np.uint32 else arr.copy())
    if arr.dtype == np.uint8:
        t = t.to(torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    arr[:] = t.numpy().astype(arr.dtype)


def loaded_libs(name):
    """Distinct files named like `name` mapped into this process (one RCCL, not two)."""
    paths = set()
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                p = line.split()[-1]
                if os.path.basename(p).startswith(name):
                    paths.add(os.path.realpath(p))
    except OSError:
        pass
    return sorted(paths)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override rows per GPU")
    ap.add_argument("--k", type=int, default=0, help="override factors")
    ap.add_argument("--ids", type=int, default=0, help="override ids per field (column length = rows / ids)")
    ap.add_argument("--method", default="vb", choices=["vb", "mcmc", "als", "vb_online"],
                    help="vb: the metric (fm_learn_vb); mcmc / als: config 5's Gibbs draw_v path "
                         "(device counter-based RNG streams); vb_online: OVBFM epochs of --batch "
                         "mini-batches (one GPU); all reported in the same unit")
    ap.add_argument("--batch", type=int, default=50, help="vb_online: mini-batches per epoch (-batch)")
    ap.add_argument("--shard", default="rows", choices=["rows", "features"],
                    help="rows: exact row shards, each rank its own rows (weak scaling, default); "
                         "features: the north star's column partition, every rank all rows (strong "
                         "scaling, Jacobi across shards)")
    ap.add_argument("--layout", default="auto", choices=["auto", "column", "level", "entry"],
                    help="row-cache layout of the sweeps (include/vbfm.h VBFM_LAYOUT_*)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="row shards: strong = the config's rows in total (default), weak = per rank")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="rank exchange: rccl (one GPU per rank, xGMI) or host (every all-reduce staged "
                         "through host memory and a gloo all_reduce: a rehearsal of N ranks on fewer GPUs)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's launch and shard plan as JSON and exit (no GPU)")
    ap.add_argument("--no-launch-events", action="store_true",
                    help="no HIP event pair around every level launch (the roofline then divides the "
                         "sweep phase by the launch count: gaps between launches included)")
    ap.add_argument("--one-rank-comm", action="store_true",
                    help="one GPU through a real 1-rank RCCL communicator and the row-shard (split) kernels "
                         "(VBFM_FORCE_SPLIT / VBFM_FORCE_COMM): the per-rank path of an N-GPU run, minus the "
                         "other ranks -- for A/B of the per-level exchange on one GPU")
    ap.add_argument("--host-upload", action="store_true",
                    help="hand the train set over from host memory (vbfm_set_train: the copy to the device and "
                         "the device's CSR build, the drop-in CLI's path) instead of generating it in HBM; the "
                         "data is the same (generated on the device by a scratch context and copied back first)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=20_000_000,
                    help="rows of the CPU baseline's sample (reported); a 2e6-row, 2-factor sample runs beside it")
    ap.add_argument("--cpu-factors", type=int, default=0,
                    help="factors of the CPU sample's sweep (default 1; C2: all k, the whole sweep of ~2 s)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    # stdout carries the JSON line only: native libraries write to fd 1 (RCCL prints a version
    # banner when a communicator is created), so fd 1 goes to stderr for the whole run (each rank
    # process does this itself: the launcher above hands its own stdout down) and the
    # line is written to a saved copy of the real stdout
    out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    bench_fault_hook(rank)
    if args.one_rank_comm:   # read by vbfm_create / vbfm_comm_init
        if world != 1:
            raise SystemExit("--one-rank-comm is a one-rank mode")
        os.environ["VBFM_FORCE_SPLIT"] = "1"
        os.environ["VBFM_FORCE_COMM"] = "1"
    cfg = dict(CONFIGS[args.config])
    if args.rows:
        cfg["rows"] = args.rows
    if args.k:
        cfg["k"] = args.k
    if args.ids:
        cfg["ids"] = args.ids
    k = cfg["k"]
    multihot = "features" in cfg
    movielens = cfg.get("movielens", False)
    F, S = (0, 0) if multihot else (2, 0) if movielens else (cfg["fields"], cfg["ids"])
    NF = cfg["features"] if multihot else 6040 + 3952 if movielens else F * S       # train features
    D = NF + 1
    fshard = args.shard == "features"
    plan = shard_plan(cfg["rows"], world, rank, "features" if fshard else args.scaling)
    N, row0, n_total = plan["rows"], plan["row_offset"], plan["rows_total"]
    tplan = shard_plan(cfg.get("test_rows", max(cfg["rows"] // 100, 1000)), world, rank,
                       "features" if fshard else args.scaling)
    n_test, trow0 = tplan["rows"], tplan["row_offset"]
    if args.dry_run:
        out.write(json.dumps({"rank": rank, "local_rank": local_rank, "world_size": world,
                          "master": "%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")),
                          "train": plan, "test": tplan, "config": args.config, "k": k}) + "\n")
        out.flush()
        return

    import numpy as np
    import torch
    import torch.distributed as dist
    import vbfm

    # the library's deadline for a collective (VBFM_COMM_TIMEOUT_S, include/vbfm.h; 300 s by default):
    # the bench gives it 900 s, since rank 0 writes the CPU leg's sample files while the other ranks
    # already wait in the first iteration's exchanges; the gloo barriers get at least as long. A
    # rank that dies is caught sooner by the launcher (spawn_ranks) or torchrun
    os.environ.setdefault("VBFM_COMM_TIMEOUT_S", "900")
    comm_timeout_s = float(os.environ["VBFM_COMM_TIMEOUT_S"])
    if world > 1:
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=max(comm_timeout_s, 1800.0)))
    ndev = torch.cuda.device_count()
    device = local_rank % max(1, ndev)      # one rank per GPU; a rehearsal with more ranks than GPUs shares them
    torch.cuda.set_device(device)

    t0 = time.time()
    upload_s = None
    online = args.method == "vb_online"
    mc = args.method in ("mcmc", "als")
    if online:
        if world > 1:
            raise SystemExit("vb_online runs on one GPU")
        fml = vbfm.FMLearnVBOnline(1, 1, k, D, min_target=1.0, max_target=5.0, device=device)
    elif mc:
        fml = vbfm.FMLearnMCMC(1, 1, k, D, min_target=1.0, max_target=5.0, device=device, method=args.method,
                               layout=args.layout)
    else:
        fml = vbfm.FMLearnVB(1, 1, k, D, min_target=1.0, max_target=5.0, device=device, layout=args.layout)
    if fshard:
        if mc:
            raise SystemExit("--shard features is a VB mode")
        fml.set_shard_mode("features")
    if args.one_rank_comm:
        fml.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
    if world > 1 and args.transport == "host":
        fml.comm_init_host(world, rank, host_allreduce)
    elif world > 1:
        obj = [vbfm.FMLearnVB.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        fml.comm_init(world, rank, obj[0])
    if not online:
        fml.init_device(42)
    # one data set, one planted model (tests/synth.py): this rank's slice of the train and
    # test rows; feature shards hold every row
    if movielens:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import synth
        fml.set_data(vbfm.DataSubset.from_csr(*synth.generate_movielens(N, 1000, row_offset=row0), NF),
                     vbfm.DataSubset.from_csr(*synth.generate_movielens(n_test, 500000, row_offset=trow0), NF))
    elif multihot:
        fml.synth_multihot(0, N, NF, cfg["lo"], cfg["hi"], seed=1000, xmode=0, row_offset=row0)
        fml.synth_multihot(1, n_test, NF, cfg["lo"], cfg["hi"], seed=500000, xmode=0, row_offset=trow0)
    elif args.host_upload:
        # the same rows, copied to host memory by a scratch context, then handed over as a caller's
        # host buffers (vbfm_set_train): at C4 nnz = 4e9 > 2^32 entries through the upload path
        scratch = vbfm.FMLearnVB(1, 1, 1, D, min_target=1.0, max_target=5.0, device=device, place_candidates=1)
        scratch.synth(0, N, F, S, seed=1000, xmode=0, row_offset=row0)
        cp, ent, y = scratch.get_csc(0)
        scratch.close()
        host_train = vbfm.DataSubset(cp, ent, y, num_feature=NF)
        del cp, ent, y
        t_up = time.time()
        fml.set_train(host_train)
        upload_s = time.time() - t_up
        del host_train
        fml.synth(1, n_test, F, S, seed=500000, xmode=0, row_offset=trow0)
    else:
        fml.synth(0, N, F, S, seed=1000, xmode=0, row_offset=row0)
        fml.synth(1, n_test, F, S, seed=500000, xmode=0, row_offset=trow0)
    if online:
        # the reference's initial draws generated on the device, the rand() stream continued
        # into the epoch shuffles (vbfm_online_init, VBFM_ONLINE_INIT_REPLAY)
        fml.init(42, 0.1, args.batch, replay=True)
    else:
        fml.init_caches()
    launch_events = not online and not args.no_launch_events
    if launch_events:   # per-launch event pairs: the online epoch has num_batch * k * levels launches
        # an event pair costs ~5 us of device time, so time a sample of ~500 launches per
        # iteration -- every stride-th launch, stride coprime with the level count so that every
        # level is sampled alike
        fml.set_profiling(True, launch_event_stride(fml.levels()[1], k))
    layout = fml.layout()
    nnz = fml.shape(0)[2]                # this rank's train entries
    setup_s = time.time() - t0
    setup = fml.setup_info()             # the library's own split of it (vbfm_setup_info)
    log("rank %d: setup %.1f s (N=%d F=%d S=%d features=%d nnz=%d k=%d, %s layout; train set %.2f s, "
        "schedule %.2f s, store %.2f s incl. placement %.2f s over %d buffers)" % (
            rank, setup_s, N, F, S, NF, nnz, k, layout, setup["s_set_train"], setup["s_schedule"],
            setup["s_store"], setup["s_placement"], setup["place_candidates"]))

    cpu_leg = None
    run_leg, leg_reason = cpu_leg_plan(rank, world, args, mc, online, multihot)
    leg_any = cpu_leg_plan(0, world, args, mc, online, multihot)[0]   # some rank runs it
    core = cpu_leg_core() if leg_any else None
    if leg_any:
        pin_away_from(core)     # every rank: the GPU-driving threads leave the CPU leg's core
    if run_leg:
        try:   # the samples written now (device generator); the reference runs during the timed steps
            rows = min(args.cpu_rows, n_total)   # rows [0, rows) of the whole data set, at any N
            samples = [(min(2_000_000, rows), min(2, k))] if rows > 2_000_000 else []
            cpu_factors = args.cpu_factors or (k if movielens else 1)
            samples.append((rows, min(cpu_factors, k)))
            cpu_leg = cpu_baseline_start(vbfm, cfg, device, samples, core=core, world=world)
        except Exception as exc:
            cpu_leg = (lambda e=str(exc): {"value": None, "error": e})
    elif rank == 0:
        cpu_leg = (lambda r=leg_reason: {"value": None, "skipped": r})

    def rmse_of(st):
        return st.rmse_all if mc else st.rmse

    n_ranks_seen, _, transport = fml.comm_info()
    if n_ranks_seen != args.gpus:   # every rank must have joined the one communicator
        raise SystemExit("bench.py: rank %d sees %d rank(s) in its communicator (%s), --gpus %d" % (
            rank, n_ranks_seen, transport, args.gpus))
    place_ms, place_kept = fml.placement()
    rccl_libs = loaded_libs("librccl")
    if len(rccl_libs) > 1:
        raise SystemExit("more than one RCCL loaded: %s" % rccl_libs)
    rmse_trace = []
    for i in range(args.warmup):
        st = fml.iterate()
        rmse_trace.append(rmse_of(st))
        log("warmup %d: %.1f ms rmse %.6f" % (i, st.ms_total, rmse_of(st)))

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t_start = time.perf_counter()
    stats = []
    xstats = []
    for i in range(args.steps):
        stats.append(fml.iterate())
        xstats.append(fml.exchange_info())
        st = stats[-1]
        rmse_trace.append(rmse_of(st))
        log("step %d: %.1f ms (v sweep %.1f, w %.1f, hyper %.1f, %s %.1f) rmse %.6f" % (
            i, st.ms_total, st.ms_v, st.ms_w, st.ms_hyper, "predict" if mc or online else "test",
            st.ms_predict if mc or online else st.ms_test, rmse_of(st)))
    barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if fshard or world == 1:
        nnz_total = nnz                  # the whole data set's (all ranks)
    else:
        tn = torch.tensor([float(nnz)], dtype=torch.float64)
        dist.all_reduce(tn)
        nnz_total = int(tn.item())
    value = nnz_total * k * args.steps / elapsed
    levels = stats[-1].num_levels
    # roofline of the dominant kernel (k_level_lord / k_v_level_fused, one launch per factor
    # and level). It does the whole factor sweep of its level (stats, posterior, correction
    # and the q-cache of the next factor), so its algorithmic bytes are SURVEY §8d's
    # per-factor model B = 128 B/nnz + 24 B/row + 32 B/feature, spread over the level
    # launches of a factor: 128 = q-build 8 (CSC) + stats 32 (8 CSC + 24 e,q,tq) +
    # correction 88 (8 CSC + 40 + 40). The same model prices both layouts.
    # MCMC / ALS draw_v (fm_learn_mcmc.h:780-835), SURVEY §8d: per factor
    # B = 72 B/nnz (q-build 8 + stats 8 CSC + 16 e,q + correction 8 CSC + 32 e,q read/write)
    #   + 8 B/row + 16 B/feature
    # OVBFM: the same per-factor model per mini-batch; every batch reads the parameters of the
    # columns it touches (<= all F*S), the level launches are num_batch * k * levels per epoch,
    # timed as the summed factor-sweep phase of the batches
    if launch_events:
        n_launch = sum(s.n_vlevel_launches for s in stats)
        ms_launch = sum(s.ms_vlevel_kernels for s in stats)
    else:   # no event pairs: the sweep phase over its launches (an upper bound: gaps included)
        n_launch = sum(s.n_vlevel_launches if online else s.num_levels * k for s in stats)
        ms_launch = sum(s.ms_v for s in stats)
    avg_ms = ms_launch / max(1, n_launch)
    if online:
        bytes_per_launch = (128.0 * nnz + 24.0 * N + 32.0 * NF * args.batch) / max(1, levels * args.batch)
    elif mc:
        bytes_per_launch = (72.0 * nnz + 8.0 * N + 16.0 * NF) / max(1, levels)
    else:
        bytes_per_launch = (128.0 * nnz + 24.0 * N + 32.0 * NF) / max(1, levels)
    if fshard:
        bytes_per_launch /= world          # each rank sweeps 1/world of every level's columns
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    sweep_ms = sum(s.ms_v for s in stats) / len(stats)
    traffic = None
    if online:
        kernel = "k_ov_lord" if stats[-1].n_lord_batches else "k_ov_v_level"
    elif mc:
        kernel = {"level": "k_mc_level_lord", "entry": "k_mc_level_lord<ENT> (entry store)"}.get(layout, "k_mc_v_level")
    else:
        kernel = {"level": "k_level_lord", "entry": "k_level_lord<ENT> (entry store)"}.get(layout, "k_v_level_fused")
    # row shards (N > 1, or the multi-rank kernels forced on one GPU): a level is the split
    # form -- statistics kernel, RCCL all-reduce, posterior / correction -- and its time (the
    # per-level events bracket all of it) is what avg_launch_ms reports
    split = (world > 1 and not fshard and not online) or os.environ.get("VBFM_FORCE_SPLIT") == "1"
    if split:
        kernel = {"k_level_lord": "k_lord_defer + all-reduce + post (per level)",
                  "k_mc_level_lord": "k_mc_lord_defer + all-reduce + post (per level)",
                  "k_v_level_fused": "k_v_level_stats + all-reduce + k_v_level_correct (per level)",
                  "k_mc_v_level": "k_mc_v_level stats + all-reduce + draw (per level)",
                  "k_level_lord<ENT> (entry store)": "entry store: statistics + all-reduce + move (per level)",
                  "k_mc_level_lord<ENT> (entry store)": "entry store: statistics + all-reduce + draw / move "
                                                        "(per level)"}.get(kernel, kernel)
    tlayout = ("level" if stats[-1].n_lord_batches else "column") if online else layout
    tf = os.path.join(ROOT, "profiles", "traffic_%s_%s%s.json" % (args.config, tlayout,
                                                                   "_" + args.method if mc or online else ""))
    traffic_source = None
    if os.path.exists(tf) and not split:
        # PMC counters cannot be read inside this timed run: the traffic comes from the
        # rocprofv3 --pmc passes of an earlier run of this bench configuration (named here)
        with open(tf) as fh:
            tj = json.load(fh)
        traffic = tj.get("bytes_per_launch")
        traffic_source = "%s (earlier PMC profile: %s)" % (os.path.relpath(tf, ROOT), tj.get("source", "?").split(" (")[0])
    fused_model = None
    if mc and not split:
        # the MCMC level kernel also carries the closing train re-prediction of draw_all
        # (fm_learn_mcmc.h:117-348, a separate pass over every entry in the reference): per factor
        # and entry the CSC entry (8 B) and the row's running sums (16 B read + 16 B write), on top
        # of SURVEY's 72 B/nnz draw_v model -- reported beside `roofline`, which keeps SURVEY's
        # model
        fb = (112.0 * nnz + 8.0 * N + 16.0 * NF) / max(1, levels)
        fa = fb / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        fused_model = {"bytes_per_launch": fb, "achieved": fa, "frac": fa / HBM_PEAK_GBS,
                       "model": "draw_v 72 B/nnz + fused re-prediction 40 B/nnz per factor"}
    result = {
        "metric": METRIC, "value": value, "unit": "nnz*k/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1000.0 / args.steps, "higher_is_better": True,
        "scaling": "strong" if fshard else args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic field-structured one-hot libfm data generated in HBM (tests/synth.py spec: "
                "planted bias + rank-2 interaction shared by train, test and all shards), "
                "device random init of mu (0.1*N(0,1))",
        "config": {"workload": cfg["desc"].replace("-method vb", "-method " + args.method),
                   "rows_total": n_total, "rows_per_gpu": N, "fields": F,
                   "ids_per_field": S, "features": NF, "k": k, "nnz_total": nnz_total, "nnz_per_gpu": nnz,
                   "test_rows_per_gpu": n_test,
                   "levels": levels, "method": args.method,
                   "step": ("one full %s iteration (draw_all + train/test re-prediction, device RNG streams)"
                            % args.method.upper()) if mc else
                           ("one OVBFM epoch (shuffle, regroup into %d mini-batches, per batch: predictions + "
                            "update_all; test RMSE)" % args.batch) if online else
                           "one full VB iteration (update_all + test RMSE)",
                   "parallelism": ("feature-sharded fs%d" if fshard else "row-sharded dp%d") % world,
                   "row_layout": ("level (per mini-batch)" if stats[-1].n_lord_batches else "column") if online
                   else layout},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_source,
                     "kernel": kernel, "avg_launch_ms": avg_ms,
                     "launches": n_launch, "bytes_per_launch": bytes_per_launch},
        "roofline_with_fused_predict": fused_model,
        # the level store's record buffers: probe time of each candidate pair (level 0's pattern,
        # 4 passes), the first allocated first, and the pair kept (VBFM_PLACE)
        "placement": {"buffer_ms": [round(x, 4) for x in place_ms], "kept": place_kept} if place_ms else None,
        # host seconds from the context's creation to the first iteration (device data generation,
        # initial parameters, schedule, row store, placement search), and the library's split of it
        "setup_s": setup_s,
        "train_handover": ("host memory (vbfm_set_train: %.2f s for the copy and the device CSR build of %d entries)"
                           % (upload_s, nnz)) if upload_s is not None else "generated in HBM (vbfm_synth_generate)",
        "setup": {"train_set_s": setup["s_set_train"], "schedule_s": setup["s_schedule"],
                  "store_s": setup["s_store"], "placement_s": setup["s_placement"],
                  "placement_bytes": setup["place_bytes"], "placement_candidates": setup["place_candidates"]},
        "factor_sweep_ms_per_step": sweep_ms,
        "factor_sweep_nnz_k_per_s": nnz_total * k / (sweep_ms * 1e-3),
        "test_rmse": rmse_of(stats[-1]),
        "test_rmse_trace": [round(x, 9) for x in rmse_trace],
        "n_ranks_seen": n_ranks_seen, "transport": transport, "rccl_libs": rccl_libs,
        # this rank's all-reduces per step (vbfm_exchange_info): calls, payload bytes, and their
        # time -- RCCL: event pairs around the sampled ones (launch-event stride), scaled to all
        # calls, the wait for the slowest rank included; host exchange: every call's wall time
        "ms_exchange": sum(x["ms_estimated"] for x in xstats) / len(xstats),
        "exchange_bytes": sum(x["bytes"] for x in xstats) // len(xstats),
        "exchange": {"calls_per_step": sum(x["n_calls"] for x in xstats) / len(xstats),
                     "timed": sum(x["n_timed"] for x in xstats),
                     "ms_timed": sum(x["ms_timed"] for x in xstats),
                     "timeout_s": xstats[-1]["timeout_s"]} if xstats else None,
        "free_energy": None if mc else stats[-1].free_energy_last if online else stats[-1].free_energy,
        "phase_ms": {kk: getattr(stats[-1], kk) for kk in (
            ("ms_hyper", "ms_w", "ms_v", "ms_predict", "ms_total") if mc else
            ("ms_regroup", "ms_predict", "ms_w0", "ms_w", "ms_v", "ms_hyper", "ms_test", "ms_total") if online else
            ("ms_w0", "ms_w", "ms_qcache_kernels", "ms_v", "ms_hyper", "ms_test", "ms_test_predict",
             "ms_total"))},
        "cpu_baseline": None,
    }
    if movielens:
        # 900k rows x 64 B of records (58 MB) and 1.8e6 entries: the level store sits in the 256 MB
        # MALL (Infinity Cache), so the fraction below is not an HBM measurement
        result["roofline"]["note"] = ("C2's working set (records %.0f MB, entries %.0f MB) is cache-resident: the "
                                      "fraction of 8 TB/s is not an HBM roofline" % (64e-6 * N, 8e-6 * nnz))
    if cpu_leg is not None:
        result["cpu_baseline"] = cpu_leg()
    if rank == 0:   # the line first: nothing in the teardown can cost it
        out.write(json.dumps(result) + "\n")
        out.flush()
    log("rank %d: closing" % rank)
    fml.close()
    log("rank %d: closed" % rank)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
