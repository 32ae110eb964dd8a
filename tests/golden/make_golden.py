#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the COMPILED REFERENCE.

Run in the build container (needs oracle/_ref/ref_driver, built by `make -C oracle ref`
from /root/reference/src; the reference itself never travels). Each case directory holds:

  inputs      train.libfm / test.libfm (+ meta)   -- tiny hand-built cases only; the larger
              cases are regenerated from tests/synth.py or tests/golden/sa_split/*.gz
  trace.json  per-iteration values printed by the reference at 17 significant digits
  arrays.npz  raw fp64 dumps of the reference's state (init draws, caches after each
              step of update_all, parameters per iteration)

Usage: python tests/golden/make_golden.py [--ref oracle/_ref/ref_driver]
"""
import argparse
import ctypes
import gzip
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import synth  # noqa: E402


def run_ref(ref, mode, train, test, dim, iters, seed, extra=(), env_extra=None):
    out = tempfile.mkdtemp(prefix="golden_")
    env = dict(os.environ)
    if env_extra:
        env.update(env_extra)
    if mode == "vb_online":
        # the reference writes <train>batch<j> next to the train file and opens them through a
        # dangling c_str() (fm_learn_vb_online_simultaneous.h:80-82): a private copy under a
        # short (small-string-optimised) name keeps that well defined
        shutil.copy(train, os.path.join(out, "t"))
        train = "t"
    cmd = [ref, mode, "--train", train, "--test", test, "--dim", dim, "--iter", str(iters),
           "--seed", str(seed), "--dump", out] + list(extra)
    res = subprocess.run(cmd, cwd=out, env=env, capture_output=True, text=True, check=True)
    arrays = {}
    for fn in sorted(os.listdir(out)):
        if fn.endswith(".f64"):
            arrays[fn[:-4]] = np.fromfile(os.path.join(out, fn), dtype="<f8")
    vfile = os.path.join(out, "v_file.txt")
    shutil.rmtree(out)
    return res.stdout, arrays


def parse_vb(stdout):
    trace, fe = [], []
    nums = {}
    for line in stdout.splitlines():
        if line.startswith("NUMS "):
            t = line.split()[1:]
            nums = {t[i]: float(t[i + 1]) for i in range(0, len(t), 2)}
        elif line.startswith("free energy "):
            fe.append(float(line.split()[2]))
        elif line.startswith("ITER_BEGIN"):
            fe_marker = len(fe)
            trace.append({"_fe_before": fe_marker})
        elif line.startswith("ITER "):
            t = line.split()
            d = {t[i]: float(t[i + 1]) for i in range(2, len(t), 2)}
            d["iter"] = int(t[1])
            rec = trace[-1]
            d["free_energy"] = fe[rec["_fe_before"]] if len(fe) > rec["_fe_before"] else None
            trace[-1] = d
    return nums, trace


def parse_mcmc(stdout):
    nums, trace = {}, []
    for line in stdout.splitlines():
        if line.startswith("NUMS "):
            t = line.split()[1:]
            nums = {t[i]: float(t[i + 1]) for i in range(0, len(t), 2)}
        m = re.match(r"#Iter=\s*(\d+)\s+Train=(\S+)\s+Test=(\S+)", line)
        if m:
            trace.append({"iter": int(m.group(1)), "train": float(m.group(2)),
                          "rmse_all": float(m.group(3))})
    return nums, trace


def parse_online(stdout):
    nums, trace, fe = {}, [], []
    for line in stdout.splitlines():
        if line.startswith("NUMS "):
            t = line.split()[1:]
            nums = {t[i]: float(t[i + 1]) for i in range(0, len(t), 2)}
        elif line.startswith("free energy "):
            fe.append(float(line.split()[2]))
        m = re.match(r"#Iter=\s*(\d+)\s+Test=(\S+)", line)
        if m:
            trace.append({"iter": int(m.group(1)), "rmse": float(m.group(2)), "free_energy": fe})
            fe = []
    return nums, trace


def online_cases(ref):
    """-method vb_online (OVBFM): fm_learn_vb_online_simultaneous.h, run by the reference itself."""
    keep = ("final_", "init_mu", "init_nat", "init_fm_v")
    for case in ("tiny", "tiny_dup"):
        d = os.path.join(HERE, case)
        tr, te = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
        for nb, it in ((3, 4), (5, 3), (1, 2)):
            out, arr = run_ref(ref, "vb_online", tr, te, "1,1,3", it, 5, extra=["--batch", str(nb)])
            nums, trace = parse_online(out)
            save_case("%s/online_b%d" % (case, nb), nums, trace, {k: arr[k] for k in arr if k.startswith(keep)},
                      {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1, "iter": it, "batch": nb})
    d = os.path.join(HERE, "tiny")
    tr, te, meta = (os.path.join(d, n) for n in ("train.libfm", "test.libfm", "groups.meta"))
    out, arr = run_ref(ref, "vb_online", tr, te, "0,1,2", 3, 11,
                       extra=["--meta", meta, "--init_stdev", "0.2", "--batch", "4"])
    nums, trace = parse_online(out)
    save_case("tiny/online_meta", nums, trace, {k: arr[k] for k in arr if k.startswith(keep)},
              {"dim": "0,1,2", "seed": 11, "init_stdev": 0.2, "iter": 3, "batch": 4, "meta": "groups.meta"})
    tmp = tempfile.mkdtemp()
    spec = {"n_rows": 20000, "n_fields": 10, "ids_per_field": 200, "seed": 7, "xmode": 1,
            "test_rows": 2000, "test_seed": 8}
    rp, f, v, y = synth.generate(spec["n_rows"], spec["n_fields"], spec["ids_per_field"], spec["seed"], 1)
    synth.write_libfm(os.path.join(tmp, "tr.libfm"), rp, f, v, y)
    rp, f, v, y = synth.generate(spec["test_rows"], spec["n_fields"], spec["ids_per_field"], spec["test_seed"], 1)
    synth.write_libfm(os.path.join(tmp, "te.libfm"), rp, f, v, y)
    out, arr = run_ref(ref, "vb_online", os.path.join(tmp, "tr.libfm"), os.path.join(tmp, "te.libfm"), "1,1,4", 3, 7)
    nums, trace = parse_online(out)
    save_case("synth_online", nums, trace, {k: arr[k] for k in arr if k.startswith("final_scalars")},
              dict(spec, dim="1,1,4", init_stdev=0.1, iter=3, batch=50,
                   array_sums={k: [float(np.sum(arr[k])), float(np.sum(arr[k] ** 2))] for k in arr}))
    shutil.rmtree(tmp)
    sa = os.path.join(HERE, "sa_split")
    tmp = tempfile.mkdtemp()
    for part in ("train", "test"):
        with gzip.open(os.path.join(sa, part + ".libfm.gz"), "rt") as fi, \
                open(os.path.join(tmp, part + ".libfm"), "w") as fo:
            fo.write(fi.read())
    out, arr = run_ref(ref, "vb_online", os.path.join(tmp, "train.libfm"), os.path.join(tmp, "test.libfm"),
                       "1,1,8", 5, 42)
    nums, trace = parse_online(out)
    save_case("sa_online", nums, trace, {k: arr[k] for k in arr if k.startswith("final_scalars")},
              {"dim": "1,1,8", "seed": 42, "init_stdev": 0.1, "iter": 5, "batch": 50,
               "array_sums": {k: [float(np.sum(arr[k])), float(np.sum(arr[k] ** 2))] for k in arr}})
    shutil.rmtree(tmp)


def levels_cases(ref):
    """update_all's sweeps one dependency level at a time (ref_driver levels): caches and
    parameters after every level of the w sweep and of every factor's v sweep."""
    for case in ("tiny", "tiny_dup"):
        d = os.path.join(HERE, case)
        tr, te = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
        out, arr = run_ref(ref, "levels", tr, te, "1,1,3", 1, 5)
        nums, _ = parse_vb(out)
        L = int(re.search(r"^LEVELS (\d+)$", out, re.M).group(1))
        keep = {k: arr[k] for k in arr if k.startswith("l_") or k == "levels" or k.startswith("init_")}
        save_case(case + "/levels", nums, [], keep, {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1, "num_levels": L})


def save_case(name, nums, trace, arrays, meta):
    d = os.path.join(HERE, name)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "trace.json"), "w") as fh:
        json.dump({"nums": nums, "trace": trace, "meta": meta}, fh, indent=1)
    if arrays:
        np.savez_compressed(os.path.join(d, "arrays.npz"), **arrays)


def tiny_dataset(path_train, path_test, dup=False):
    """3 fields (ids 0-3, 4-6, 7-11), non-unit x, feature 10 never in train, feature 12 only
    in test (so D = nf_test + 1 > nf_train + 1), one train row without features, rows
    listing their ids out of order."""
    rng = np.random.RandomState(1234)
    fields = [(0, 4), (4, 3), (7, 5)]

    def rows(n, allow):
        out = []
        for r in range(n):
            ents = []
            for (b, s) in fields:
                j = b + rng.randint(s)
                if not allow and j == 10:
                    j = 9
                ents.append((j, np.float32(rng.uniform(0.25, 1.75) * (1 if rng.rand() > .15 else -1))))
            if r % 5 == 3:
                ents = ents[::-1]            # ids out of ascending order within the row
            y = float(rng.randint(1, 6))
            out.append((y, ents))
        return out

    tr = rows(24, allow=False)
    tr[7] = (tr[7][0], [])                   # a row with no features
    if dup:
        y, ents = tr[11]
        tr[11] = (y, ents + [(ents[0][0], np.float32(0.625))])   # duplicated id in one row
    te = rows(8, allow=True)
    te[2] = (te[2][0], te[2][1] + [(12, np.float32(0.875))])
    for path, data in ((path_train, tr), (path_test, te)):
        with open(path, "w") as fh:
            for y, ents in data:
                fh.write(" ".join(["%g" % y] + ["%d:%.9g" % (j, float(x)) for j, x in ents]) + "\n")


def mcmc_cases(ref):
    """-method mcmc / als traces and final states (fm_learn_mcmc_simultaneous.h)."""
    for case in ("tiny", "tiny_dup"):
        d = os.path.join(HERE, case)
        tr, te = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
        out, arr = run_ref(ref, "mcmc", tr, te, "1,1,3", 6, 5)
        nums, trace = parse_mcmc(out)
        save_case(case + "/mcmc", nums, trace, arr, {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1, "iter": 6})
    d = os.path.join(HERE, "tiny")
    tr, te, meta = (os.path.join(d, n) for n in ("train.libfm", "test.libfm", "groups.meta"))
    out, arr = run_ref(ref, "mcmc", tr, te, "1,1,2", 5, 11, extra=["--meta", meta, "--init_stdev", "0.2"])
    nums, trace = parse_mcmc(out)
    save_case("tiny/mcmc_meta", nums, trace, arr,
              {"dim": "1,1,2", "seed": 11, "init_stdev": 0.2, "iter": 5, "meta": "groups.meta"})
    for case in ("tiny", "tiny_dup"):
        dc = os.path.join(HERE, case)
        out, arr = run_ref(ref, "als", os.path.join(dc, "train.libfm"), os.path.join(dc, "test.libfm"), "1,1,3", 6, 5,
                           extra=["--regular", "0.5,1,2"])
        nums, trace = parse_mcmc(out)
        save_case(case + "/als_reg", nums, trace, arr,
                  {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1, "iter": 6, "regular": [0.5, 1.0, 2.0]})
    reg = [0.25, 0.5, 1.0, 2.0, 0.75, 1.5, 3.0]
    out, arr = run_ref(ref, "als", tr, te, "0,1,2", 5, 11,
                       extra=["--meta", meta, "--regular", ",".join(str(r) for r in reg)])
    nums, trace = parse_mcmc(out)
    save_case("tiny/als_meta_reg", nums, trace, arr,
              {"dim": "0,1,2", "seed": 11, "init_stdev": 0.1, "iter": 5, "meta": "groups.meta", "regular": reg})
    tmp = tempfile.mkdtemp()
    spec = {"n_rows": 20000, "n_fields": 10, "ids_per_field": 200, "seed": 7, "xmode": 1,
            "test_rows": 2000, "test_seed": 8}
    rp, f, v, y = synth.generate(spec["n_rows"], spec["n_fields"], spec["ids_per_field"], spec["seed"], 1)
    synth.write_libfm(os.path.join(tmp, "tr.libfm"), rp, f, v, y)
    rp, f, v, y = synth.generate(spec["test_rows"], spec["n_fields"], spec["ids_per_field"], spec["test_seed"], 1)
    synth.write_libfm(os.path.join(tmp, "te.libfm"), rp, f, v, y)
    out, arr = run_ref(ref, "mcmc", os.path.join(tmp, "tr.libfm"), os.path.join(tmp, "te.libfm"), "1,1,4", 5, 7)
    nums, trace = parse_mcmc(out)
    save_case("synth_mcmc", nums, trace, {k: arr[k] for k in arr if k.startswith("final")},
              dict(spec, dim="1,1,4", init_stdev=0.1, iter=5))
    shutil.rmtree(tmp)
    sa = os.path.join(HERE, "sa_split")
    tmp = tempfile.mkdtemp()
    for part in ("train", "test"):
        with gzip.open(os.path.join(sa, part + ".libfm.gz"), "rt") as fi, \
                open(os.path.join(tmp, part + ".libfm"), "w") as fo:
            fo.write(fi.read())
    out, arr = run_ref(ref, "mcmc", os.path.join(tmp, "train.libfm"), os.path.join(tmp, "test.libfm"),
                       "1,1,8", 10, 42)
    nums, trace = parse_mcmc(out)
    save_case("sa_mcmc", nums, trace, {k: arr[k] for k in arr if k.startswith("final_mcmc") or k.endswith("_mu")
                                       or k.endswith("_lambda")},
              {"dim": "1,1,8", "seed": 42, "init_stdev": 0.1, "iter": 10,
               "array_sums": {k: [float(np.sum(arr[k])), float(np.sum(arr[k] ** 2))] for k in arr}})
    shutil.rmtree(tmp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.path.join(HERE, "..", "..", "oracle", "_ref", "ref_driver"))
    ap.add_argument("--only", default="", help="comma list of groups: rng,tiny,meta,synth,sa,mcmc,online,levels")
    args = ap.parse_args()
    ref = os.path.abspath(args.ref)
    only = set(filter(None, args.only.split(",")))

    def want(group):
        return not only or group in only

    if want("levels"):
        levels_cases(ref)
    if want("mcmc"):
        mcmc_cases(ref)
    if want("online"):
        online_cases(ref)
    if only and not only - {"mcmc", "online", "levels"}:
        return

    # --- RNG known answers: glibc rand() as the reference calls it (random.h:174-176)
    libc = ctypes.CDLL(None)
    kat = {}
    for seed in (1, 42, 12345, 0, 2147483647):
        libc.srand(ctypes.c_uint(seed))
        kat[str(seed)] = [int(libc.rand()) for _ in range(40)]
    os.makedirs(os.path.join(HERE, "rng"), exist_ok=True)
    with open(os.path.join(HERE, "rng", "glibc_rand.json"), "w") as fh:
        json.dump(kat, fh, indent=1)

    # --- tiny hand-built cases (inputs committed)
    for case, dup in (("tiny", False), ("tiny_dup", True)):
        d = os.path.join(HERE, case)
        os.makedirs(d, exist_ok=True)
        tr, te = os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm")
        tiny_dataset(tr, te, dup=dup)
        out, arr = run_ref(ref, "steps", tr, te, "1,1,3", 1, 5)
        nums, _ = parse_vb(out)
        save_case(case + "/steps", nums, [], arr, {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1})
        out, arr = run_ref(ref, "vb", tr, te, "1,1,3", 6, 5, env_extra={"REF_DUMP_ITER_PARAMS": "1"})
        nums, trace = parse_vb(out)
        save_case(case + "/vb", nums, trace, arr, {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1, "iter": 6})
        out, arr = run_ref(ref, "als", tr, te, "1,1,3", 6, 5)
        nums, trace = parse_mcmc(out)
        save_case(case + "/als", nums, trace, arr, {"dim": "1,1,3", "seed": 5, "init_stdev": 0.1, "iter": 6})
    # tiny with a -meta group file (one group per field) and k0=0
    d = os.path.join(HERE, "tiny")
    meta = os.path.join(d, "groups.meta")
    with open(meta, "w") as fh:
        for j in range(14):
            fh.write("%d\n" % (0 if j < 4 else (1 if j < 7 else 2)))
    out, arr = run_ref(ref, "vb", os.path.join(d, "train.libfm"), os.path.join(d, "test.libfm"),
                       "0,1,2", 5, 11, extra=["--meta", meta, "--init_stdev", "0.2"],
                       env_extra={"REF_DUMP_ITER_PARAMS": "1"})
    nums, trace = parse_vb(out)
    save_case("tiny/vb_meta", nums, trace, arr,
              {"dim": "0,1,2", "seed": 11, "init_stdev": 0.2, "iter": 5, "meta": "groups.meta"})

    # --- field-structured synthetic, real-valued x (inputs regenerated from tests/synth.py)
    tmp = tempfile.mkdtemp()
    spec = {"n_rows": 20000, "n_fields": 10, "ids_per_field": 200, "seed": 7, "xmode": 1,
            "test_rows": 2000, "test_seed": 8}
    rp, f, v, y = synth.generate(spec["n_rows"], spec["n_fields"], spec["ids_per_field"], spec["seed"], 1)
    synth.write_libfm(os.path.join(tmp, "tr.libfm"), rp, f, v, y)
    rp, f, v, y = synth.generate(spec["test_rows"], spec["n_fields"], spec["ids_per_field"], spec["test_seed"], 1)
    synth.write_libfm(os.path.join(tmp, "te.libfm"), rp, f, v, y)
    out, arr = run_ref(ref, "vb", os.path.join(tmp, "tr.libfm"), os.path.join(tmp, "te.libfm"),
                       "1,1,4", 8, 7)
    nums, trace = parse_vb(out)
    keep = {k: arr[k] for k in arr if k.startswith("final") or k.startswith("init_mu") or k == "init_test_e"
            or k.startswith("init_e") or k.startswith("init_t")}
    save_case("synth", nums, trace, keep, dict(spec, dim="1,1,4", init_stdev=0.1, iter=8))
    out, arr = run_ref(ref, "als", os.path.join(tmp, "tr.libfm"), os.path.join(tmp, "te.libfm"),
                       "1,1,4", 5, 7)
    nums, trace = parse_mcmc(out)
    save_case("synth_als", nums, trace, {k: arr[k] for k in arr if k.startswith("final")},
              dict(spec, dim="1,1,4", init_stdev=0.1, iter=5))
    shutil.rmtree(tmp)

    # --- bundled MovieLens-1M test split: rows 1-90000 train, rest test
    sa = os.path.join(HERE, "sa_split")
    tmp = tempfile.mkdtemp()
    for part in ("train", "test"):
        with gzip.open(os.path.join(sa, part + ".libfm.gz"), "rt") as fi, \
                open(os.path.join(tmp, part + ".libfm"), "w") as fo:
            fo.write(fi.read())
    out, arr = run_ref(ref, "vb", os.path.join(tmp, "train.libfm"), os.path.join(tmp, "test.libfm"),
                       "1,1,8", 20, 42)
    nums, trace = parse_vb(out)
    sums = {k: [float(np.sum(arr[k])), float(np.sum(arr[k] ** 2))] for k in arr}
    save_case("sa_k8", nums, trace, {k: arr[k] for k in ("final_mu_w", "final_scalars", "init_mu_w")},
              {"dim": "1,1,8", "seed": 42, "init_stdev": 0.1, "iter": 20, "array_sums": sums})
    shutil.rmtree(tmp)
    print("golden fixtures written under", HERE)


if __name__ == "__main__":
    main()
