#!/usr/bin/env python3
"""bench.py's C4 VB iteration without importing torch (one GPU, device 0).

Why: with torch imported first, libvbfm.so's NEEDED libamdhip64.so.7 is satisfied by the HIP
runtime torch bundles (torch/lib/libamdhip64.so, ROCm 7.0; same SONAME), while rocprofv3 and its
counter-collection library come from /opt/rocm (7.2). Without torch the process runs the HIP
runtime libvbfm.so was built against (RUNPATH /opt/rocm/lib). Used to rerun the k = 100
`rocprofv3 --pmc` pass that aborted under bench.py (profiles/r03_final/pmc_fetch_3step_segfault.txt,
symbolized in profiles/r04_pmc_segfault/README.md).

usage: python3 tools/pmc_notorch.py [--rows N] [--ids S] [--k K] [--steps K] [--warmup W]
Prints one JSON line: the HIP runtime file mapped into the process and each step's phase times.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd"))


def mapped(name):
    paths = set()
    with open("/proc/self/maps") as fh:
        for line in fh:
            p = line.split()[-1]
            if os.path.basename(p).startswith(name):
                paths.add(os.path.realpath(p))
    return sorted(paths)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--fields", type=int, default=40)
    ap.add_argument("--ids", type=int, default=125_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    import vbfm
    assert "torch" not in sys.modules
    F, S = a.fields, a.ids
    g = vbfm.FMLearnVB(1, 1, a.k, F * S + 1, min_target=1.0, max_target=5.0, device=0)
    g.init_device(42)
    g.synth(0, a.rows, F, S, seed=1000, xmode=0)
    g.synth(1, max(a.rows // 100, 1000), F, S, seed=500000, xmode=0)
    g.init_caches()
    steps = []
    for i in range(a.warmup + a.steps):
        t0 = time.perf_counter()
        st = g.iterate()
        steps.append({"wall_ms": (time.perf_counter() - t0) * 1e3, "ms_v": st.ms_v, "rmse": st.rmse,
                      "timed": i >= a.warmup})
        print("step %d: %.1f ms (v sweep %.1f) rmse %.6f" % (i, steps[-1]["wall_ms"], st.ms_v, st.rmse),
              file=sys.stderr, flush=True)
    print(json.dumps({"hip_runtime": mapped("libamdhip64"), "hsa_runtime": mapped("libhsa-runtime64"),
                      "torch_imported": "torch" in sys.modules, "layout": g.layout(), "rows": a.rows,
                      "k": a.k, "steps": steps}))
    g.close()


if __name__ == "__main__":
    main()
