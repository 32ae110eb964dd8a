"""A/B of the level kernels on skewed (Zipf) two-field data -- user/item-like columns up to
tens of thousands of rows, so most item columns take the chunked (n > CAP) path.
usage: python tools/ab_skew.py ROUNDS label=libpath ..."""
import json, os, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json
import numpy as np
sys.path.insert(0, os.environ["AB_PKG"])
import vbfm
N, U, I, k = 20000000, 200000, 20000, 8
rng = np.random.default_rng(3)
u = rng.integers(0, U, N).astype(np.uint32)
it = (rng.zipf(1.3, N) - 1) % I
f = np.empty(2 * N, np.uint32); f[0::2] = u; f[1::2] = U + it.astype(np.uint32)
v = np.ones(2 * N, np.float32)
y = rng.integers(1, 6, N).astype(np.float32)
rp = np.arange(0, 2 * N + 1, 2, dtype=np.uint64)
tr = vbfm.DataSubset.from_csr(rp, f, v, y, U + I)
te = vbfm.DataSubset.from_csr(rp[:100001], f[:200000], v[:200000], y[:100000], U + I)
fml = vbfm.FMLearnVB(1, 1, k, U + I + 1, min_target=1.0, max_target=5.0, device=0)
fml.init_device(42)
fml.set_data(tr, te)
fml.init_caches()
fml.set_profiling(True)
fml.iterate()
st = [fml.iterate() for _ in range(2)]
ms = sum(s.ms_vlevel_kernels for s in st) / sum(s.n_vlevel_launches for s in st)
print(json.dumps({"ms_launch": ms, "ms_iter": sum(s.ms_total for s in st) / 2, "layout": fml.layout(), "rmse": st[-1].rmse}))
'''


def main():
    rounds = int(sys.argv[1])
    variants = []
    for a in sys.argv[2:]:
        label, rest = a.split("=", 1)
        parts = rest.split(":")
        env = dict(kv.split("=") for kv in parts[1].split(",")) if len(parts) > 1 else {}
        variants.append((label, parts[0], env))
    res = {v[0]: [] for v in variants}
    for r in range(rounds):
        for label, lib, env in variants:
            e = dict(os.environ)
            e.update(env)
            e["VBFM_LIB"] = os.path.join(ROOT, lib)
            e["AB_PKG"] = os.path.join(ROOT, "tools", "ab_head") if "head" in lib else \
                os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd")
            out = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stderr[-2000:], flush=True)
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[label].append(d)
            print("round %d %-6s launch %.3f ms  iter %.1f ms  %s  rmse %.9f" % (r, label, d["ms_launch"], d["ms_iter"],
                                                                               d["layout"], d["rmse"]), flush=True)


if __name__ == "__main__":
    main()
