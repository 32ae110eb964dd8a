"""A/B of level-kernel variants in separate processes, interleaved (A B C A B C ...), because
the scatter-bound launch time moves by up to +-10 % from one process (allocation) to the next.
usage: python tools/ab_level.py ROUNDS label=libpath[:ENV=V,...] ...
Each child: C4 rows (1e8 x 40 fields x 125000 ids), k=8, 1 warm-up + 2 iterations, prints the
average v-level launch ms. AB_METHOD=mcmc|als in the environment: the MCMC / ALS learner."""
import json, os, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json
sys.path.insert(0, os.environ["AB_PKG"])
import vbfm
N, F, S, k = 100000000, 40, 125000, 8
meth = os.environ.get("AB_METHOD", "vb")
if meth == "vb":
    fml = vbfm.FMLearnVB(1, 1, k, F * S + 1, min_target=1.0, max_target=5.0, device=0)
else:
    fml = vbfm.FMLearnMCMC(1, 1, k, F * S + 1, min_target=1.0, max_target=5.0, device=0, method=meth)
fml.init_device(42)
fml.synth(0, N, F, S, seed=1000, xmode=0)
fml.synth(1, N // 100, F, S, seed=500000, xmode=0)
fml.init_caches()
events = os.environ.get("AB_NO_EVENTS") != "1"
fml.set_profiling(events)
fml.iterate()
st = [fml.iterate() for _ in range(2)]
if events:
    ms = sum(s.ms_vlevel_kernels for s in st) / sum(s.n_vlevel_launches for s in st)
else:   # the v-sweep phase over its launches (gaps included)
    ms = sum(s.ms_v for s in st) / sum(s.num_levels * k for s in st)
print(json.dumps({"ms_launch": ms, "ms_iter": sum(s.ms_total for s in st) / 2, "ms_w": st[-1].ms_w,
                  "rmse": st[-1].rmse if meth == "vb" else st[-1].rmse_all}))
fml.close()
'''


def main():
    rounds = int(sys.argv[1])
    variants = []
    for spec in sys.argv[2:]:
        label, rest = spec.split("=", 1)
        parts = rest.split(":")
        lib, env = parts[0], {}
        for kv in (parts[1].split(",") if len(parts) > 1 else []):
            k, v = kv.split("=")
            env[k] = v
        variants.append((label, lib, env))
    res = {v[0]: [] for v in variants}
    for r in range(rounds):
        for label, lib, env in variants:
            e = dict(os.environ)
            e.update(env)
            e["VBFM_LIB"] = os.path.join(ROOT, lib)
            e["AB_PKG"] = os.path.join(ROOT, "tools", "ab_head") if "head" in lib else \
                os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd")
            out = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], flush=True)
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[label].append(d)
            print("round %d %-10s launch %.3f ms  iter %.1f ms  w %.1f ms  rmse %.9f" % (
                r, label, d["ms_launch"], d["ms_iter"], d["ms_w"], d["rmse"]), flush=True)
    for label in res:
        xs = sorted(d["ms_launch"] for d in res[label])
        print("%-10s launch ms: min %.3f median %.3f max %.3f" % (label, xs[0], xs[len(xs) // 2], xs[-1]))


if __name__ == "__main__":
    main()
