"""How long does the VBFM_FAULT=comm_stall kernel hold the stream (diagnostic for the deadline test)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
for k, v in (("VBFM_FORCE_COMM", "1"), ("VBFM_FORCE_SPLIT", "1"), ("VBFM_FAULT", "comm_stall"), ("VBFM_FAULT_RANK", "0")):
    os.environ[k] = v
os.environ["VBFM_COMM_TIMEOUT_S"] = sys.argv[1]
import vbfm, synth
rp, f, v, y = synth.generate(8000, 6, 250, 5, 1)
rpt, ft, vt, yt = synth.generate(1500, 6, 250, 6, 1)
nf = 1500
g = vbfm.FMLearnVB(1, 1, 4, nf + 1, min_target=float(y.min()), max_target=float(y.max()), device=0)
g.comm_init(1, 0, vbfm.FMLearnVB.comm_unique_id())
g.init(7, 0.1)
g.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, nf), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, nf))
g.init_caches()
print("layout", g.layout(), "levels", g.levels()[1], flush=True)
t0 = time.time()
try:
    st = g.iterate()
    print("iterate returned after %.3f s, ms_total %.1f, exchange %s" % (time.time() - t0, st.ms_total, g.exchange_info()), flush=True)
except vbfm.VbfmError as e:
    print("iterate raised after %.3f s: %s" % (time.time() - t0, e), flush=True)
t0 = time.time()
try:
    st = g.iterate()
    print("2nd iterate returned after %.3f s" % (time.time() - t0), flush=True)
except vbfm.VbfmError as e:
    print("2nd iterate raised after %.3f s: %s" % (time.time() - t0, e), flush=True)
g.close()
print("closed", flush=True)
