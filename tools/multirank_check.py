"""2-rank row-sharded run over RCCL vs a single-rank run on all rows (same GPU or two GPUs).
Launch: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/multirank_check.py"""
import os, sys, json
import numpy as np
import torch
import torch.distributed as dist
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scalable-variational-bayesian-factorization-machine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vbfm, synth

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ndev = torch.cuda.device_count()
dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
dist.init_process_group("gloo")
N, F, S, K = 40000, 6, 300, 4
rp, f, v, y = synth.generate(N, F, S, 5, 1)
rpt, ft, vt, yt = synth.generate(2000, F, S, 6, 1)
D = F * S + 1
lo, hi = rank * N // world, (rank + 1) * N // world
sl = slice(int(rp[lo]), int(rp[hi]))
shard = vbfm.DataSubset.from_csr(rp[lo:hi + 1] - rp[lo], f[sl], v[sl], y[lo:hi], F * S)
tlo, thi = rank * 2000 // world, (rank + 1) * 2000 // world
tsl = slice(int(rpt[tlo]), int(rpt[thi]))
tshard = vbfm.DataSubset.from_csr(rpt[tlo:thi + 1] - rpt[tlo], ft[tsl], vt[tsl], yt[tlo:thi], F * S)
fml = vbfm.FMLearnVB(1, 1, K, D, min_target=float(y.min()), max_target=float(y.max()), device=dev)
obj = [vbfm.FMLearnVB.comm_unique_id() if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)
fml.comm_init(world, rank, obj[0])
fml.init(7, 0.1)
fml.set_data(shard, tshard)
fml.init_caches()
st = [fml.iterate() for _ in range(3)]
res = {"rank": rank, "dev": dev, "rmse": [s.rmse for s in st], "fe": [s.free_energy for s in st],
       "alpha": [s.alpha for s in st], "mu_v": float(np.sum(fml.get_params()["mu_v"] ** 2))}
if rank == 0:
    full = vbfm.FMLearnVB(1, 1, K, D, min_target=float(y.min()), max_target=float(y.max()), device=dev)
    full.init(7, 0.1)
    full.set_data(vbfm.DataSubset.from_csr(rp, f, v, y, F * S), vbfm.DataSubset.from_csr(rpt, ft, vt, yt, F * S))
    full.init_caches()
    sf = [full.iterate() for _ in range(3)]
    ref = {"rmse": [s.rmse for s in sf], "fe": [s.free_energy for s in sf], "alpha": [s.alpha for s in sf],
           "mu_v": float(np.sum(full.get_params()["mu_v"] ** 2))}
    ok = all(abs(a - b) <= 1e-9 * abs(b) for k in ("rmse", "fe", "alpha") for a, b in zip(res[k], ref[k]))
    ok = ok and abs(res["mu_v"] - ref["mu_v"]) <= 1e-9 * ref["mu_v"]
    print(json.dumps({"sharded": res, "single": ref, "match_1e-9": ok}), flush=True)
dist.barrier()
fml.close()
