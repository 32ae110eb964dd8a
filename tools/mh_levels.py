"""Per-level shape of the multi-hot bench's schedule (diagnostic): for every dependency level its
column count and mean column length, grouped by the workgroup shape dispatch_shape() gives it and
by the rounds of resident workgroups it needs. usage: python tools/mh_levels.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scalable-variational-bayesian-factorization-machine_amd"))
import vbfm  # noqa: E402

N, NF, LO, HI, K = 10_000_000, 1_000_000, 5, 60, 50
g = vbfm.FMLearnVB(1, 1, K, NF + 1, min_target=1.0, max_target=5.0)
g.init_device(42)
g.synth_multihot(0, N, NF, LO, HI, seed=1000, xmode=0, row_offset=0)
g.synth_multihot(1, 1000, NF, LO, HI, seed=500000, xmode=0, row_offset=0)
g.init_caches()
lv, L = g.levels()
cp, _, _ = g.get_csc(0)
ln = np.diff(cp.astype(np.int64))
nfeat = np.bincount(lv, minlength=L)
ent = np.bincount(lv, weights=ln, minlength=L)
avg = ent // np.maximum(nfeat, 1)


def shape(a):
    return (64, 2) if a <= 128 else (256, 1) if a <= 200 else (128, 3) if a <= 384 else (256, 2) if a <= 640 else (512, 2)


slots = {(64, 2): 18 * 256, (256, 1): 9 * 256, (128, 3): 6 * 256, (256, 2): 4 * 256, (512, 2): 2 * 256}
print("levels %d, entries %d" % (L, int(ent.sum())))
rows = {}
for l in range(L):
    s = shape(int(avg[l]))
    r = -(-int(nfeat[l]) // slots[s])
    key = (s, r)
    d = rows.setdefault(key, [0, 0, [], []])
    d[0] += 1
    d[1] += int(ent[l])
    d[2].append(int(nfeat[l]))
    d[3].append(int(avg[l]))
for (s, r), (n, e, nf, av) in sorted(rows.items()):
    print("shape %3dx%d rounds %2d: %4d levels, %5.1f %% of entries, columns %d-%d, mean column %d-%d" % (
        s[0], s[1], r, n, 100.0 * e / ent.sum(), min(nf), max(nf), min(av), max(av)))
g.close()
