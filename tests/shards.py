"""Dependency levels and the feature-shard assignment of libvbfm's VBFM_SHARD_FEATURES mode,
restated in numpy for the tests (vbfm_capi.hip: build_schedule, build_fshards)."""
import numpy as np


def levels(row_ptr, feat, nf):
    """level(j) = 1 + max level of an earlier feature sharing a row (1-based; 1 for features
    without rows): least fixed point of level[b] >= level[a] + 1 over consecutive distinct
    features a < b of every row."""
    lv = np.ones(nf, dtype=np.int64)
    a, b = [], []
    for r in range(len(row_ptr) - 1):
        ids = np.unique(feat[row_ptr[r]:row_ptr[r + 1]])
        a.append(ids[:-1])
        b.append(ids[1:])
    a = np.concatenate(a) if a else np.zeros(0, np.int64)
    b = np.concatenate(b) if b else np.zeros(0, np.int64)
    while True:
        new = lv.copy()
        np.maximum.at(new, b, lv[a] + 1)
        if np.array_equal(new, lv):
            return lv
        lv = new


def feature_shards(row_ptr, feat, nf, nshards):
    """Shard of every train feature: each level's features (ascending id) in nshards
    contiguous chunks, chunk s = [n_l*s // P, n_l*(s+1) // P)."""
    lv = levels(row_ptr, feat, nf)
    shard = np.zeros(nf, dtype=np.int32)
    for level in np.unique(lv):
        js = np.flatnonzero(lv == level)
        nl = len(js)
        for s in range(nshards):
            shard[js[nl * s // nshards: nl * (s + 1) // nshards]] = s
    return shard
