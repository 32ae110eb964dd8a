#!/usr/bin/env python3
"""Summarise the per-workgroup phase stamps of the diagnostic online build (tools/ov_stamps.sh,
VBFM_OV_STAMP): for every stamped k_ov_lord launch, the workgroups' start spread, the phases
(entry -> staged -> posterior -> corrected -> stores issued) and the launch's span, in µs of the
100-MHz real-time counter; then the median over the stamped launches.

usage: tools/ov_stamp_summary.py <stderr of the bench run>"""
import sys

import numpy as np


def main():
    launches, cur = [], None
    for line in open(sys.argv[1]):
        if not line.startswith("OVSTAMP"):
            continue
        f = line.split()
        if f[1] == "launch":
            cur = {"launch": int(f[2]), "nfeat": int(f[4]), "rows": []}
            launches.append(cur)
        elif cur is not None:
            cur["rows"].append([int(x) for x in f[2:7]])
    us = 0.01   # 100 MHz ticks -> µs
    keys = ("start spread p50", "start spread max", "entry->staged p50", "staged->posterior p50",
            "posterior->corrected p50", "corrected->stores issued p50", "workgroup life p50", "workgroup life max",
            "last store issued after first start")
    table = []
    for L in launches:
        t = np.array(L["rows"], dtype=np.float64)
        if len(t) == 0 or np.any(t == 0):
            continue
        t0 = t[:, 0].min()
        st = (t[:, 0] - t0) * us
        d = np.diff(t, axis=1) * us
        life = (t[:, 4] - t[:, 0]) * us
        table.append([np.median(st), st.max(), np.median(d[:, 0]), np.median(d[:, 1]), np.median(d[:, 2]),
                      np.median(d[:, 3]), np.median(life), life.max(), (t[:, 4].max() - t0) * us])
    if not table:
        print("no complete stamps")
        return
    a = np.array(table)
    print("%d stamped launches (%d workgroups each)" % (len(a), len(launches[0]["rows"])))
    for i, k in enumerate(keys):
        print("  %-40s median %7.2f us   [min %.2f, max %.2f]" % (k, np.median(a[:, i]), a[:, i].min(), a[:, i].max()))


if __name__ == "__main__":
    main()
