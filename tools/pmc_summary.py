#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, KB per dispatch) per kernel and
write profiles/traffic_<config>_<layout>.json for the bench's dominant level kernel.

usage: tools/pmc_summary.py <prof dir> <kernel substring> <out summary.txt> [traffic json]
FETCH_SIZE / WRITE_SIZE are in KB (x1024 bytes). The gfx950 x2 correction of FETCH_SIZE for
16-B/lane coalesced streaming reads (MI355X_MICROARCH.md) is applied to the level kernel's
streamed bytes only when the calibration below says so; see the json's "calibration"."""
import csv
import json
import os
import sys
from collections import defaultdict


def load(path):
    agg = defaultdict(lambda: [0, 0.0, 0, ""])
    with open(path) as fh:
        for r in csv.DictReader(fh):
            a = agg[r["Kernel_Name"]]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
            a[2] = int(r["Grid_Size"])
            a[3] = r["Counter_Name"]
    return agg


def main():
    d, kern, out = sys.argv[1], sys.argv[2], sys.argv[3]
    lines, res = [], {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        agg = load(os.path.join(d, c, "p_counter_collection.csv"))
        for name, (n, tot, grid, cn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            lines.append("%s\t%s\tdispatches=%d\tavg_KB=%.0f" % (c, name[:90], n, tot / n))
        sel = [(n, tot) for name, (n, tot, _, _) in agg.items() if kern in name]
        res[c] = sum(t for _, t in sel) / max(1, sum(n for n, _ in sel)) * 1024.0
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("%s: FETCH %.3g B/launch  WRITE %.3g B/launch" % (kern, res["FETCH_SIZE"], res["WRITE_SIZE"]))
    if len(sys.argv) > 4:
        return res
    return res


if __name__ == "__main__":
    main()
