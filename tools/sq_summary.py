#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc pass of SQ counters per kernel (tools/gpu.sh step `sq`).

usage: tools/sq_summary.py <p_counter_collection.csv[.gz]> [...]
Per kernel: dispatches, mean duration, VGPR / LDS of the dispatch, and every counter's mean per
dispatch. SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md);
the derived columns are the shares of wave time parked on s_waitcnt / barriers (WAIT_ANY),
stalled at issue (WAIT_INST_ANY) and issuing (ACTIVE_INST_ANY), and the mean number of resident
waves per CU (WAVE_CYCLES * 4 / (duration cycles * 256 CUs), at the dispatch's own clock)."""
import csv
import gzip
import sys
from collections import defaultdict


def main():
    for path in sys.argv[1:]:
        k = defaultdict(lambda: {"n": set(), "dur": {}, "c": defaultdict(float), "meta": ""})
        with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as fh:
            for r in csv.DictReader(fh):
                e = k[r["Kernel_Name"]]
                did = r["Dispatch_Id"]
                e["n"].add(did)
                e["dur"][did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
                e["meta"] = "grid %s wg %s lds %s vgpr %s agpr %s sgpr %s" % (
                    r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"],
                    r["Accum_VGPR_Count"], r["SGPR_Count"])
        print("==", path)
        for name, e in sorted(k.items(), key=lambda kv: -sum(kv[1]["dur"].values())):
            n = len(e["n"])
            dur = sum(e["dur"].values()) / n
            c = {x: v / n for x, v in e["c"].items()}
            print("%s\n  %d dispatches, %.1f us, %s" % (name[:110], n, dur / 1e3, e["meta"]))
            for x in sorted(c):
                print("    %-22s %16.0f" % (x, c[x]))
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                parts = ["%s %.1f %%" % (x[3:], 100 * c[x] / wc) for x in
                         ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if x in c]
                print("    shares of wave time: " + ", ".join(parts))
                if "SQ_BUSY_CYCLES" in c:
                    # BUSY_CYCLES is summed over the 32 shader engines (8 XCDs x 4): / 32 = the
                    # dispatch's cycles (its ratio to the duration is the clock); WAVE_CYCLES in
                    # quad-cycles over 256 CUs gives the mean resident waves per CU
                    cyc = c["SQ_BUSY_CYCLES"] / 32.0
                    print("    clock %.2f GHz, mean resident waves per CU %.1f" % (
                        cyc / dur, wc * 4 / (cyc * 256)))
                if "SQ_WAVES" in c:
                    print("    wave lifetime: %.0f cycles" % (wc * 4 / c["SQ_WAVES"]))


if __name__ == "__main__":
    main()
