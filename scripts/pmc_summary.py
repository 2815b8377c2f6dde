#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter_collection CSVs: each
counter summed per dispatch (over XCDs / SEs), then averaged over the
kernel's dispatches; with GRBM_GUI_ACTIVE the held clock (GRBM_GUI_ACTIVE / 8
XCDs / duration, MI355X_MICROARCH.md 'DVFS give-back') and, with
SQ_LDS_IDX_ACTIVE / SQ_INSTS_VALU, the LDS busy fraction and VALU
wave-instructions per CU-clock.  Usage: pmc_summary.py CSV [CSV ...] [--match S]"""
import collections
import csv
import sys

NUM_CUS, XCDS = 256, 8


def summarize(paths, match=None):
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter -> value
    dur = {}
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            key = (k, path, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = collections.OrderedDict()
    for (k, path, d), cnt in per.items():
        o = out.setdefault(k, collections.defaultdict(list))
        o["duration_ms"].append(dur[(k, path, d)] * 1e3)
        for c, v in cnt.items():
            o[c].append(v)
        if "GRBM_GUI_ACTIVE" in cnt and dur[(k, path, d)] > 0:
            cyc = cnt["GRBM_GUI_ACTIVE"] / XCDS
            o["clock_ghz"].append(cyc / dur[(k, path, d)] / 1e9)
            if "SQ_LDS_IDX_ACTIVE" in cnt:
                o["lds_busy"].append(cnt["SQ_LDS_IDX_ACTIVE"] / (NUM_CUS * cyc))
            if "SQ_INSTS_VALU" in cnt:
                o["valu_per_cu_clk"].append(cnt["SQ_INSTS_VALU"] / (NUM_CUS * cyc))
    return {k: {c: sum(v) / len(v) for c, v in o.items()} for k, o in out.items()}


if __name__ == "__main__":
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        del args[i:i + 2]
    for k, o in summarize(args, match).items():
        print(k[:70])
        for c, v in sorted(o.items()):
            print("   %-32s %.6g" % (c, v))
