#!/usr/bin/env python3
"""Summary of an amd-smi sample file written by scripts/archive/gpu_power.sh /
gpu_r4_power.sh ("== <time>" then `amd-smi metric -g 0 -p -c --json`): socket
power and the mean gfx clock over the 8 XCDs, for the samples taken under
load (socket power >= --min-w, default 900 W: the encode's steady state, not
the fill or idle phases).  Usage: power_summary.py FILE [FILE ...] [--min-w W]"""
import json
import re
import statistics
import sys


def samples(path):
    txt = open(path).read()
    for chunk in re.split(r"^== [0-9.]+\n", txt, flags=re.M):
        chunk = chunk.strip()
        if not chunk.startswith("{"):
            continue
        try:
            d = json.loads(chunk)
        except ValueError:
            continue
        g = d["gpu_data"][0]
        w = g["power"]["socket_power"]["value"]
        clks = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_") and isinstance(v, dict)
                and isinstance(v.get("clk", {}).get("value"), (int, float))]
        if isinstance(w, (int, float)) and clks:
            yield float(w), sum(clks) / len(clks)


def main(argv):
    min_w = 900.0
    if "--min-w" in argv:
        i = argv.index("--min-w")
        min_w = float(argv[i + 1])
        del argv[i:i + 2]
    for path in argv:
        s = [x for x in samples(path) if x[0] >= min_w]
        if not s:
            print("%s: no loaded samples" % path)
            continue
        ws, cs = [x[0] for x in s], [x[1] for x in s]
        print("%s: n=%d  power median %.0f W (%.0f-%.0f)  gfx clock median %.0f MHz (%.0f-%.0f)" % (
            path, len(s), statistics.median(ws), min(ws), max(ws), statistics.median(cs), min(cs), max(cs)))


if __name__ == "__main__":
    main(sys.argv[1:])
