#!/usr/bin/env python3
"""Refresh profiles/pmc_traffic.json["c3"] from one FETCH_SIZE pass, one
WRITE_SIZE pass and one SQ pass (GRBM_GUI_ACTIVE, SQ_LDS_IDX_ACTIVE,
SQ_INSTS_VALU) of `bench.py --steps 1 --warmup 0` at configs[2] (64 GiB).

HBM bytes per launch, corrected as MI355X_MICROARCH.md prescribes for gfx950:
FETCH_SIZE tallies the 128-B requests of wide coalesced reads at 64 B (the
streaming hb_read_kernel over the same 64 GiB reports exactly 1/2), so the
first pass's file reads count x2; what its FETCH_SIZE holds beyond file / 2
is the per-block 1-byte prefix-image lookup (64-B requests, counted 1:1);
WRITE_SIZE x 1024 B.
Usage: pmc_traffic.py FETCH.csv WRITE.csv SQ.csv"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize   # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILE = 64 << 30


def pick(summ, part):
    for k, v in summ.items():
        if part in k:
            return v
    return {}


def compute(fetch_csv, write_csv, sq_csv):
    """The pmc_traffic.json["c3"] record of these three PMC passes."""
    f, w, q = summarize([fetch_csv]), summarize([write_csv]), summarize([sq_csv])
    kb = 1024
    ff, fr, fp = (pick(f, n).get("FETCH_SIZE", 0.0) for n in ("encode_first", "encode_retry", "prefix_kernel"))
    wf, wr, wp = (pick(w, n).get("WRITE_SIZE", 0.0) for n in ("encode_first", "encode_retry", "prefix_kernel"))
    p3 = ff * kb - FILE / 2
    fetch = FILE + p3 + (fr + fp) * kb
    write = (wf + wr + wp) * kb
    sq = pick(q, "encode_first")
    rec = {
        "file_bytes": FILE,
        "hbm_bytes_per_launch": int(round(fetch + write)),
        "fetch_bytes_corrected": int(round(fetch)),
        "write_bytes": int(round(write)),
        "breakdown": {"sector_reads": FILE, "prefix_image_lookups": int(round(p3)),
                      "retry_list_reads": int(round(fr * kb)), "tag_and_retry_list_writes": int(round((wf + wr) * kb)),
                      "prefix_image_build": int(round((fp + wp) * kb))},
        "raw_kB": {"FETCH_SIZE_first": ff, "FETCH_SIZE_retry": fr, "FETCH_SIZE_prefix": fp,
                   "WRITE_SIZE_first": wf, "WRITE_SIZE_retry": wr, "WRITE_SIZE_prefix": wp},
        "correction": __doc__.split("HBM bytes per launch, ")[1].split("Usage")[0].strip().replace("\n", " "),
        "source": "%s, %s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one per pass, bench.py --steps 1 --warmup 0)"
                  % (fetch_csv, write_csv),
        "ratio_to_algorithmic": round((fetch + write) / (FILE + FILE // 512 * 32), 3),
        "lds_busy": round(sq.get("lds_busy", 0.0), 3),
        "held_clock_ghz": round(sq.get("clock_ghz", 0.0), 3),
        "valu_wave_instr_per_cu_clk": round(sq.get("valu_per_cu_clk", 0.0), 3),
        "source_pmc": "%s (first-pass kernel, one rocprofv3 --pmc pass): held clock = GRBM_GUI_ACTIVE / 8 XCDs / "
                      "duration; lds_busy = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE/8); valu = SQ_INSTS_VALU / "
                      "(256 CUs x GRBM_GUI_ACTIVE/8); SQ_LDS_BANK_CONFLICT = %d" % (sq_csv, sq.get("SQ_LDS_BANK_CONFLICT", -1)),
    }
    return rec


def main(fetch_csv, write_csv, sq_csv):
    rec = compute(fetch_csv, write_csv, sq_csv)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(path))
    d["c3"] = rec
    json.dump(d, open(path, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
