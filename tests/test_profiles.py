"""Provenance of the committed measurement records (CPU): the traffic figure
bench.py quotes (profiles/pmc_traffic.json, roofline.traffic) is exactly what
scripts/pmc_traffic.py derives from the committed rocprofv3 --pmc passes it
names, and every profile file DESIGN.md cites for rounds 4 to 6 exists."""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def test_pmc_traffic_reproduces_from_committed_passes():
    from pmc_traffic import compute
    rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))["c3"]
    csvs = re.findall(r"(profiles/\S+?\.csv)", rec["source"]) + re.findall(r"(profiles/\S+?\.csv)", rec["source_pmc"])
    assert len(csvs) == 3
    again = compute(*[os.path.join(ROOT, c) for c in csvs])
    for k in ("hbm_bytes_per_launch", "fetch_bytes_corrected", "write_bytes", "ratio_to_algorithmic", "lds_busy",
              "held_clock_ghz", "valu_wave_instr_per_cu_clk"):
        assert again[k] == rec[k], k


def test_design_cites_existing_round4_to_round6_profiles():
    text = open(os.path.join(ROOT, "DESIGN.md")).read()
    for rnd in ("r04", "r05", "r06"):
        cited = set(re.findall(r"`(profiles/%s/[^`*{}\n]+?)`" % rnd, text))
        assert cited, rnd
        missing = [c for c in cited if not os.path.exists(os.path.join(ROOT, c.rstrip("/").split(" ")[0]))]
        assert not missing, missing
