#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes written by tools/pmc_stft.sh: per-dispatch averages per
kernel, plus derived HBM bytes (FETCH_SIZE x2 per the gfx950 rule + WRITE_SIZE, both in KiB)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/pmc_counter_collection.csv")):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        per[(row["Kernel_Name"], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, d, c), v in per.items():
        vals[k][c].append(v)
out = {}
for k, cs in vals.items():
    short = k.replace("void ", "").replace("msd::(anonymous namespace)::", "").split("(")[0]
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    out[short] = avg
    print(short)
    for c in sorted(avg):
        print(f"   {c:28s} {avg[c]:.4g}")
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        hbm = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        print(f"   {'HBM bytes (2xFETCH+WRITE)':28s} {hbm:.4g}")
        out[short]["hbm_bytes"] = hbm
    if "SQ_WAVE_CYCLES" in avg and "SQ_WAIT_ANY" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        print(f"   wait_any {avg['SQ_WAIT_ANY']/w:.2f}  wait_inst {avg.get('SQ_WAIT_INST_ANY',0)/w:.2f}  "
              f"active {avg.get('SQ_ACTIVE_INST_ANY',0)/w:.2f}")
json.dump(out, open(f"{root}/summary.json", "w"), indent=1)
