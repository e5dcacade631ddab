#!/usr/bin/env python3
"""Copy one round's measurements from gpurun_out/round_<tag> (tools/profile_round.sh) into
profiles/: the bench lines, rocprofv3 kernel statistics, PMC summaries and the HBM traffic files
bench.py reads for roofline.traffic.  Usage: tools/profile_collect.py TAG"""
import json
import os
import shutil
import subprocess
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"round_{tag}")
dst = os.path.join(root, "profiles")
pmc = os.path.join(root, "gpurun_out", "pmc")


def last_json(path):
    with open(path) as fh:
        return json.loads([ln for ln in fh.read().splitlines() if ln.startswith("{")][-1])


json.dump(last_json(f"{src}/bench.json"), open(f"{dst}/{tag}_bench.json", "w"))
for wl, suffix in (("", ""), ("_live", "_live"), ("_c5", "_c5"), ("_c5x", "_c5_exact")):
    if not os.path.exists(f"{src}/kt{wl}"):
        continue
    shutil.copy(f"{src}/kt{wl}/kt_kernel_stats.csv", f"{dst}/{tag}_kernel_stats{suffix}.csv")
    json.dump(last_json(f"{src}/kt{wl}.log"), open(f"{dst}/{tag}_bench{suffix}_under_rocprof.json", "w"))
for sub, name, kernel, match in ((tag, "stft", "stft1024_kernel<short, 0, true, false>", {"files": 1440, "nperseg": 1024}),
                                 (f"{tag}_c5", "cstft", "cstft4096_kernel<short, 4, false, 2, true>", None),
                                 (f"{tag}_c5det", None, None, None), (f"{tag}_c5i8", None, None, None)):
    if not os.path.isdir(f"{pmc}/{sub}"):
        continue
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "pmc_summary.py"), f"{pmc}/{sub}"],
                         capture_output=True, text=True, check=True).stdout
    suffix = sub[len(tag):]
    open(f"{dst}/{tag}_pmc_summary{suffix}.txt", "w").write(out)
    if name is None:
        continue
    summ = json.load(open(f"{pmc}/{sub}/summary.json"))[kernel]
    if "hbm_bytes" not in summ:  # a pass missing (FETCH_SIZE or WRITE_SIZE): keep the last traffic file
        print(f"{sub}: no complete FETCH_SIZE + WRITE_SIZE pair for {kernel}; profiles/{name}_pmc.json kept")
        continue
    rec = {"kernel": kernel, "hbm_bytes_per_launch": summ["hbm_bytes"], "fetch_size_kib": summ["FETCH_SIZE"],
           "write_size_kib": summ["WRITE_SIZE"],
           "rule": "HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950: FETCH_SIZE reports half of wide "
                   "streaming reads, MI355X_MICROARCH.md HBM/rocprofv3 section)",
           "source": f"tools/pmc_stft.sh {sub} (4 separate --pmc passes), per-dispatch averages"}
    if match:
        rec.update(match)
    else:  # C5: frames per launch and nperseg as bench.py reports them
        b = last_json(f"{src}/kt_c5.log")
        rec.update({"frames": b["config"]["frames_per_gpu"], "nperseg": 4096})
    json.dump(rec, open(f"{dst}/{name}_pmc.json", "w"), indent=1)
# per-dispatch durations of each workload's roofline kernel from the kernel trace: the stats
# average includes the cold first (warm-up) dispatch; the timed steps' average is the figure
# the bench line's live HIP-event timing reports under the profiler
kt0 = last_json(f"{src}/kt.log")
KW, KS = kt0.get("warmup", 1), kt0.get("steps", 5)
lines = ["roofline kernel, per-dispatch durations (ms) from rocprofv3 --kernel-trace; the run is "
         f"bench.py --steps {KS} --warmup {KW}: dispatches 1-{KW} are the warm-up, {KW + 1}-{KW + KS} the timed "
         f"steps, {KW + KS + 1} the step after the timed region that times every kernel for the breakdown"]
import csv
for wl, key in (("", "stft1024_kernel"), ("_live", "welch_i8_kernel"), ("_c5", "cstft4096_kernel"),
                ("_c5x", "cstft4096_kernel")):
    if not os.path.exists(f"{src}/kt{wl}"):
        continue
    rows = list(csv.DictReader(open(f"{src}/kt{wl}/kt_kernel_trace.csv")))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if key in r["Kernel_Name"]]
    if wl == "_live":  # the live line's kernel_ms is welch_i8_kernel + welch_i8_bands_kernel (one each per step)
        bd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
              if "welch_i8_bands_kernel" in r["Kernel_Name"]]
        if len(bd) == len(d):
            d = [a + b for a, b in zip(d, bd)]
            key = "welch_i8_kernel + welch_i8_bands_kernel"
    b = last_json(f"{src}/kt{wl}.log")
    live = b["roofline"].get("kernel_ms")
    lines.append(f"{key} ({wl[1:] or 'c3'}): " + " ".join(f"{x:.3f}" for x in d) +
                 f" | all {sum(d) / len(d):.3f} | timed steps {sum(d[KW:KW + KS]) / max(1, len(d[KW:KW + KS])):.3f}"
                 f" | bench live HIP events {live}")
open(f"{dst}/{tag}_dispatches.txt", "w").write("\n".join(lines) + "\n")
print("profiles updated for", tag)
