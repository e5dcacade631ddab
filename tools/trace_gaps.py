"""Per-kernel summary and the last bench step's timeline from a rocprofv3 --kernel-trace CSV run
(`-d DIR -o NAME --output-format csv`): where the C5 step's time goes between kernels.

usage: python3 tools/trace_gaps.py DIR [STEP_MARK]
STEP_MARK: the kernel that opens a step (default cstft4096); the last complete step is printed
with each kernel's start offset, duration and the idle gap before it."""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(n):
    """the kernel's own name (and template arguments) without namespaces and parameters"""
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = n.split("(")[0]
    return n.split("::")[-1][:60] if "<" not in n else n[n.rfind("::", 0, n.find("<")) + 2:][:60]


def main():
    d = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "cstft4096"
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not f:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = list(csv.DictReader(open(f[0])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    tot = defaultdict(lambda: [0, 0.0])
    for s, e, n in ks:
        tot[short(n)][0] += 1
        tot[short(n)][1] += (e - s) / 1e6
    print("kernel  calls  total_ms  avg_ms")
    for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
        print(f"{n:72s} {c:6d} {t:10.3f} {t / c:9.4f}")
    starts = [i for i, (_, _, n) in enumerate(ks) if mark in n]
    if len(starts) < 2:
        return
    a, b = starts[-2], starts[-1]
    t0 = ks[a][0]
    print(f"\nstep timeline (kernels {a}..{b - 1}, {(ks[b][0] - t0) / 1e6:.3f} ms start to next start)")
    prev_end = t0
    busy = 0.0
    for s, e, n in ks[a:b]:
        gap = (s - prev_end) / 1e6
        busy += (e - s) / 1e6
        print(f"  +{(s - t0) / 1e6:8.3f}  {(e - s) / 1e6:8.4f} ms  gap {gap:7.4f}  {short(n)}")
        prev_end = max(prev_end, e)
    print(f"busy {busy:.3f} ms of {(ks[b][0] - t0) / 1e6:.3f}")


if __name__ == "__main__":
    main()
