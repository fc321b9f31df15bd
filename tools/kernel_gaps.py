"""Idle gaps between consecutive kernels of the bench step, from a rocprofv3 --kernel-trace CSV
(tools/profile.sh): per kernel pair (previous -> next), the median time from the previous kernel's end
to the next kernel's start, over the timed steps.  usage: python tools/kernel_gaps.py <kernel_trace.csv>"""
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.split(r"[(<]", n)[0][:28]
gaps = {}
for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
    gaps.setdefault((short(n0), short(n1)), []).append((s1 - e0) / 1000.0)
for (a, b), g in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
    if len(g) >= 5:
        print("%-28s -> %-28s  n=%3d  median gap %6.2f us  (p10 %.2f, p90 %.2f)" % (
            a, b, len(g), statistics.median(g), sorted(g)[len(g) // 10], sorted(g)[9 * len(g) // 10]))
