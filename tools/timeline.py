"""Kernel timeline of the last step of a rocprofv3 --kernel-trace run: every dispatch from the
last occurrence of MARK on, with its start (ms from the first), duration and the idle gap
before it.  Usage: python tools/timeline.py <run_kernel_trace.csv> <mark substring> [min_gap_us]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark, min_gap = sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
starts = [i for i, e in enumerate(ev) if mark in e[2]]
i0 = starts[-1]
t0 = ev[i0][0]
busy_end, idle = t0, 0.0
for s, e, name, q in ev[i0:]:
    gap = (s - busy_end) / 1e3
    if gap > 0:
        idle += gap
    if gap >= min_gap or "dq::" in name:
        print("%9.2f %8.2f gap %7.2f q%s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, q, name.split("(")[0][-70:]))
    busy_end = max(busy_end, e)
print("span %.2f ms, idle %.2f ms" % ((busy_end - t0) / 1e3, idle / 1e3))
