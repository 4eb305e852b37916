"""Per-dispatch timeline of the last dispatches of a rocprofv3 kernel trace
(gpurun_out/<dir>/run_kernel_trace.csv): duration and the idle gap before
each dispatch.

  python scripts/trace_timeline.py gpurun_out/r05c/trace_r64n7 [last=20]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
prev = None
for r in rows[-last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev is not None else 0.0
    prev = e
    print(f"{r['Kernel_Name'][:58]:58s} {(e - s) / 1000:10.1f} us  gap {gap:8.1f} us")
