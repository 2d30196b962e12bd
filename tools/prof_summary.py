"""Average duration of the step's GEMM kernel (all template instances
together) from a rocprofv3 --stats kernel_stats.csv, for comparison with the
`roofline.avg_launch_us` bench.py measures with dispatch events.

usage: python tools/prof_summary.py <rocprof output dir>"""
import csv
import glob
import os
import sys

d = sys.argv[1]
f = max(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True), key=os.path.getmtime)
calls = total = 0
for row in csv.DictReader(open(f)):
    name = row["Name"]
    if "oac::" not in name:
        continue
    n, t = int(row["Calls"]), float(row["TotalDurationNs"])
    short = name.split("(")[0].replace("void ", "")
    print(f"{short:48s} calls {n:6d}  avg {t / n / 1e3:8.3f} us")
    if "oac::gemm_" in name:   # every GEMM kernel family
        calls += n
        total += t
if calls:
    print(f"GEMM kernel (all instances): {calls} calls, avg {total / calls / 1e3:.3f} us")
