"""Per-kernel averages of the rocprofv3 PMC passes written by tools/pmc.sh.

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch; on gfx950 FETCH_SIZE
counts wide coalesced reads at half their bytes (MI355X_MICROARCH.md, HBM),
so HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
usage: python tools/pmc_summary.py <tag> [json-out]"""
import collections
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")


def load(kind):
    files = glob.glob(os.path.join(R, f"pmc_{tag}_{kind}", "**", "*counter_collection.csv"),
                      recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            if "oac::" not in name:
                continue
            per[name + "@grid" + row["Grid_Size"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


out = {}
for kind in ("fetch", "write", "sq"):
    for k, d in load(kind).items():
        for c, v in d.items():
            out.setdefault(k, {})[c] = sum(v) / len(v)
for k, d in sorted(out.items()):
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
    print(k.ljust(40), " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1, sort_keys=True)
