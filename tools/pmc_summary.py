"""Per-kernel averages of the rocprofv3 PMC passes written by tools/pmc.sh.

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch; on gfx950 FETCH_SIZE
counts wide coalesced reads at half their bytes (MI355X_MICROARCH.md, HBM),
so HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

usage: python tools/pmc_summary.py <tag> [json-out] [--traffic BATCH FILE]
  --traffic: also merge {BATCH: HBM bytes per GEMM launch} (the mean over every
  dispatch of the step's GEMM kernels: every oac::gemm_* family)
  into FILE -- the `roofline.traffic` bench.py reports."""
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
    # the newest pass only: gpurun merges every call's output into the same
    # directory, so earlier runs' files (other process ids) sit beside it
    files = [max(files, key=os.path.getmtime)] if files else []
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            if "oac::" not in name:
                continue
            per[name + "@grid" + row["Grid_Size"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


out = {}
gemm = collections.defaultdict(list)   # counter -> per-dispatch values of the GEMM kernel
for kind in ("fetch", "write", "sq"):
    for k, d in load(kind).items():
        for c, v in d.items():
            out.setdefault(k, {})[c] = sum(v) / len(v)
            if "oac::gemm_" in k:   # every GEMM kernel family of the step
                gemm[c].extend(v)
for k, d in sorted(out.items()):
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_bytes"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
    print(k.ljust(40), " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
args = [a for a in sys.argv[2:]]
if "--traffic" in args:
    i = args.index("--traffic")
    batch, path = args[i + 1], args[i + 2]
    del args[i:i + 3]
    if gemm.get("FETCH_SIZE") and gemm.get("WRITE_SIZE"):
        f = sum(gemm["FETCH_SIZE"]) / len(gemm["FETCH_SIZE"])
        w = sum(gemm["WRITE_SIZE"]) / len(gemm["WRITE_SIZE"])
        per_launch = 2 * f * 1024 + w * 1024
        d = {}
        if os.path.exists(path):
            d = json.load(open(path))
        d[str(batch)] = round(per_launch)
        json.dump(d, open(path, "w"), indent=1, sort_keys=True)
        print(f"GEMM launches: {len(gemm['FETCH_SIZE'])} dispatches, "
              f"HBM bytes per launch {per_launch:.4g} -> {path}")
if args:
    json.dump(out, open(args[0], "w"), indent=1, sort_keys=True)
