"""Per-kernel (name@grid) averages of a rocprofv3 --pmc counter CSV.
usage: pmc_kernels.py <rocprof output dir> [kernel-name filter]"""
import collections, csv, glob, os, sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "oac::"
fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
f = max(fs, key=os.path.getmtime)
per = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(f)):
    n = row["Kernel_Name"].split("(")[0].replace("void ", "")
    if flt in n:
        per[n + "@grid" + row["Grid_Size"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(per):
    c = {n: sum(v) / len(v) for n, v in per[k].items()}
    extra = ""
    if c.get("SQ_BUSY_CU_CYCLES"):
        extra += f"  mfma/(4*cu)={c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (4 * c['SQ_BUSY_CU_CYCLES']):.3f}"
    if c.get("SQ_INSTS_VALU_MFMA_MOPS_F32"):
        extra += f"  valu/mfma_inst={c['SQ_INSTS_VALU'] / (c['SQ_INSTS_VALU_MFMA_MOPS_F32'] / 8):.2f}"
    if c.get("SQ_WAVE_CYCLES"):
        extra += f"  wait_inst/wave={c.get('SQ_WAIT_INST_ANY', 0) / c['SQ_WAVE_CYCLES']:.2f}" \
                 f" wait_any/wave={c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']:.2f}"
    print(f"{k:52s} n={len(next(iter(per[k].values())))}" + extra)
    print("    " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
