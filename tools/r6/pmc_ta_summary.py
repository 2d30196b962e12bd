"""Summarise tools/r6/pmc_ta4096.sh: per (kernel, grid) the mean of each
counter over its dispatches, and the TA / TD busy fraction of the kernel's
cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "."
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/*/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "oac::" not in name:
            continue
        key = name.split("(")[0].replace("oac::", "")[:40] + "@" + r["Grid_Size"]
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in sorted(acc):
    c = {k: sum(v) / len(v) for k, v in acc[key].items()}
    gui = c.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
    line = f"{key:50s} cycles {gui:9.0f}"
    for k in ("TA_BUSY_avr", "TA_BUSY_max", "TD_BUSY_avr", "TD_BUSY_max"):
        if k in c:
            line += f"  {k}={c[k] / gui:.2f}"
    for k in ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "SQ_INSTS_VMEM_RD",
              "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE",
              "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"):
        if k in c:
            line += f"  {k}={c[k]:.3g}"
    if "TCC_HIT_sum" in c:
        line += f"  hit_rate={c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}"
    print(line)
