#!/bin/bash
# one rocprofv3 PMC pass (kernel trace only) of MFMA-pipe / LDS counters over a short B=4096 bench run
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CU_CYCLES \
  --kernel-trace --output-format csv -d $R/gpurun_out/pmc_b4096_mfma \
  -- python3 $R/bench.py --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 --steps-per-launch 1 --batch 4096 \
  > $R/gpurun_out/pmc_b4096_mfma.log 2>&1
cd $R
python3 - <<'PY'
import collections, csv, glob, os
fs = glob.glob("gpurun_out/pmc_b4096_mfma/**/*counter_collection.csv", recursive=True)
f = max(fs, key=os.path.getmtime)
per = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(f)):
    n = row["Kernel_Name"].split("(")[0].replace("void ", "")
    if "oac::" in n:
        per[n + "@grid" + row["Grid_Size"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
with open("gpurun_out/pmc_b4096_mfma.txt", "w") as o:
    for k in sorted(per):
        o.write(f"{k:44s} " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(per[k].items())) + "\n")
print(open("gpurun_out/pmc_b4096_mfma.txt").read())
PY
