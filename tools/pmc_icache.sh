#!/bin/bash
# rocprofv3 PMC passes (kernel trace only, one counter group per pass) of the
# instruction-fetch counters over a short B=256 drop-in bench run: how much of
# a launch's time goes to fetching its code (the step's kernels are 10-46 KB each)
R=$PWD
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_ic_$1 \
    -- python3 $R/bench.py --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 \
    > $R/gpurun_out/pmc_ic_$1.log 2>&1
}
run sqc "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" || echo "sqc pass rc $?"
run sq "SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" || echo "sq pass rc $?"
cd $R
python3 - <<'PY'
import collections, csv, glob, os
for tag in ("sqc", "sq"):
    fs = glob.glob(f"gpurun_out/pmc_ic_{tag}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(tag, "no counter file"); continue
    f = max(fs, key=os.path.getmtime)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        n = row["Kernel_Name"].split("(")[0].replace("void ", "")
        if "oac::" in n:
            per[n[:50] + "@grid" + row["Grid_Size"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(per):
        print(f"{tag} {k:60s} " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(per[k].items())))
PY
