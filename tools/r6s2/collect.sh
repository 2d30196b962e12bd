#!/bin/bash
# Copy the summaries of a tools/r6s2/final.sh run (gpurun_out/r6f) into
# profiles/r06 (the final tree's B=256 figures) and refresh
# profiles/pmc_gemm_traffic.json (bench.py's roofline.traffic) for B=256.
set -e
S=gpurun_out/r6f
D=profiles/r06
cp $S/gputest_final.txt $S/smoke.txt $D/
for i in 1 2 3; do tail -1 $S/bench_driver_shape_$i.json > $D/bench_driver_shape_$i.json; done
tail -1 $S/bench256.log > $D/bench_default.json
cp "$(ls -t $S/prof_b256/*/*kernel_stats.csv | head -1)" $D/b256_kernel_stats.csv
python3 tools/prof_summary.py $S/prof_b256 > $D/b256_gemm_avg.txt
python3 tools/trace.py $S/prof_b256 10 > $D/b256_step_trace.txt || true
for k in fetch write sq; do rm -rf gpurun_out/pmc_b256_$k; cp -r $S/pmc_b256_$k gpurun_out/pmc_b256_$k; done
python3 tools/pmc_summary.py b256 $D/pmc_b256.json --traffic 256 profiles/pmc_gemm_traffic.json > $D/pmc_b256.txt
cp $S/lt_b256.log $D/launch_times_b256.txt
echo "profiles -> $D"
