#!/bin/bash
# Copy the summaries of a tools/measure_r4.sh run (gpurun_out/) into profiles/<round>/
# and refresh profiles/pmc_gemm_traffic.json (read by bench.py's roofline.traffic).
set -e
R=${1:-r04}
D=profiles/$R
mkdir -p $D
tail -1 gpurun_out/bench256.log > $D/bench_default.json
tail -1 gpurun_out/bench4096.log > $D/bench_b4096.json
cp "$(ls -t gpurun_out/prof_b256/*/*kernel_stats.csv | head -1)" $D/b256_kernel_stats.csv
cp "$(ls -t gpurun_out/prof_b4096/*/*kernel_stats.csv | head -1)" $D/b4096_kernel_stats.csv
cp "$(ls -t gpurun_out/prof_poac4096/*/*kernel_stats.csv | head -1)" $D/poac4096_kernel_stats.csv
cp "$(ls -t gpurun_out/prof_expl/*/*kernel_stats.csv | head -1)" $D/expl_kernel_stats.csv
python3 tools/prof_summary.py gpurun_out/prof_b256 > $D/b256_gemm_avg.txt
python3 tools/prof_summary.py gpurun_out/prof_b4096 > $D/b4096_gemm_avg.txt
python3 tools/prof_summary.py gpurun_out/prof_poac4096 > $D/poac4096_gemm_avg.txt
python3 tools/prof_summary.py gpurun_out/prof_expl > $D/expl_kernel_avg.txt
python3 tools/trace.py gpurun_out/prof_b256 11 > $D/b256_step_trace.txt
python3 tools/trace.py gpurun_out/prof_b4096 13 > $D/b4096_step_trace.txt
python3 tools/trace.py gpurun_out/prof_poac4096 17 > $D/poac4096_step_trace.txt || true
rm -f profiles/pmc_gemm_traffic.json
python3 tools/pmc_summary.py b256 $D/pmc_b256.json --traffic 256 profiles/pmc_gemm_traffic.json > $D/pmc_b256.txt
python3 tools/pmc_summary.py b4096 $D/pmc_b4096.json --traffic 4096 profiles/pmc_gemm_traffic.json > $D/pmc_b4096.txt
python3 tools/pmc_summary.py poac4096 $D/pmc_poac4096.json --traffic poac4096 profiles/pmc_gemm_traffic.json > $D/pmc_poac4096.txt
[ -f gpurun_out/pmc_b4096_mfma.txt ] && cp gpurun_out/pmc_b4096_mfma.txt $D/pmc_b4096_mfma.txt
cp gpurun_out/lt_b256.log $D/launch_times_b256.txt
cp gpurun_out/lt_b4096.log $D/launch_times_b4096.txt
cp gpurun_out/lt_poac.log $D/launch_times_poac.txt
cp gpurun_out/expl_micro.log $D/expl_micro.txt
cp gpurun_out/dataflow_micro.log $D/dataflow_micro_b256.txt
echo "profiles -> $D"
