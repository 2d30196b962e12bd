#!/bin/bash
# Copy the summaries of a tools/r6/measure.sh run (gpurun_out/r6m) into
# profiles/r06 and refresh profiles/pmc_gemm_traffic.json (bench.py's
# roofline.traffic).  Run in the container after the GPU session.
set -e
S=gpurun_out/r6m
D=profiles/r06
mkdir -p $D
cp $S/gputest_final.txt $S/smoke.txt $D/
for i in 1 2 3; do tail -1 $S/bench_driver_shape_$i.json > $D/bench_driver_shape_$i.json; done
tail -1 $S/bench256.log > $D/bench_default.json
tail -1 $S/bench4096.log > $D/bench_b4096.json
for t in b256 b4096 poac4096 expl; do
  cp "$(ls -t $S/prof_$t/*/*kernel_stats.csv | head -1)" $D/${t}_kernel_stats.csv
  python3 tools/prof_summary.py $S/prof_$t > $D/${t}_gemm_avg.txt
done
mv $D/expl_gemm_avg.txt $D/expl_kernel_avg.txt
python3 tools/trace.py $S/prof_b256 11 > $D/b256_step_trace.txt || true
python3 tools/trace.py $S/prof_b4096 13 > $D/b4096_step_trace.txt || true
for b in b256 b4096; do
  for k in fetch write sq; do rm -rf gpurun_out/pmc_${b}_$k; cp -r $S/pmc_${b}_$k gpurun_out/pmc_${b}_$k; done
done
cp -r gpurun_out/r6m/pmc_poac4096_* gpurun_out/ 2>/dev/null || true
python3 tools/pmc_summary.py b256 $D/pmc_b256.json --traffic 256 profiles/pmc_gemm_traffic.json > $D/pmc_b256.txt
python3 tools/pmc_summary.py b4096 $D/pmc_b4096.json --traffic 4096 profiles/pmc_gemm_traffic.json > $D/pmc_b4096.txt
python3 tools/pmc_summary.py poac4096 $D/pmc_poac4096.json --traffic poac4096 profiles/pmc_gemm_traffic.json > $D/pmc_poac4096.txt
python3 tools/r6/pmc_kernels.py $S/pmc_b4096_mfma gemm > $D/pmc_b4096_mfma.txt
cp $S/lt_b256.log $D/launch_times_b256.txt
cp $S/lt_b4096.log $D/launch_times_b4096.txt
cp $S/lt_poac.log $D/launch_times_poac.txt
cp $S/expl_micro.log $D/expl_micro.txt
cp $S/bwd_micro.log $D/bwd_micro.txt
cp $S/bwd_clock.log $D/bwd_clock.txt
echo "profiles -> $D"
