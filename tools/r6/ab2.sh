#!/bin/bash
# round 6: interleaved same-box A/B over (library build, backward cfg) pairs:
# MICRO="variant:cfg ..." runs tools/micro/bwd_micro <cfg> against the build
# in tools/r6/libs/<variant>; STEP="variant:cfg ..." runs tools/launch_times.py
# (B=4096 SAC, and configs[4] when POAC=1) with OAC_BWDP_CFG=<cfg>
R=$PWD
O=$R/gpurun_out/r6/${TAG:-ab2}
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for vc in $MICRO; do
    v=${vc%%:*}; c=${vc##*:}
    LD_LIBRARY_PATH=$R/tools/r6/libs/$v timeout -k 5 60 tools/micro/bwd_micro $c 1 > $O/m_${v}_${c}_$r.txt 2>&1; crash $?
    echo "micro $v cfg$c r$r: $(sed 's/.*cfg'$c' *//' $O/m_${v}_${c}_$r.txt | awk '{printf "%s ", $1}')"
  done
  for vc in $STEP; do
    v=${vc%%:*}; c=${vc##*:}
    OAC_BWDP_CFG=$c OAC_TUNE=bwdp_cfg=$c OAC_LIB=$R/tools/r6/libs/$v/liboac_amd.so timeout -k 10 150 python tools/launch_times.py --batch 4096 --rate-steps 600 > $O/s_${v}_${c}_$r.txt 2>&1; crash $?
    echo "b4096 $v cfg$c r$r: $(grep drop-in $O/s_${v}_${c}_$r.txt | cut -c1-60)"
    grep "launch " $O/s_${v}_${c}_$r.txt | awk '{printf "%s ", $4}'; echo
    if [ -n "$POAC" ]; then
      OAC_BWDP_CFG=$c OAC_TUNE=bwdp_cfg=$c OAC_LIB=$R/tools/r6/libs/$v/liboac_amd.so timeout -k 10 150 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > $O/p_${v}_${c}_$r.txt 2>&1; crash $?
      echo "poac $v cfg$c r$r: $(grep drop-in $O/p_${v}_${c}_$r.txt | cut -c1-60)"
      grep "launch " $O/p_${v}_${c}_$r.txt | awk '{printf "%s ", $4}'; echo
    fi
  done
done
