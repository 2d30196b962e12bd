#!/bin/bash
# round 4 validation + A/B on one box (~15 min):
#  1. the new tests (teacher-forced, mid-state, forced-overlap DP) and the exploration tests
#  2. the B=256 variants' parity subsets (OAC_SMALL_STAGE, OAC_PBWD_FUSE, OAC_HEAD_FUSE), each
#     recorded pass / fail; a crash, abort or time-out ends the script
#  3. the A/B bench of the variants that passed, per-launch times
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_dp.py -v $T -s > gpurun_out/r4_new_tests.log 2>&1
rc=$?; crash $rc; grep -E "PASS|FAIL|worst|Error" gpurun_out/r4_new_tests.log | tail -45; echo "new tests rc=$rc"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "expl or philox" -q $T > gpurun_out/r4_expl_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r4_expl_tests.log; echo "expl tests rc=$rc"
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > gpurun_out/r4_expl_micro.log 2>&1; crash $?
head -20 gpurun_out/r4_expl_micro.log
SUB="tests/test_gpu_parity.py tests/test_gpu_teacher.py"
ok=""
for arm in "1 0 0" "0 1 0" "0 0 1" "1 1 1"; do
  set -- $arm
  X=""; [ "$arm" = "1 1 1" ] && X="tests/test_gpu_dropin.py tests/test_gpu_ring.py"
  OAC_SMALL_STAGE=$1 OAC_PBWD_FUSE=$2 OAC_HEAD_FUSE=$3 timeout -k 10 400 python -u -m pytest $SUB $X -q -x -k "not b4096 and not poac and not particle" $T > gpurun_out/r4_arm_$1$2$3.log 2>&1
  rc=$?; crash $rc; echo "arm stage=$1 pbwd=$2 head=$3 rc=$rc: $(tail -1 gpurun_out/r4_arm_$1$2$3.log)"
  [ $rc -eq 0 ] && ok="$ok $1$2$3"
done
echo "arms passing:$ok"
for i in 1 2; do
  for a in 000 $ok; do
    OAC_SMALL_STAGE=${a:0:1} OAC_PBWD_FUSE=${a:1:1} OAC_HEAD_FUSE=${a:2:1} timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-extras --no-cpu-baseline > gpurun_out/ab_$a.log 2>&1
    rc=$?; crash $rc
    python -c "import json;d=json.loads(open('gpurun_out/ab_$a.log').read().strip().splitlines()[-1]);print('arm $a', d['value'], d['roofline']['avg_launch_us'], d['roofline']['launches_per_step'])"
  done
done
for a in 000 $ok; do
  OAC_SMALL_STAGE=${a:0:1} OAC_PBWD_FUSE=${a:1:1} OAC_HEAD_FUSE=${a:2:1} timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_$a.log 2>&1
  crash $?; echo "arm $a"; head -16 gpurun_out/lt_$a.log
done
