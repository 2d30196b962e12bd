#!/bin/bash
# round 5: the whole GPU suite and smoke on the current tree, then the default bench line
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_pytest_all.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1; rc=$?; crash $rc; tail -2 gpurun_out/r5_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r5_bench_default.log 2>&1; rc=$?; crash $rc
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5_bench_default.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "roof", d["roofline"]["frac"])
print("b4096", d["b4096"]["steps_per_s"], "poac", d["poac_ant_b4096"]["steps_per_s"], "ring", d["ring"]["steps_per_s"])
dp = d["dp1"]; print("dp1", dp.get("steps_per_s"), dp.get("vs_single_process"), dp.get("with_rccl_allreduces"), dp.get("with_rccl_allreduces_overlap_schedule"))
print("expl", d["exploration"]["us_per_call_1obs"], "goac", d["goac"]["steps_per_s"], "poac256", d["poac"]["steps_per_s"])
print("cpu", d["cpu_baseline"]["value"], d["b4096"].get("cpu_baseline", {}).get("value"), d["poac_ant_b4096"].get("cpu_baseline", {}).get("value"))
PY
