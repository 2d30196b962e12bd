#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_parity.py tests/test_gpu_particle.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_eval.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_eval.log | head -40; exit $rc
