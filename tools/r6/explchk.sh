set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "expl or philox or single" > gpurun_out/r6/expl_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/r6/expl_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 200 taskset -c 0-3 python tools/r6/expl_py.py 2>&1 | grep -v amdgpu.ids
