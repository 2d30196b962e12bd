O=$PWD/gpurun_out/r6/la3; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_altkernels.py -k "last_arrival or side_workgroup" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
grep -E "PASS|FAIL" $O/tests.txt | cut -c1-150
TAG=la3 bash tools/r6/la2.sh
