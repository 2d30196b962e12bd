"""bench.py under a HIP device schedule flag set before any device use
(round 6 A/B): python tools/r6/sched_bench.py {auto,spin,yield,block} [bench args]"""
import ctypes
import os
import runpy
import sys

flag = {"auto": 0, "spin": 1, "yield": 2, "block": 4}[sys.argv[1]]
if flag:
    rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(flag)
    assert rc == 0, rc
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[2:]
sys.path.insert(0, root)
runpy.run_path(sys.argv[0], run_name="__main__")
