"""ctypes loader for the C restatement of numpy's legacy randint
(mt19937_randint.c).  TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "build", "liboracle_mt.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(path)
        L.oracle_mt_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_randint.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64,
                                     ctypes.c_void_p]
        L.oracle_mt_next.restype = ctypes.c_uint32
        L.oracle_mt_next.argtypes = [ctypes.c_void_p]
        _LIB = L
    return _LIB


class MT:
    def __init__(self, seed):
        L = lib()
        self.buf = ctypes.create_string_buffer(L.oracle_mt_state_bytes())
        L.oracle_mt_seed(self.buf, seed)

    def randint(self, n, B):
        out = np.empty(B, np.int64)
        lib().oracle_randint(self.buf, n, B, out.ctypes.data)
        return out

    def next_u32(self, k):
        return np.array([lib().oracle_mt_next(self.buf) for _ in range(k)], np.uint32)
