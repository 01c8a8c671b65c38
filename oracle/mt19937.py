"""ORACLE ctypes wrapper around oracle/mt19937_oracle.c -- test infrastructure only."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libmt19937_oracle.so")
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C")
        _LIB.oracle_mt_stream.argtypes = [ctypes.c_uint32, ctypes.c_int,
                                          np.ctypeslib.ndpointer(np.uint32, flags="C")]
        _LIB.oracle_inbatch.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, i64p]
        _LIB.oracle_catalogue.argtypes = [ctypes.c_uint32, ctypes.c_int, i64p, ctypes.c_int,
                                          i64p, i64p, i64p, ctypes.c_int, ctypes.c_int, i64p]
    return _LIB


def mt_stream(seed, n):
    out = np.empty(n, dtype=np.uint32)
    lib().oracle_mt_stream(seed, n, out)
    return out


def inbatch(seed, B, N):
    out = np.empty((B, N), dtype=np.int64)
    assert lib().oracle_inbatch(seed, B, N, out) == 0
    return out


def catalogue(seed, reseed, split_items, indptr, indices, users, N):
    split_items = np.ascontiguousarray(split_items, dtype=np.int64)
    users = np.ascontiguousarray(users, dtype=np.int64)
    out = np.empty((len(users), N), dtype=np.int64)
    rc = lib().oracle_catalogue(seed, int(bool(reseed)), split_items, len(split_items),
                                np.ascontiguousarray(indptr, dtype=np.int64),
                                np.ascontiguousarray(indices, dtype=np.int64),
                                users, len(users), N, out)
    if rc != 0:
        raise ValueError("oracle_catalogue failed: %d" % rc)
    return out
