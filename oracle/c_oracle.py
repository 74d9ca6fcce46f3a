"""ctypes loader for oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The C restatement of the reference SpMM (oracle/spmm_oracle.c), built by
``make -C oracle``.  Used as the fast checker at large sizes and as bench.py's
cpu_baseline ("port") leg.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "liboracle.so"
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        lib = ctypes.CDLL(str(LIB_PATH))
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.oracle_spmm_csr.argtypes = [vp, vp, vp, i64, i64, vp, i64, i64, vp, vp, i64]
        lib.oracle_spmm_csr.restype = None
        lib.oracle_num_threads.restype = ctypes.c_int
        lib.oracle_set_threads.argtypes = [ctypes.c_int]
        _lib = lib
    return _lib


def set_threads(n: int) -> None:
    load().oracle_set_threads(int(n))


def num_threads() -> int:
    return int(load().oracle_num_threads())


def spmm_csr(rowptr, col, val, x, bias=None, row0: int = 0, row1: int | None = None):
    """fp32 Y[row0:row1] = A X (+ bias) with double accumulation (GCN/GCN.py:43-45)."""
    lib = load()
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    x = np.ascontiguousarray(x, dtype=np.float32)
    n_rows = rowptr.size - 1
    row1 = n_rows if row1 is None else row1
    feat = x.shape[1]
    y = np.empty((row1 - row0, feat), dtype=np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    lib.oracle_spmm_csr(rowptr.ctypes.data, col.ctypes.data, val.ctypes.data, row0, row1,
                        x.ctypes.data, feat, feat, None if b is None else b.ctypes.data,
                        y.ctypes.data, feat)
    return y
