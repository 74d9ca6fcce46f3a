"""ctypes loader for oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The C restatement of the reference SpMM, both GAT layers and the GraphSAGE
gather-reduce (oracle/spmm_oracle.c), built by
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
        lib.oracle_gat_csr.argtypes = [vp, vp, i64, i64, vp, i64, vp, vp, i64, i64, i64,
                                       ctypes.c_double, ctypes.c_int, vp, i64]
        lib.oracle_gat_csr.restype = None
        lib.oracle_sage_gather.argtypes = [vp, i64, vp, i64, i64, i64, i64, ctypes.c_int, vp, i64]
        lib.oracle_sage_gather.restype = None
        lib.oracle_sage_argmax.argtypes = [vp, i64, vp, i64, i64, i64, i64, vp, i64]
        lib.oracle_sage_argmax.restype = None
        lib.oracle_gat_block_grad.argtypes = [vp, vp, i64, vp, vp, vp, vp, vp, i64, i64,
                                              ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_double, ctypes.c_uint64, vp, vp, vp, vp,
                                              vp, vp]
        lib.oracle_gat_block_grad.restype = ctypes.c_int
        lib.oracle_dropout_keep.argtypes = [ctypes.c_uint64, vp, vp, i64, ctypes.c_float, vp]
        lib.oracle_dropout_keep.restype = None
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


def gat_csr(rowptr, col, wh, el, er, heads: int, fh: int, slope: float, sparse: bool,
            row0: int = 0, row1: int | None = None):
    """fp32 [row1 - row0, heads * fh] GAT aggregation (float64 inside) over CSR rows
    [row0, row1): the dense (layers.py:25-32) or sparse (layers.py:105-122) layer, no
    activation; an edgeless row is NaN. ``el`` has rows of the CSR (indexed by the global
    row id), ``er`` rows of the columns."""
    lib = load()
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    wh = np.ascontiguousarray(wh, dtype=np.float32)
    el = np.ascontiguousarray(el, dtype=np.float32)
    er = np.ascontiguousarray(er, dtype=np.float32)
    if el.shape[1] != heads or er.shape[1] != heads or wh.shape[1] != heads * fh:
        raise ValueError("el / er must be [*, heads], wh [*, heads * fh]")
    row1 = rowptr.size - 1 if row1 is None else row1
    y = np.empty((row1 - row0, heads * fh), dtype=np.float32)
    # one row stride for el and er: the wider of the two is not needed (both are [*, heads])
    lib.oracle_gat_csr(rowptr.ctypes.data, col.ctypes.data, row0, row1, wh.ctypes.data,
                       wh.shape[1], el.ctypes.data, er.ctypes.data, heads, heads, fh,
                       float(slope), int(bool(sparse)), y.ctypes.data, heads * fh)
    return y


_SAGE_MODES = {"MEAN": 0, "SUM": 2, "MAXPOOL": 3}


def sage_argmax(table, idx):
    """int64 [M, F] argmax over k of table[idx[m, j]] (Aggregator 'MAX', graph_utils.py:7-8:
    torch.argmax order -- NaN largest, first index on ties)."""
    lib = load()
    table = np.ascontiguousarray(table, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    M, k = idx.shape
    F = table.shape[1]
    out = np.empty((M, F), dtype=np.int64)
    if k:
        lib.oracle_sage_argmax(table.ctypes.data, F, idx.ctypes.data, k, M, k, F, out.ctypes.data,
                               F)
    return out


def sage_gather(table, idx, mode: str = "MEAN"):
    """fp32 [M, F] reduce over k of table[idx[m, j]] (float64 inside): MEAN, SUM or
    MAXPOOL (torch.max(dim=1).values, NaN-propagating)."""
    lib = load()
    table = np.ascontiguousarray(table, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    M, k = idx.shape
    F = table.shape[1]
    out = np.empty((M, F), dtype=np.float32)
    lib.oracle_sage_gather(table.ctypes.data, F, idx.ctypes.data, k, M, k, F, _SAGE_MODES[mode],
                           out.ctypes.data, F)
    return out


def gat_block_grad(rowptr, col, x, W, a_src, a_dst, gy, heads: int, fh: int, slope: float,
                   sparse: bool, elu: bool = True, drop_p: float = 0.0, drop_seed: int = 0):
    """float64 forward + backward of the H-head GAT attention block (GAT/models/GAT.py:16 over
    GAT/models/layers.py:22-37 / :94-131, all heads concatenated) for the loss sum(out * gy):
    Wh = x W in float64, the C restatement of the aggregation and its gradients
    (oracle_gat_block_grad), then dW = x^T dWh, d a_src / d a_dst per head and dx = dWh W^T.
    Dropout masks re-derived from the HIP kernels' (seed, edge, head) hash. Returns a dict of
    float64 arrays: out, dW, da_src, da_dst, dx, dwh, del, der, and ``slack_*`` for dwh, dW,
    da_src, da_dst, dx: the per-element bound on how far an fp32 implementation may move from
    these values by taking the other LeakyReLU' branch on edges whose t_ij is within rounding
    of the kink at 0 (oracle_gat_block_grad's kink_del / kink_der, propagated with absolute
    values); zero where no such edge contributes."""
    lib = load()
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    x64 = np.asarray(x, dtype=np.float64)
    W64 = np.asarray(W, dtype=np.float64)
    n, F = x64.shape[0], heads * fh
    wh = np.ascontiguousarray(x64 @ W64)
    wh_abs = np.ascontiguousarray(np.abs(x64) @ np.abs(W64))
    a_s = np.ascontiguousarray(a_src, dtype=np.float32)
    a_d = np.ascontiguousarray(a_dst, dtype=np.float32)
    g = np.ascontiguousarray(gy, dtype=np.float32)
    out = np.empty((n, F))
    dwh = np.empty((n, F))
    dl = np.empty((n, heads))
    der = np.empty((n, heads))
    kdl = np.empty((n, heads))
    kdr = np.empty((n, heads))
    rc = lib.oracle_gat_block_grad(rowptr.ctypes.data, col.ctypes.data, n, wh.ctypes.data,
                                   wh_abs.ctypes.data, a_s.ctypes.data, a_d.ctypes.data, g.ctypes.data, heads, fh,
                                   float(slope), int(bool(sparse)), int(bool(elu)), float(drop_p),
                                   int(drop_seed), out.ctypes.data, dwh.ctypes.data,
                                   dl.ctypes.data, der.ctypes.data, kdl.ctypes.data,
                                   kdr.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_gat_block_grad failed ({rc}: -1 edgeless row, -2 memory)")
    whh = wh.reshape(n, heads, fh)
    r = {"out": out, "dwh": dwh, "del": dl, "der": der, "dW": x64.T @ dwh,
         "da_src": np.einsum("nh,nhf->hf", dl, whh).reshape(-1),
         "da_dst": np.einsum("nh,nhf->hf", der, whh).reshape(-1), "dx": dwh @ W64.T,
         "kink_del": kdl, "kink_der": kdr}
    sdwh = (np.repeat(kdr, fh, axis=1) * np.abs(a_d.astype(np.float64)) +
            np.repeat(kdl, fh, axis=1) * np.abs(a_s.astype(np.float64)))
    awh = np.abs(whh)
    r.update(slack_dwh=sdwh, slack_dW=np.abs(x64).T @ sdwh, slack_dx=sdwh @ np.abs(W64).T,
             slack_da_src=np.einsum("nh,nhf->hf", kdl, awh).reshape(-1),
             slack_da_dst=np.einsum("nh,nhf->hf", kdr, awh).reshape(-1))
    return r


def dropout_keep(seed: int, rows, cols, p: float):
    """bool keep mask of the hashed element dropout (oracle_dropout_keep: csrc/common.hpp
    dropout_hash) for broadcastable int64 row / column ids -- GCN_Model's Dropout (GCN/GCN.py:14)
    as the fused training layer draws it."""
    lib = load()
    r, c = np.broadcast_arrays(np.asarray(rows, np.int64), np.asarray(cols, np.int64))
    r = np.ascontiguousarray(r)
    c = np.ascontiguousarray(c)
    out = np.empty(r.shape, np.uint8)
    lib.oracle_dropout_keep(int(seed) & (2 ** 64 - 1), r.ctypes.data, c.ctypes.data, r.size,
                            float(p), out.ctypes.data)
    return out.astype(bool)

