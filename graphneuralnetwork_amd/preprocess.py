"""Reference GCN adjacency preprocessing, on the device.

Restates the reference pipeline that feeds the SpMM
(GCN/data_utils.py:32-35 symmetrise, :78 ``+ sp.eye``, :54-60
``normalize_adj``, :63-70 fp32 COO) as sort/unique passes over int64 edge keys
resident in HBM, so a 100M-edge graph is prepared in seconds instead of the
reference's scipy minutes:

    A      = coo(ones(E), (src, dst))   duplicates summed        (:32-33)
    A_sym  = elementwise max(A, A^T)                             (:35)
    A_til  = A_sym + I                  float64                  (:78)
    d      = rowsum(A_til)^-1/2, inf -> 0                        (:55-57)
    A_hat[i, j] = (A_til[j, i] * d[i]) * d[j]  -> fp32           (:60, :65)

The structure is bit-exact with the reference and the values are computed in
float64 then rounded to fp32 exactly like scipy does (checked against the
reference-generated fixtures in tests/test_preprocess.py).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .graph import CsrGraph


def gcn_adjacency(src, dst, n: int, device=None) -> CsrGraph:
    """The reference GCN adjacency built by the HIP graph builder (graph_build.hip).

    Same result as :func:`gcn_normalized_csr` (bit-identical), as native
    sort / reduce passes on the device. Device tensors only."""
    src = torch.as_tensor(src, dtype=torch.int64, device=device).contiguous()
    dst = torch.as_tensor(dst, dtype=torch.int64, device=device).contiguous()
    if not src.is_cuda:
        raise RuntimeError("gcn_adjacency runs on the ROCm device (no CPU fallback)")
    if src.shape != dst.shape:
        raise ValueError("src and dst must have the same length")
    lib = _lib.load()
    e = src.numel()
    nbytes = int(lib.gnn_gcn_adjacency_workspace_bytes(e, n))
    if nbytes < 0:
        _lib.check(nbytes, "gnn_gcn_adjacency_workspace_bytes")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=src.device)
    nnz = ctypes.c_int64(0)
    stream = _lib.stream_handle(src.device)
    rc = lib.gnn_gcn_adjacency_build(src.data_ptr() if e else None, dst.data_ptr() if e else None,
                                     e, n, ws.data_ptr(), nbytes, ctypes.byref(nnz), stream)
    if rc == -1 and e:
        raise IndexError("edge endpoint out of range")
    _lib.check(rc, "gnn_gcn_adjacency_build")
    m = int(nnz.value)
    rowptr = torch.empty(n + 1, dtype=torch.int64, device=src.device)
    col = torch.empty(m, dtype=torch.int32, device=src.device)
    val = torch.empty(m, dtype=torch.float32, device=src.device)
    _lib.check(lib.gnn_gcn_adjacency_fill(ws.data_ptr(), e, n, m, rowptr.data_ptr(),
                                          col.data_ptr(), val.data_ptr(), stream),
               "gnn_gcn_adjacency_fill")
    # D^-1/2 (max(A, A^T) + I) D^-1/2: symmetric in structure; v_ij and v_ji are the same
    # float64 product in two orders, equal after the fp32 rounding to within one ulp
    return CsrGraph(rowptr, col, val, n, n, symmetric=True)


def gcn_normalized_csr(src, dst, n: int, device=None) -> CsrGraph:
    """CSR of D^-1/2 (A_sym + I)^T D^-1/2 for a directed edge list (src -> dst).

    torch sort/unique formulation (runs on CPU tensors too: the CPU tests and
    the oracle cross-check use it); the device path of record is gcn_adjacency."""
    src = torch.as_tensor(src, dtype=torch.int64, device=device)
    dst = torch.as_tensor(dst, dtype=torch.int64, device=device)
    dev = src.device
    if src.numel() and (int(src.min()) < 0 or int(src.max()) >= n or int(dst.min()) < 0
                        or int(dst.max()) >= n):
        raise IndexError("edge endpoint out of range")
    # A: duplicate edges summed (counts are exact in the reference's fp32)
    key, cnt = torch.unique(src * n + dst, return_counts=True)
    r, c = key // n, key % n
    del src, dst
    # A_sym = max(A, A^T)
    k2 = torch.cat([key, c * n + r])
    v2 = torch.cat([cnt, cnt]).to(torch.float64)
    del key, cnt, r, c
    key, inv = torch.unique(k2, return_inverse=True)
    w = torch.zeros(key.numel(), dtype=torch.float64, device=dev)
    w.scatter_reduce_(0, inv, v2, reduce="amax", include_self=False)
    del k2, v2, inv
    # + I (float64): every key is unique on both sides, so plain scatters (no atomics)
    diag = torch.arange(n, dtype=torch.int64, device=dev) * (n + 1)
    merged = torch.unique(torch.cat([key, diag]))
    w3 = torch.zeros(merged.numel(), dtype=torch.float64, device=dev)
    w3[torch.searchsorted(merged, key)] = w
    pd = torch.searchsorted(merged, diag)
    w3[pd] = w3[pd] + 1.0
    del key, w, diag, pd
    r, c = merged // n, merged % n
    del merged
    # rowsum(A_til): keys are row-major sorted -> one segmented sum per row
    offs = torch.searchsorted(r, torch.arange(n + 1, dtype=torch.int64, device=dev))
    rowsum = torch.segment_reduce(w3, "sum", offsets=offs)
    w = w3
    d = rowsum.pow(-0.5)
    d[torch.isinf(d)] = 0.0
    # transpose: output row = c, gathered col = r
    val = ((w * d[c]) * d[r]).to(torch.float32)
    order = torch.argsort(c * n + r)
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(torch.bincount(c, minlength=n), 0, out=rowptr[1:])
    return CsrGraph(rowptr, r[order].to(torch.int32).contiguous(), val[order].contiguous(), n, n,
                    symmetric=True)


def normalize_features(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Row-normalised features as the reference loader produces them: normalize_features
    (GCN/data_utils.py:39-51) on sp.csr_matrix(x, float32), then
    torch.Tensor(features.toarray()) (:81-83) -- bit for bit (gnn_normalize_features_f32,
    features.hip: numpy's float32 pairwise row sum over the nonzeros, a float64 reciprocal
    with inf -> 0, float64 products rounded to fp32). ``x``: device float32 [N, F]
    (F <= 16384); ``out`` must not overlap it."""
    if not x.is_cuda:
        raise RuntimeError("normalize_features runs on the GPU (HIP); got a CPU tensor")
    if x.dtype != torch.float32 or x.dim() != 2:
        raise ValueError("x must be a float32 [N, F] tensor")
    if x.stride(1) != 1:
        x = x.contiguous()
    if out is None:
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    elif out.shape != x.shape or out.dtype != torch.float32 or out.stride(1) != 1:
        raise ValueError("out must be float32 with x's shape and unit column stride")
    lib = _lib.load()
    _lib.check(lib.gnn_normalize_features_f32(x.data_ptr(), x.stride(0), x.shape[0], x.shape[1],
                                              out.data_ptr(), out.stride(0),
                                              _lib.stream_handle(x.device)),
               "gnn_normalize_features_f32")
    return out

