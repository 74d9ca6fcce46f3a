"""Device ops over the C-ABI: every call launches hand-written gfx950 kernels.

No op here has a CPU path: tensors must live on a ROCm device and the HIP
library must be loadable, otherwise a RuntimeError is raised.
"""
from __future__ import annotations

import torch

from . import _lib
from .graph import CsrGraph, seg_len_for

_ACT_FLAGS = {None: 0, "relu": _lib.EPI_RELU, "elu": _lib.EPI_ELU}


def _require_device(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "graphneuralnetwork_amd ops run only on a ROCm (MI355X) device tensor; "
                f"got a tensor on {t.device}. There is no CPU fallback.")


def _rows_f32(x: torch.Tensor, name: str) -> torch.Tensor:
    if x.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {x.dtype})")
    if x.dim() != 2:
        raise ValueError(f"{name} must be 2-D [rows, features]")
    if x.stride(1) != 1:
        x = x.contiguous()
    return x


def spmm_forward(g: CsrGraph, x: torch.Tensor, bias: torch.Tensor | None = None,
                 activation: str | None = None, out: torch.Tensor | None = None,
                 seg_len: int | None = None) -> torch.Tensor:
    """Y = A.X (+ bias) (act) with A in CSR -- the GCN aggregation (GCN/GCN.py:43-45).

    ``seg_len`` overrides the long-row threshold (rows with more edges are split
    across wavefronts); by default it is sized from the feature width.
    """
    _require_device(g.rowptr, x, bias, out)
    x = _rows_f32(x, "X")
    if x.shape[0] != g.n_cols:
        raise ValueError(f"X has {x.shape[0]} rows, adjacency has {g.n_cols} columns")
    feat = x.shape[1]
    if bias is not None:
        bias = bias.contiguous()
        if bias.dtype != torch.float32 or bias.numel() != feat:
            raise ValueError("bias must be float32 [features]")
    if out is None:
        out = torch.empty((g.n_rows, feat), dtype=torch.float32, device=x.device)
    elif out.shape != (g.n_rows, feat) or out.stride(1) != 1 or out.dtype != torch.float32:
        raise ValueError("out must be float32 [n_rows, features] with unit column stride")
    if g.n_rows == 0 or feat == 0:
        return out
    plan = g.plan(seg_len if seg_len is not None else seg_len_for(feat))
    partial = None
    if plan.n_seg:
        partial = torch.empty((plan.n_seg, feat), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    rc = lib.gnn_spmm_csr_f32(
        g.rowptr.data_ptr(), g.col.data_ptr(), g.val.data_ptr(), g.n_rows,
        x.data_ptr(), x.stride(0), feat, _lib.ptr(bias), out.data_ptr(), out.stride(0),
        plan.seg_len, _lib.ptr(plan.seg_row), _lib.ptr(plan.seg_begin), plan.n_seg,
        _lib.ptr(plan.long_row), plan.long_seg_ptr.data_ptr(), plan.n_long, _lib.ptr(partial),
        _ACT_FLAGS[activation], _lib.stream_handle(x.device))
    _lib.check(rc, "gnn_spmm_csr_f32")
    return out


class _SpmmFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, g):
        ctx.g = g
        ctx.has_bias = bias is not None
        return spmm_forward(g, x, bias)

    @staticmethod
    def backward(ctx, gy):
        g = ctx.g
        gx = gb = None
        if ctx.needs_input_grad[0]:
            gx = spmm_forward(g.transpose(), gy.contiguous())  # dX = A^T dY (same kernel)
        if ctx.has_bias and ctx.needs_input_grad[1]:
            gb = gy.sum(0)
        return gx, gb, None


def spmm(g: CsrGraph, x: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Differentiable (w.r.t. X and bias) CSR SpMM on the device."""
    if torch.is_grad_enabled() and (x.requires_grad or (bias is not None and bias.requires_grad)):
        return _SpmmFn.apply(x, bias, g)
    return spmm_forward(g, x, bias)
