"""Device ops over the C-ABI: every call launches hand-written gfx950 kernels.

No op here has a CPU path: tensors must live on a ROCm device and the HIP
library must be loadable, otherwise a RuntimeError is raised.
"""
from __future__ import annotations

import contextlib

import torch

from . import _lib
from .graph import GAT_SEG_BYTES, CsrGraph, seg_len_for, staged_plan

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


# Hub staging (gnn_spmm_csr_hub_f32 / gnn_gat_csr_hub_f32): when the gathered table is
# too large to stay in the Infinity Cache, its highest-degree rows (at most HUB_ROWS rows,
# at most HUB_BYTES) are copied into one compact table per call. A/B on MI355X
# (tools/hub_ab.py, profiles/r01f_hub_ab_*.log): SpMM 10M/207M F=128 20.9 -> 14.4 ms
# (best 64-128 Ki rows), F=256 40.0 -> 30.0 ms (flat 32-128 Ki rows); 1M/20M F=128
# 1.57 -> 1.16 ms (flat 8-128 Ki rows), F=64 0.71 -> 0.59 ms (best 64 Ki rows); GAT
# 8x8 heads on 1M/20M 1.00 -> 0.94-0.95 ms (best 16-64 Ki rows); a 128 MB table (F=32)
# gains ~1 % and a 64 MB one (F=16) loses ~2 %, hence the size threshold.
HUB_MIN_X_BYTES = 192 << 20
HUB_BYTES = 64 << 20
HUB_ROWS = 131072


def hub_rows_for(n_cols: int, feat: int) -> int:
    """Default number of staged hub rows for a gathered table of n_cols x feat fp32
    (0 = no staging)."""
    if n_cols * 4 * feat < HUB_MIN_X_BYTES:
        return 0
    return min(n_cols, HUB_ROWS, max(1, HUB_BYTES // (4 * feat)))


# XCD-sliced hub staging (graph.XcdHubPlan): on graphs with at least XCD_MIN_NNZ stored
# entries whose X would be hub-staged, the hub edges of rows of degree >= XCD_MIN_DEG are
# reduced per (row, XCD slice) first, so each XCD's L2 serves 1/8 of the hub table.
# Measured with tools/workingset_probe.py and tools/xcd_hub_probe.py (profiles/r02y_*):
# a gather set that fits one XCD's L2 runs at ~50 G rows/s, 16-256 MiB sets at 14-19 (the
# Infinity Cache hardly beats HBM's 12); emulated, cfg2 1.14 -> 0.96 ms and the north star
# 14.4 -> 12.4 ms at 256 Ki hub rows, degree >= 128, items of <= 128 edges.
XCD_MIN_NNZ = 4_000_000
XCD_HUB_BYTES = 128 << 20
XCD_HUB_ROWS = 262144
XCD_MIN_DEG = 128
XCD_CHUNK = 128
XCD_PHASES = 1  # slices per XCD, run one after another (graph.xcd_hub_coo ``phases``)
XCD_ITEM_ROWS = None  # items read only the hottest XCD_ITEM_ROWS hub rows (None: all K)
# rows below XCD_MIN_DEG get items too, for each slice holding >= XCD_SMALL_ITEM of their hub
# edges (None: off; graph.xcd_hub_coo ``small_item``)
XCD_SMALL_ITEM = None
# on a degree-ordered graph (graph.degree_order) the hub rows are X's first rows: read them
# in place instead of copying them into a staged table (XcdHubPlan.prefix / direct)
XCD_DIRECT = True


def xcd_hub_rows_for(n_cols: int, feat: int) -> int:
    """Default hub rows of the XCD-sliced staging (0 = X too small to stage)."""
    if n_cols * 4 * feat < HUB_MIN_X_BYTES:
        return 0
    return min(n_cols, XCD_HUB_ROWS, max(64, XCD_HUB_BYTES // (4 * feat)))


# Packed row tasks (gnn_spmm_csr_tasks_f32, spmm.hip packed_rows): rows of degree <=
# TASK_MAX_DEG are streamed a task (<= 63 consecutive rows, ~TASK_COST edges + rows) per wave
# instead of one wave per row, so the rowptr -> col -> X chain of short rows is paid once per
# task. Needs the 16-B vector path. Narrow rows (feat <= 32: LPR <= 8 lanes per row, 8 or more
# edge slots per wave) take tasks of up to TASK_COST_NARROW edges + rows, so that every slot of
# the wave gets rows (one wave per row left most of its lanes idle at feat 8).
SPMM_TASKS = True
SPMM_TASKS_NARROW = True
TASK_MAX_DEG = 128
TASK_COST = 128  # 256 until late round 4: 128 is 0.7 % faster with the slice groups (cfg2, north star)
TASK_COST_NARROW = 2048


def _task_cost(feat: int) -> int:
    return TASK_COST_NARROW if feat <= 32 else TASK_COST


def _tasks_ok(feat: int, *ts) -> bool:
    # every column block of the launch (<= 2048 wide) must be a vector block; one of 32 or
    # fewer columns only with the narrow tasks
    if not SPMM_TASKS or feat % 4 or (not SPMM_TASKS_NARROW and (feat <= 32
                                                                  or 0 < feat % 2048 <= 32)):
        return False
    return all(t is None or (t.data_ptr() % 16 == 0 and (t.dim() == 1 or t.stride(0) % 4 == 0))
               for t in ts)


def _spmm_tasks_call(lib, g: CsrGraph, col: torch.Tensor, tp, x, xh, feat, bias, y, ldy,
                     partial, flags, stream, what):
    _lib.check(lib.gnn_spmm_csr_tasks_f32(
        g.rowptr.data_ptr(), col.data_ptr(), g.val.data_ptr(), g.n_rows, x.data_ptr(),
        x.stride(0), _lib.ptr(xh), xh.stride(0) if xh is not None else 0, feat, _lib.ptr(bias),
        y.data_ptr(), ldy, tp.seg_len, *tp.args(), _lib.ptr(partial), flags, stream), what)


def _spmm_hub_call(lib, g: CsrGraph, col: torch.Tensor, plan, pargs, x, xh, feat, bias, y, ldy,
                   partial, flags, stream, what):
    _lib.check(lib.gnn_spmm_csr_hub_f32(
        g.rowptr.data_ptr(), col.data_ptr(), g.val.data_ptr(), g.n_rows, x.data_ptr(),
        x.stride(0), xh.data_ptr(), xh.stride(0), feat, _lib.ptr(bias), y.data_ptr(), ldy,
        plan.seg_len, *pargs, _lib.ptr(partial), flags, stream), what)


def spmm_forward(g: CsrGraph, x: torch.Tensor, bias: torch.Tensor | None = None,
                 activation: str | None = None, out: torch.Tensor | None = None,
                 seg_len: int | None = None, accumulate: bool = False,
                 hubs: int | None = None, xcd: bool | None = None) -> torch.Tensor:
    """Y = A.X (+ bias) (act) with A in CSR -- the GCN aggregation (GCN/GCN.py:43-45).

    ``accumulate=True`` adds into ``out`` (Y = out + A.X ...): the halo pass of
    the multi-GPU edge-cut aggregation.

    ``seg_len`` overrides the long-row threshold (rows with more edges are split
    across wavefronts); by default it is sized from the feature width.

    ``hubs`` = number of highest-degree rows of X staged into a compact table before
    the gather (0: none; default ``hub_rows_for``). It changes speed, not results: the
    output is bit-identical to the unstaged kernel's.

    ``xcd`` = XCD-sliced hub staging (``graph.XcdHubPlan``; default: on for graphs of at
    least XCD_MIN_NNZ entries whose X is staged and no explicit ``hubs``). Same sums,
    regrouped: equal to the unstaged result to fp32 rounding, bitwise reproducible.
    """
    if accumulate and out is None:  # checked first: it is a usage error on any device
        raise ValueError("accumulate=True needs `out` (it adds into the caller's buffer)")
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
    seg = seg_len if seg_len is not None else seg_len_for(feat)
    if x.numel() == 0:  # no column to gather from (e.g. an empty halo): never read
        x = torch.empty((1, feat), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    flags = _ACT_FLAGS[activation] | (_lib.EPI_ACCUMULATE if accumulate else 0)
    stream = _lib.stream_handle(x.device)
    # out += A.X with no bias / activation: rows without edges stay as they are
    skip_empty = accumulate and bias is None and activation is None
    if xcd is None:
        xcd = hubs is None and g.nnz >= XCD_MIN_NNZ and xcd_hub_rows_for(g.n_cols, feat) > 0
    if xcd and g.nnz:
        kx = xcd_hub_rows_for(g.n_cols, feat) if hubs is None else min(int(hubs), g.n_cols)
        chunk = min(XCD_CHUNK, seg)
        xp = (g.xcd_hub_plan(kx, XCD_MIN_DEG, chunk, XCD_PHASES, XCD_ITEM_ROWS, XCD_SMALL_ITEM)
              if kx >= 8 * XCD_PHASES and chunk >= 4 else None)
        if xp is not None:
            _spmm_xcd(lib, g, xp, x, feat, bias, out, seg, skip_empty, flags, stream)
            return out
    plan = g.plan(seg)
    partial = None
    if plan.n_seg:
        partial = torch.empty((plan.n_seg, feat), dtype=torch.float32, device=x.device)
    pargs = plan.args(skip_empty=skip_empty)
    k = hub_rows_for(g.n_cols, feat) if hubs is None else min(int(hubs), g.n_cols)
    tasks = _tasks_ok(feat, x, out, bias, partial)
    if k > 0 and g.nnz:
        hp = g.hub_plan(k)
        if XCD_DIRECT and hp.prefix:  # degree-ordered columns: the hub rows are X's first rows
            xh = x
        else:
            xh = torch.empty((hp.k, feat), dtype=torch.float32, device=x.device)
            _lib.check(lib.gnn_gather_rows_f32(x.data_ptr(), x.stride(0), x.shape[0],
                                               hp.hub_ids.data_ptr(), hp.k, feat, xh.data_ptr(),
                                               feat, hp.err.data_ptr(), stream),
                       "gnn_gather_rows_f32")
        if tasks:
            gh = CsrGraph(g.rowptr, hp.col_hub, g.val, g.n_rows, g.n_cols)
            _spmm_tasks_call(lib, gh, hp.col_hub,
                             g.task_plan(seg, TASK_MAX_DEG, _task_cost(feat)), x,
                             xh, feat, bias, out, out.stride(0), partial,
                             flags | (_lib.EPI_SKIP_EMPTY if skip_empty else 0), stream,
                             "gnn_spmm_csr_tasks_f32 (hub)")
            return out
        rc = lib.gnn_spmm_csr_hub_f32(
            g.rowptr.data_ptr(), hp.col_hub.data_ptr(), g.val.data_ptr(), g.n_rows,
            x.data_ptr(), x.stride(0), xh.data_ptr(), xh.stride(0), feat, _lib.ptr(bias),
            out.data_ptr(), out.stride(0), plan.seg_len, *pargs, _lib.ptr(partial), flags, stream)
        _lib.check(rc, "gnn_spmm_csr_hub_f32")
        return out
    if tasks and g.nnz:
        _spmm_tasks_call(lib, g, g.col, g.task_plan(seg, TASK_MAX_DEG, _task_cost(feat)), x,
                         None, feat,
                         bias, out, out.stride(0), partial,
                         flags | (_lib.EPI_SKIP_EMPTY if skip_empty else 0), stream,
                         "gnn_spmm_csr_tasks_f32")
        return out
    rc = lib.gnn_spmm_csr_f32(
        g.rowptr.data_ptr(), g.col.data_ptr(), g.val.data_ptr(), g.n_rows,
        x.data_ptr(), x.stride(0), feat, _lib.ptr(bias), out.data_ptr(), out.stride(0),
        plan.seg_len, *pargs, _lib.ptr(partial), flags, stream)
    _lib.check(rc, "gnn_spmm_csr_f32")
    return out


def _spmm_xcd(lib, g: CsrGraph, xp, x, feat, bias, out, seg, skip_empty, flags, stream):
    """The XCD-sliced hub SpMM: hub rows -> staged buffer, pass 1 (items -> partial rows of
    the same buffer, workgroup w on XCD w % 8 holds only slice w % 8), pass 2 (remaining
    edges + partial refs, with the epilogue). Three launches on one stream."""
    k, n_pos = xp.k, xp.n_pos
    if XCD_DIRECT and xp.prefix:
        _spmm_xcd_direct(lib, xp, x, feat, bias, out, seg, skip_empty, flags, stream)
        return
    buf = torch.empty((k + n_pos, feat), dtype=torch.float32, device=x.device)
    hp = xp.hub
    _lib.check(lib.gnn_gather_rows_f32(x.data_ptr(), x.stride(0), x.shape[0],
                                       hp.hub_ids.data_ptr(), k, feat, buf.data_ptr(), feat,
                                       hp.err.data_ptr(), stream), "gnn_gather_rows_f32")
    p1 = xp.items.plan(seg)
    if p1.n_seg or p1.n_small:  # by construction every item is a 2..chunk-edge row
        raise RuntimeError("XCD hub plan: item rows outside the mid-row class")
    _spmm_hub_call(lib, xp.items, xp.items.col, p1, p1.args(), x, buf, feat, None, buf[k:], feat,
                   None, 0, stream, "gnn_spmm_csr_hub_f32 (xcd items)")
    if _tasks_ok(feat, x, out, bias, buf):
        tp = xp.rest.task_plan(seg, TASK_MAX_DEG, _task_cost(feat))
        partial = None
        if tp.base.n_seg:
            partial = torch.empty((tp.base.n_seg, feat), dtype=torch.float32, device=x.device)
        _spmm_tasks_call(lib, xp.rest, xp.rest.col, tp, x, buf, feat, bias, out, out.stride(0),
                         partial, flags | (_lib.EPI_SKIP_EMPTY if skip_empty else 0), stream,
                         "gnn_spmm_csr_tasks_f32 (xcd rest)")
        return
    p2 = xp.rest_plan(seg)
    partial = None
    if p2.n_seg:
        partial = torch.empty((p2.n_seg, feat), dtype=torch.float32, device=x.device)
    _spmm_hub_call(lib, xp.rest, xp.rest.col, p2, p2.args(skip_empty=skip_empty), x, buf, feat,
                   bias, out, out.stride(0), partial, flags, stream,
                   "gnn_spmm_csr_hub_f32 (xcd rest)")


# Graph_conv_layer runs its aggregation over the column-degree-ordered graph A P^T
# (graph.degree_order(rows=False)) whenever the SpMM would take the XCD-sliced path: the
# transform writes the support rows in that order (gcn_transform rows=perm) and the SpMM reads
# the hub rows in place (no staging copy). Output rows stay in the original order.
DEGREE_ORDER = True


# None: every column ranked by in-degree; an int: only that many hub columns ranked first, the
# rest in id order (graph.degree_order ``prefix``), so the scattered-row producers (transform /
# projection) store the non-hub rows in ascending order. Must be >= every hub count K taken
# from the order (XCD_HUB_ROWS, HUB_ROWS).
COLUMN_ORDER_PREFIX = None


def _cached_column_order(g: CsrGraph):
    prefix = COLUMN_ORDER_PREFIX
    if prefix is not None and prefix < max(XCD_HUB_ROWS, HUB_ROWS):
        raise ValueError("COLUMN_ORDER_PREFIX must cover the hub rows (XCD_HUB_ROWS, HUB_ROWS)")
    key = ("_colorder",) if prefix is None else ("_colorder", prefix)
    o = g._plans.get(key)
    if o is None:
        from .graph import degree_order
        o = g._plans[key] = degree_order(g, rows=False, prefix=prefix)
    return o


def column_order(g: CsrGraph, feat: int):
    """The cached ``DegreeOrder(rows=False)`` of ``g`` when a feat-wide SpMM over it would
    take the XCD-sliced hub path (else None)."""
    if not (DEGREE_ORDER and XCD_DIRECT) or g.nnz < XCD_MIN_NNZ or g._plans.get("_degree_ordered"):
        return None
    if xcd_hub_rows_for(g.n_cols, feat) < 8 * XCD_PHASES:
        return None
    return _cached_column_order(g)


def gat_column_order(g: CsrGraph, heads: int, fh: int):
    """The cached ``DegreeOrder(rows=False)`` of ``g`` when the GAT aggregation over it would
    stage hub rows of Wh / er (``hub_rows_for``; else None): over A P^T those rows are the
    first rows of the projection's column-ordered output, read in place."""
    if not (DEGREE_ORDER and XCD_DIRECT) or g.nnz == 0 or g._plans.get("_degree_ordered"):
        return None
    if hub_rows_for(g.n_cols, heads * fh + heads) == 0:
        return None
    return _cached_column_order(g)


# Training (forward + backward) over P A P^T: every node relabelled once by degree, so the hub
# rows of every gathered table (X / S, Wh / er, dY / dout) are its first rows in the forward and
# in both backward passes, read in place (XCD-direct hub plans, no staging copy). The models
# (GATBase.forward, GCN_Model.forward) permute their input once on entry and the logits once
# on exit. cfg3 8-head GAT block: 3.89 -> 3.41 ms, node pass 1.16 -> 0.84 ms
# (profiles/r06c_gat_order_ab.log, tools/gat_order_ab.py).
GAT_TRAIN_ORDER = True
GCN_TRAIN_ORDER = True


def node_order(g: CsrGraph):
    """The cached ``DegreeOrder(rows=True)`` of a symmetric square graph: P A P^T, itself
    symmetric (marked so: backward passes walk it as its own transpose) and marked
    ``_degree_ordered`` (column_order / gat_column_order then return None for it: its hub rows
    already lead every table). Each row's edges keep their CSR order, renamed: the row sums run
    in the same order as over A."""
    o = g._plans.get(("_nodeorder",))
    if o is None:
        from .graph import degree_order
        o = degree_order(g, rows=True)
        o.graph.symmetric = True  # P A P^T of a symmetric A
        o.graph._plans["_degree_ordered"] = True
        g._plans[("_nodeorder",)] = o
    return o


# GCN_Model in training: a first layer over input features that need no gradient reads X in
# its original row order through P A (rows relabelled, column ids as in A) instead of
# permuting X onto P A P^T first (one [n, F] gather pass fewer; its SpMM stages the hub rows)
GCN_FIRST_ROWS = True


def row_order_graph(g: CsrGraph) -> CsrGraph:
    """P A for ``node_order(g)``'s P: row i is A's row perm[i] with its edges as in A (column ids
    not renamed), cached on g. A layer over it maps X in the original order to output rows in
    the degree order."""
    rg = g._plans.get(("_nodeorder_rows",))
    if rg is None:
        o = node_order(g)
        n = g.n_rows
        deg = g.rowptr[1:] - g.rowptr[:-1]
        nd = deg.index_select(0, o.perm)
        rp = torch.zeros(n + 1, dtype=torch.int64, device=g.rowptr.device)
        torch.cumsum(nd, 0, out=rp[1:])
        src = torch.repeat_interleave(g.rowptr[:-1].index_select(0, o.perm) - rp[:-1], nd,
                                      output_size=g.nnz)
        src += torch.arange(g.nnz, dtype=torch.int64, device=src.device)
        rg = CsrGraph(rp, g.col.index_select(0, src).contiguous(),
                      g.val.index_select(0, src).contiguous(), n, g.n_cols)
        del src
        g._plans[("_nodeorder_rows",)] = rg
    return rg


def _orderable(g: CsrGraph) -> bool:
    return (DEGREE_ORDER and g.nnz > 0 and g.symmetric and g.n_rows == g.n_cols
            and g.col.is_cuda and not g._plans.get("_degree_ordered"))


def gat_train_order(g: CsrGraph, heads: int, fh: int):
    """``node_order(g)`` when GAT training over it pays: a symmetric graph whose Wh / er table
    is large enough to stage hub rows (else None)."""
    if not (GAT_TRAIN_ORDER and _orderable(g)) or hub_rows_for(g.n_cols, heads * fh + heads) == 0:
        return None
    return node_order(g)


def gcn_train_order(g: CsrGraph, feat: int):
    """``node_order(g)`` when GCN training over it pays: a symmetric graph whose feat-wide
    SpMM takes the XCD-sliced hub path (else None)."""
    if not (GCN_TRAIN_ORDER and _orderable(g)) or column_order(g, feat) is None:
        return None
    return node_order(g)


def permute_rows(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """x[idx] for a 2-D fp32 device tensor and int64 row ids from a permutation, unchecked (no
    host read of the error flag: the training steps run it 2-4 times per step; the checked
    ``gather_rows`` below synced the host each time) (gnn_gather_rows_f32: 16-B row
    pieces per lane; torch's index_select moved the 1M x 128 permutation at ~1.7 TB/s,
    profiles/r06i_*); other inputs take index_select."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1
            and idx.dtype == torch.int64 and idx.is_cuda and idx.dim() == 1):
        return x.index_select(0, idx)
    idx = idx.contiguous()
    out = torch.empty((idx.numel(), x.shape[1]), dtype=torch.float32, device=x.device)
    err = _err_flag(x.device, False)  # ids come from a permutation: the flag is never read
    _lib.check(_lib.load().gnn_gather_rows_f32(x.data_ptr(), x.stride(0), x.shape[0],
                                               idx.data_ptr(), idx.numel(), x.shape[1],
                                               out.data_ptr(), out.stride(0), err.data_ptr(),
                                               _lib.stream_handle(x.device)),
               "gnn_gather_rows_f32")
    return out


class PermuteRows(torch.autograd.Function):
    """y = x[perm] with the gradient gathered back through inv (a permutation: no index_add):
    the models' one relabelling on entry to and exit from the degree-ordered graph."""

    @staticmethod
    def forward(ctx, x, perm, inv):
        ctx.inv = inv
        return permute_rows(x, perm)

    @staticmethod
    def backward(ctx, gy):
        return permute_rows(gy.contiguous(), ctx.inv), None, None


# F.dropout (GAT/models/GAT.py:15,17) in training as gnn_dropout_rows_f32: a hashed element mask
# that is never stored, fused with the entry relabelling where there is one. torch's dropout
# wrote a byte mask beside its output and read it back in the backward (~0.1 ms forward +
# ~0.08 ms backward per [1M, 64] at cfg3, profiles/r06y_*).
HASHED_DROPOUT = True


def dropout_rows(x: torch.Tensor, p: float, seed: int, idx: torch.Tensor | None = None,
                 key_by_source: bool = False) -> torch.Tensor:
    """out[i] = x[r] with r = idx[i] (or i), element (i, c) kept iff the (seed, key, c) hash clears
    p (key = r when ``key_by_source``, else i), kept values scaled by 1 / (1 - p). Unchecked ids
    (they come from a permutation)."""
    n = idx.numel() if idx is not None else x.shape[0]
    out = torch.empty((n, x.shape[1]), dtype=torch.float32, device=x.device)
    if idx is not None:
        idx = idx.contiguous()
    _lib.check(_lib.load().gnn_dropout_rows_f32(
        x.data_ptr(), x.stride(0), x.shape[0], idx.data_ptr() if idx is not None else None,
        int(key_by_source), n, x.shape[1], float(p), int(seed) & (2 ** 64 - 1), out.data_ptr(),
        out.stride(0), _err_flag(x.device, False).data_ptr(), _lib.stream_handle(x.device)),
        "gnn_dropout_rows_f32")
    return out


class DropoutRows(torch.autograd.Function):
    """y = dropout(x[perm]) (perm None: y = dropout(x)) with the hashed mask keyed by y's row; the
    gradient dx[j] = mask(inv[j]) dy[inv[j]] / (1 - p) re-derives the mask through inv."""

    @staticmethod
    def forward(ctx, x, p, seed, perm, inv):
        ctx.cfg = (p, seed, inv)
        return dropout_rows(x, p, seed, perm)

    @staticmethod
    def backward(ctx, gy):
        p, seed, inv = ctx.cfg
        gx = dropout_rows(gy.contiguous(), p, seed, inv, key_by_source=inv is not None)
        return gx, None, None, None, None


def hashed_dropout_ok(x: torch.Tensor, p: float) -> bool:
    """The hashed kernel takes F.dropout(x, p) in training: 2-D fp32 device rows with unit column
    stride, 0 < p < 1."""
    return (0.0 < p < 1.0 and HASHED_DROPOUT and x.dim() == 2 and x.is_cuda
            and x.dtype == torch.float32 and x.stride(1) == 1 and x.stride(0) >= x.shape[1])


def model_dropout(x: torch.Tensor, p: float, training: bool, perm=None, inv=None):
    """F.dropout(x[perm] or x, p, training) on the hashed kernel where it applies
    (``hashed_dropout_ok``), else PermuteRows + torch's dropout."""
    ok = training and hashed_dropout_ok(x, p)
    if not ok:
        if perm is not None:
            x = PermuteRows.apply(x, perm, inv)
        return torch.nn.functional.dropout(x, p, training=training)
    return DropoutRows.apply(x, p, dropout_seed(), perm, inv)


def _spmm_xcd_direct(lib, xp, x, feat, bias, out, seg, skip_empty, flags, stream):
    """The XCD-sliced SpMM of a degree-ordered graph (graph.degree_order): the hub rows are
    X's first k rows, so there is no staging copy. Pass 1 (plain kernel) reads the items'
    hub rows from X into a partial-row buffer; pass 2 reads X and that buffer (c < 0 ->
    partial row -1-c)."""
    items, rest = xp.direct()
    part = torch.empty((xp.n_pos, feat), dtype=torch.float32, device=x.device)
    p1 = items.plan(seg)
    if p1.n_seg or p1.n_small:
        raise RuntimeError("XCD hub plan: item rows outside the mid-row class")
    _lib.check(lib.gnn_spmm_csr_f32(
        items.rowptr.data_ptr(), items.col.data_ptr(), items.val.data_ptr(), items.n_rows,
        x.data_ptr(), x.stride(0), feat, None, part.data_ptr(), feat, p1.seg_len, *p1.args(),
        None, 0, stream), "gnn_spmm_csr_f32 (xcd direct items)")
    if _tasks_ok(feat, x, out, bias, part):
        tp = rest.task_plan(seg, TASK_MAX_DEG, _task_cost(feat))
        partial = None
        if tp.base.n_seg:
            partial = torch.empty((tp.base.n_seg, feat), dtype=torch.float32, device=x.device)
        _spmm_tasks_call(lib, rest, rest.col, tp, x, part, feat, bias, out, out.stride(0),
                         partial, flags | (_lib.EPI_SKIP_EMPTY if skip_empty else 0), stream,
                         "gnn_spmm_csr_tasks_f32 (xcd direct rest)")
        return
    p2 = staged_plan(rest, seg)
    partial = None
    if p2.n_seg:
        partial = torch.empty((p2.n_seg, feat), dtype=torch.float32, device=x.device)
    _lib.check(lib.gnn_spmm_csr_hub_f32(
        rest.rowptr.data_ptr(), rest.col.data_ptr(), rest.val.data_ptr(), rest.n_rows,
        x.data_ptr(), x.stride(0), part.data_ptr(), feat, feat, _lib.ptr(bias), out.data_ptr(),
        out.stride(0), p2.seg_len, *p2.args(skip_empty=skip_empty), _lib.ptr(partial), flags,
        stream), "gnn_spmm_csr_hub_f32 (xcd direct rest)")


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


def gemm_tn(a: torch.Tensor, b: torch.Tensor, d: torch.Tensor | None = None,
            trans: bool = False):
    """(A^T B, column sums of D) over the row axis (gnn_gemm_tn_f32): the weight / bias
    gradients of the training step. ``trans``: return (A^T B)^T = B^T A. None when the shape is
    not covered (the caller uses torch.mm)."""
    _require_device(a, b, d)
    if (a.dtype != torch.float32 or b.dtype != torch.float32 or a.dim() != 2 or b.dim() != 2
            or a.shape[0] != b.shape[0] or (d is not None and d.shape != b.shape)):
        return None
    n, m = a.shape
    k = b.shape[1]
    lib = _lib.load()
    kind = lib.gnn_gemm_tn_supported(m, k)  # 1 wide, 2 narrow (k <= 16: classifier layers)
    if not kind:
        return None

    def fits(t):
        if kind == 2:  # narrow shapes: any row stride, unit column stride
            return (t.stride(1) == 1 or t.shape[1] == 1) and t.data_ptr() % 4 == 0
        return t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0

    # a copy for an operand the kernel cannot read in place: clone, not .contiguous(), which
    # hands back a contiguous view at a misaligned storage offset unchanged
    ts = [t if fits(t) else t.clone(memory_format=torch.contiguous_format)
          for t in [a, b] + ([d] if d is not None else [])]
    if not all(fits(t) for t in ts):  # rows of a length the 16-B loads cannot take
        return None
    a, b = ts[0], ts[1]
    d = ts[2] if d is not None else None
    c = torch.empty((k, m) if trans else (m, k), dtype=torch.float32, device=a.device)
    dsum = torch.empty(k, dtype=torch.float32, device=a.device) if d is not None else None
    ws = torch.empty(int(lib.gnn_gemm_tn_workspace_bytes(n, m, k)), dtype=torch.uint8,
                     device=a.device)
    _lib.check(lib.gnn_gemm_tn_f32(a.data_ptr(), max(a.stride(0), m), b.data_ptr(),
                                   max(b.stride(0), k), n, m, k, c.data_ptr(), c.stride(0),
                                   1 if trans else 0, _lib.ptr(d),
                                   max(d.stride(0), k) if d is not None else 0, _lib.ptr(dsum),
                                   ws.data_ptr(), ws.numel(), _lib.stream_handle(a.device)),
               "gnn_gemm_tn_f32")
    return c, dsum


def gemm_tn_masked(a: torch.Tensor, b: torch.Tensor, h: torch.Tensor, scale: float,
                   want_dsum: bool, trans: bool = False):
    """(A^T B', column sums of B' if want_dsum) for B' = B . [H > 0] * scale
    (gnn_gemm_tn_masked_f32): the weight / bias gradients behind a fused ReLU + dropout epilogue
    whose output is H. Where the kernel does not take the shape, B' is formed with torch and
    handed to ``gemm_tn`` (None if that does not take it either)."""
    _require_device(a, b, h)
    lib = _lib.load()
    n, m = a.shape
    k = b.shape[1]
    ok = (a.dtype == b.dtype == h.dtype == torch.float32 and h.shape == b.shape
          and lib.gnn_gemm_tn_masked_supported(m, k)
          and all(t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0
                  for t in (a, b, h)))
    if not ok:
        bm = torch.where(h > 0, b * scale, torch.zeros((), dtype=b.dtype, device=b.device))
        return gemm_tn(a, bm, bm if want_dsum else None, trans=trans)
    c = torch.empty((k, m) if trans else (m, k), dtype=torch.float32, device=a.device)
    dsum = torch.empty(k, dtype=torch.float32, device=a.device) if want_dsum else None
    ws = torch.empty(int(lib.gnn_gemm_tn_workspace_bytes(n, m, k)), dtype=torch.uint8,
                     device=a.device)
    _lib.check(lib.gnn_gemm_tn_masked_f32(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                          h.data_ptr(), h.stride(0), float(scale), n, m, k,
                                          c.data_ptr(), c.stride(0), 1 if trans else 0,
                                          _lib.ptr(dsum), ws.data_ptr(), ws.numel(),
                                          _lib.stream_handle(a.device)), "gnn_gemm_tn_masked_f32")
    return c, dsum


LINEAR_SMALL_MAX_FOUT = 64  # widest output the k <= 16 kernel takes by default


def linear_small(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor | None:
    """x @ w^T with one narrow side (gnn_linear_small_f32: fout <= 16 on fp32 MFMA rows, or
    k <= 16 on a broadcast kernel) -- the classifier layer's support and its dX; None when the
    shape is not covered."""
    _require_device(x, w)
    if (x.dtype != torch.float32 or w.dtype != torch.float32 or x.dim() != 2 or w.dim() != 2
            or x.shape[1] != w.shape[1]):
        return None
    lib = _lib.load()
    fout, k = w.shape
    kind = lib.gnn_linear_small_supported(k, fout)
    # the broadcast kernel (k <= 16) beat hipBLASLt at fout 64 (GAT out_att dX: 0.055 vs 0.120
    # ms) but not at 128 inside the GCN_Model step (0.189 vs 0.146 ms,
    # profiles/r06y_gcn_model_train_step_kernel_stats.csv): 128 and 256 stay on torch.mm
    if not kind or (kind == 2 and fout > LINEAR_SMALL_MAX_FOUT):
        return None
    if x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
        # rows copied to a 16-B aligned pitch (a multiple of 4 floats >= k)
        xp = torch.empty((x.shape[0], k + (-k) % 4), dtype=torch.float32, device=x.device)
        xp[:, :k] = x
        x = xp[:, :k]
    w = w.contiguous()
    y = torch.empty((x.shape[0], fout + (-fout) % 4), dtype=torch.float32, device=x.device)
    _lib.check(lib.gnn_linear_small_f32(x.data_ptr(), x.stride(0), x.shape[0], k, w.data_ptr(),
                                        fout, y.data_ptr(), y.stride(0),
                                        _lib.stream_handle(x.device)), "gnn_linear_small_f32")
    return y[:, :fout] if y.shape[1] != fout else y


def _transform_or_mm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x @ w^T: the MFMA transform where it covers the shape, the narrow kernels where one side
    is narrow (linear_small), else torch.mm (hipBLASLt)."""
    y = gcn_transform(x, w)
    if y is None:
        y = linear_small(x, w)
    return y if y is not None else torch.mm(x, w.t())


# A layer with in_features <= out_features trains as (A X) W^T + b: the same product as the
# reference's A (X W^T) + b (GCN/GCN.py:42-45), reassociated. The SpMM then gathers rows of X
# instead of the support (no wider), and the backward needs dY and Z = A X only: dW = dY^T Z
# and db = sum dY come out of ONE gemm_tn pass over (Z, dY) (dY read once, not next to dS and
# X), and where X needs no gradient -- a first layer over the input features -- the backward
# runs no SpMM at all (the A (X W^T) form needs dS = A^T dY for dW regardless).
GCN_REASSOC = True
# the A (X W^T) form zero-pads an output width below 64 to a multiple of 4 (see _GcnLayerFn)
GCN_PAD_NARROW = True


# The reassociated backward's dW / db pass (gemm_tn over Z and dY) and its dX chain (transform
# dZ = dY W, then the SpMM A^T dZ) read the same dY and nothing of each other: when X needs a
# gradient the weight pass runs on a side stream beside the chain (the SpMM is bound by gather
# latency and leaves the matrix cores and VALUs idle).
GCN_OVERLAP_DW = True  # tools/train_step_probe.py --set: 2.49-2.53 vs 2.51-2.64 ms at cfg2
_SIDE_STREAMS: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return s


def _reassociate(x, weight, g) -> bool:
    fout, fin = weight.shape
    return GCN_REASSOC and fin <= fout and x.shape[0] == g.n_cols


# GCN_Model's Graph_conv_layer -> ReLU -> Dropout run in training as ONE op when the layer takes
# the (A X) W^T + b form: ReLU and dropout in the transform's store epilogue, their backward
# folded into the weight-gradient pass (gemm_tn_masked) -- two elementwise passes forward and
# two backward fewer over the [n, hidden] activations
GCN_FUSE_RELU_DROPOUT = True


def fuses_relu_dropout(x, weight, g) -> bool:
    """Whether ``gcn_layer(..., relu_dropout=...)`` applies to this layer: the reassociated form
    (``_reassociate``) on a shape the MFMA transform takes."""
    fout, fin = weight.shape
    return (GCN_FUSE_RELU_DROPOUT and _reassociate(x, weight, g)
            and bool(_lib.load().gnn_gcn_transform_supported(fin, fout)))


def dropout_seed() -> int:
    """A 62-bit seed for the HIP kernels' hashed dropout, drawn from torch's CPU generator (so
    torch.manual_seed fixes it)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _GcnLayerFn(torch.autograd.Function):
    """Graph_conv_layer (GCN/GCN.py:41-47) as one differentiable op, trained the way the
    reference's loop runs it (GCN/train_eval.py:43-48: forward, loss.backward()). Two forms:

    A (X W^T) + b (in_features > out_features: the narrower SpMM)
      forward   S = X W^T on the MFMA transform -- scattered into the column-degree order of
                A P^T when the graph takes that path (``column_order``), as at inference --
                then Y = A S + b (the forward SpMM path, bias in its epilogue);
      backward  dS = A^T dY (the same SpMM kernels; A itself when it is symmetric, as the GCN
                normalisation is: no transposed copy), dX = dS W on the MFMA transform,
                dW = dS^T X and db = the column sums of dY in one pass (gnn_gemm_tn_f32, a
                K = n_rows reduction: 1.81 ms on hipBLASLt at cfg2). S is not kept.
    (A X) W^T + b (in_features <= out_features, ``GCN_REASSOC``)
      forward   Z = A X (the SpMM over X), Y = Z W^T + b (the transform, bias in its store
                epilogue: gnn_gcn_transform_epi_f32); Z is kept for backward;
      backward  dW = dY^T Z and db = the column sums of dY in one gemm_tn pass that reads dY
                once (d = b), and only when X needs a gradient dZ = dY W (transform) and
                dX = A^T dZ (SpMM).
    The two forms agree to fp32 rounding (a sum of products regrouped).

    ``relu_dropout`` = (p, seed), reassociated form only (``fuses_relu_dropout``): the output
    is H = dropout_p(ReLU(Y)) -- GCN_Model's ReLU and Dropout after the layer (GCN/GCN.py:12-14)
    -- from the transform's epilogue (hashed dropout: element (i, c) kept iff the (seed, i, c)
    hash clears p); H is kept, and the backward's upstream gradient passes exactly where
    H > 0, scaled by 1 / (1 - p): folded into the dW / db pass (gemm_tn_masked), formed
    explicitly only when X needs a gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, g, relu_dropout=None):
        ctx.g = g
        ctx.has_bias = bias is not None
        ctx.reassoc = _reassociate(x, weight, g)
        ctx.relu_dropout = relu_dropout
        if relu_dropout is not None:
            if not fuses_relu_dropout(x, weight, g):
                raise ValueError("relu_dropout= needs the reassociated form on a transform shape")
            p, seed = relu_dropout
            z = spmm_forward(g, x)
            h = gcn_transform(z, weight, relu=True, bias=bias, dropout_p=p, seed=seed)
            ctx.save_for_backward(z, weight, h)
            return h
        if ctx.reassoc:
            z = spmm_forward(g, x)
            y = gcn_transform(z, weight, bias=bias)
            if y is None:
                y = torch.mm(z, weight.t()) if bias is None else torch.addmm(bias, z, weight.t())
            ctx.save_for_backward(z, weight)
            return y
        # an output width that is not a multiple of 4 (a classifier layer: 7 classes) is
        # zero-padded to one: the SpMMs then gather 16-B pieces of the support / dY rows in
        # packed row tasks (7 -> 8 at cfg2: 0.30 -> 0.27 ms per SpMM pass), the support and dX
        # products take the narrow kernels (linear_small)
        fout = weight.shape[0]
        ctx.pad = (-fout) % 4 if GCN_PAD_NARROW and fout < 64 else 0
        if ctx.pad:
            weight = torch.nn.functional.pad(weight, (0, 0, 0, ctx.pad))
            bias = torch.nn.functional.pad(bias, (0, ctx.pad)) if bias is not None else None
        order = column_order(g, weight.shape[0]) if x.shape[0] == g.n_cols else None
        s = None
        if order is not None:
            s = gcn_transform(x, weight, out_rows=order.inv, check_rows=False)
        if s is not None:
            y = spmm_forward(order.graph, s, bias)
        else:
            y = spmm_forward(g, _transform_or_mm(x, weight), bias)
        ctx.save_for_backward(x, weight)
        return y[:, :fout] if ctx.pad else y

    @staticmethod
    def backward(ctx, gy):
        gy = gy.contiguous()
        gx = gw = gb = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.relu_dropout is not None:
            z, weight, h = ctx.saved_tensors
            scale = 1.0 / (1.0 - ctx.relu_dropout[0])
            if ctx.needs_input_grad[1]:
                r = gemm_tn_masked(z, gy, h, scale, want_b, trans=True)
                if r is not None:
                    gw, gb = r
            dy = None
            if (ctx.needs_input_grad[1] and gw is None) or (want_b and gb is None) \
                    or ctx.needs_input_grad[0]:
                dy = torch.where(h > 0, gy * scale, torch.zeros((), dtype=gy.dtype,
                                                                device=gy.device))
            if ctx.needs_input_grad[1] and gw is None:
                gw = torch.mm(dy.t(), z)
            if want_b and gb is None:
                gb = dy.sum(0)
            if ctx.needs_input_grad[0]:
                gx = spmm_forward(ctx.g.transpose(), _transform_or_mm(dy, weight.t().contiguous()))
            return gx, gw, gb, None, None
        x, weight = ctx.saved_tensors  # Z = A X in the reassociated form
        if ctx.reassoc:
            main = side = None
            if GCN_OVERLAP_DW and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:
                main = torch.cuda.current_stream(gy.device)
                side = _side_stream(gy.device)
                side.wait_stream(main)
            if ctx.needs_input_grad[1]:
                with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                    # dW = dY^T Z as (Z^T dY)^T; db = the column sums of dY from the same loads
                    r = gemm_tn(x, gy, gy if want_b else None, trans=True)
                    if r is not None:
                        gw, gb = r
                    else:
                        gw = torch.mm(gy.t(), x)
                    if want_b and gb is None:
                        gb = gy.sum(0)
                if side is not None:  # read there: not recycled before the side work is done
                    x.record_stream(side)
                    gy.record_stream(side)
            if want_b and gb is None:
                gb = gy.sum(0)
            if ctx.needs_input_grad[0]:
                gx = spmm_forward(ctx.g.transpose(), _transform_or_mm(gy, weight.t().contiguous()))
            if side is not None:
                main.wait_stream(side)
                for t in (gw, gb):
                    if t is not None:
                        t.record_stream(main)
            return gx, gw, gb, None, None
        if ctx.pad:
            gy = torch.nn.functional.pad(gy, (0, ctx.pad))
        ds = spmm_forward(ctx.g.transpose(), gy)
        if ctx.needs_input_grad[0]:
            gx = _transform_or_mm(ds, weight.t().contiguous())
        if ctx.needs_input_grad[1]:
            # dW = dS^T X as (X^T dS)^T, with db = the column sums of dY read in the same pass
            r = gemm_tn(x, ds, gy if want_b else None, trans=True)
            if r is not None:
                gw, gb = r
            else:
                gw = torch.mm(ds.t(), x)
        if want_b and gb is None:
            gb = gy.sum(0)
        if ctx.pad:
            fout = weight.shape[0] - ctx.pad
            gw = gw[:fout] if gw is not None else None
            gb = gb[:fout] if gb is not None else None
        return gx, gw, gb, None, None


def gcn_layer(g: CsrGraph, x: torch.Tensor, weight: torch.Tensor,
              bias: torch.Tensor | None = None, relu_dropout=None) -> torch.Tensor:
    """A_hat (x W^T) + b, differentiable w.r.t. x, W and b (``_GcnLayerFn``); with
    ``relu_dropout`` = (p, seed): dropout_p(ReLU(A_hat x W^T + b)) as one op (see
    _GcnLayerFn; requires ``fuses_relu_dropout``)."""
    _require_device(g.rowptr, x, weight, bias)
    if x.dtype != torch.float32 or weight.dtype != torch.float32:
        raise TypeError("gcn_layer runs in float32")
    if x.dim() != 2 or weight.dim() != 2 or x.shape[1] != weight.shape[1] \
            or x.shape[0] != g.n_cols:
        raise ValueError("x must be [n_cols, F_in] and weight [F_out, F_in]")
    return _GcnLayerFn.apply(x, weight, bias, g, relu_dropout)


# ---------------------------------------------------------------------- GAT
GAT_DENSE = 0   # GraphAttentionLayer   (GAT/models/layers.py:22-37)
GAT_SPARSE = 1  # SpGraphAttentionLayer (GAT/models/layers.py:94-131)


def gat_logits(wh: torch.Tensor, heads: int, fh: int, a_src: torch.Tensor,
               a_dst: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """el[n,h] = a_src[h].Wh[n,h], er[n,h] = a_dst[h].Wh[n,h] (one HIP launch)."""
    _require_device(wh, a_src, a_dst)
    wh = _rows_f32(wh, "Wh")
    n = wh.shape[0]
    if wh.shape[1] != heads * fh or a_src.numel() != heads * fh or a_dst.numel() != heads * fh:
        raise ValueError("Wh / attention vectors do not match heads * fh")
    el = torch.empty((n, heads), dtype=torch.float32, device=wh.device)
    er = torch.empty((n, heads), dtype=torch.float32, device=wh.device)
    lib = _lib.load()
    _lib.check(lib.gnn_gat_logits_f32(wh.data_ptr(), wh.stride(0), n, heads, fh,
                                      a_src.contiguous().data_ptr(), a_dst.contiguous().data_ptr(),
                                      el.data_ptr(), er.data_ptr(), heads,
                                      _lib.stream_handle(wh.device)), "gnn_gat_logits_f32")
    return el, er


def gat_project(x: torch.Tensor, w: torch.Tensor, heads: int, fh: int, a_src: torch.Tensor,
                a_dst: torch.Tensor, packed: bool = False, col_rows: torch.Tensor | None = None):
    """(Wh = x @ w, el, er) in one MFMA pass (inference; no autograd), or None when the
    shape is not covered by gnn_gat_project_f32 (the caller then uses torch.mm +
    gat_logits). ``packed``: the three are views of ONE [n, H*Fh + 2H] buffer, rows
    [Wh | er | el], so the aggregation's er gather lands next to the Wh row it also
    gathers. Same output bits; measured neutral at cfg3 on a slow box (1.297 vs 1.298 ms,
    profiles/r01i_gat_pack_ab_slow.log), so it is not the default.

    ``col_rows`` (int64 [n], a permutation): Wh and er of node i go to row col_rows[i], el
    stays at row i (gnn_gat_project_rows_f32) -- the operands of the aggregation over a
    column-degree-ordered graph (``gat_column_order``; col_rows = its ``inv``)."""
    _require_device(x, w, a_src, a_dst)
    if (x.dtype != torch.float32 or w.dtype != torch.float32 or x.dim() != 2 or w.dim() != 2
            or x.shape[1] != w.shape[0] or w.shape[1] != heads * fh):
        return None
    lib = _lib.load()
    k, fout = w.shape
    if not lib.gnn_gat_project_supported(k, fout, fh):
        return None
    if x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
        x = x.contiguous()
    n = x.shape[0]
    if col_rows is not None:
        _require_device(col_rows)
        if packed:
            raise ValueError("col_rows= needs separate el / er buffers (packed=False)")
        if col_rows.dtype != torch.int64 or col_rows.shape != (n,):
            raise TypeError("col_rows must be int64 [rows of x]")
        col_rows = col_rows.contiguous()
    if packed:
        buf = torch.empty((n, fout + 2 * heads), dtype=torch.float32, device=x.device)
        wh, er, el = buf[:, :fout], buf[:, fout:fout + heads], buf[:, fout + heads:]
    else:
        wh = torch.empty((n, fout), dtype=torch.float32, device=x.device)
        el = torch.empty((n, heads), dtype=torch.float32, device=x.device)
        er = torch.empty((n, heads), dtype=torch.float32, device=x.device)
    if col_rows is not None:
        _lib.check(lib.gnn_gat_project_rows_f32(
            x.data_ptr(), x.stride(0), n, k, w.contiguous().data_ptr(), fout,
            a_src.contiguous().data_ptr(), a_dst.contiguous().data_ptr(), heads, fh,
            wh.data_ptr(), wh.stride(0), el.data_ptr(), er.data_ptr(), el.stride(0),
            col_rows.data_ptr(), None, _lib.stream_handle(x.device)),
            "gnn_gat_project_rows_f32")
        return wh, el, er
    _lib.check(lib.gnn_gat_project_f32(
        x.data_ptr(), x.stride(0), n, k, w.contiguous().data_ptr(), fout,
        a_src.contiguous().data_ptr(), a_dst.contiguous().data_ptr(), heads, fh, wh.data_ptr(),
        wh.stride(0), el.data_ptr(), er.data_ptr(), el.stride(0), None,
        _lib.stream_handle(x.device)), "gnn_gat_project_f32")
    return wh, el, er


# fout = 256 at k > 64 (cfg5's 256 -> 256 layer) runs as ONE 8-wave x 2-block launch, faster
# than hipBLASLt (10M x 256 -> 256: 9.63 vs 9.95 ms, profiles/r03o_transform_one256_ab.log; the
# round-3 two-launch form lost, 10.57 ms); False keeps those shapes on nn.Linear
TRANSFORM_WIDE_MFMA = True


TRANSFORM_PRECISIONS = ("split-bf16", "fp32-mfma")


def transform_precision() -> str:
    """The MFMA transforms' arithmetic at K >= 128 and of the GAT projection at K = 64 (see
    set_transform_precision), read back from the library (gnn_transform_get_precision), so a
    direct C call to gnn_transform_set_precision is seen too."""
    return TRANSFORM_PRECISIONS[0] if _lib.load().gnn_transform_get_precision() == 1 \
        else TRANSFORM_PRECISIONS[1]


def set_transform_precision(mode: str) -> str:
    """Arithmetic of the MFMA transforms at K >= 128 and of the GAT projection at K = 64
    (gnn_transform_set_precision, process-wide), returns the previous mode: 'split-bf16'
    (default: fp32 products from three-piece bf16 splits on v_mfma_f32_16x16x32_bf16, a few
    fp32 ulps per product) or 'fp32-mfma' (v_mfma_f32_16x16x4_f32, a k-ordered fp32 fmaf
    chain)."""
    if mode not in TRANSFORM_PRECISIONS:
        raise ValueError(f"transform precision must be one of {TRANSFORM_PRECISIONS}")
    prev = _lib.load().gnn_transform_set_precision(0 if mode == "fp32-mfma" else 1)
    return TRANSFORM_PRECISIONS[0] if prev == 1 else TRANSFORM_PRECISIONS[1]


def gcn_transform(x: torch.Tensor, weight: torch.Tensor, relu: bool = False,
                  out: torch.Tensor | None = None, out_rows: torch.Tensor | None = None,
                  check_rows: bool = True, live: torch.Tensor | None = None,
                  bias: torch.Tensor | None = None, dropout_p: float = 0.0,
                  seed: int = 0) -> torch.Tensor | None:
    """support = x @ weight^T on fp32 MFMA (gnn_gcn_transform_f32), the dense half of
    Graph_conv_layer.forward (GCN/GCN.py:42); ``relu=True``: max(x @ weight^T, 0)
    (gnn_linear_relu_f32, the SageLayer at GraphSAGE/GraphSAGE.py:18-20). Inference only
    (no autograd). None when the shape is not covered (the caller then uses nn.Linear /
    hipBLASLt).

    ``out_rows`` (int64 [rows of x]): x row i goes to support row out_rows[i]
    (gnn_gcn_transform_rows_f32), e.g. a degree order's ``inv`` so that the support is in the
    degree-ordered graph's column order; ``out`` (or a new [rows of x, fout] tensor) receives
    it; the ids must not repeat (two rows stored to one support row leave either).
    ``check_rows=False`` skips the host read of the range-check flag (trusted ids, e.g. a
    ``DegreeOrder``'s; the kernel still skips the store of a bad id).

    ``live`` (with ``relu=True``): a device int64 scalar; only rows [0, min(live, rows of x))
    are computed (gnn_linear_relu_live_f32) -- a sampled batch's frontier whose size the host
    never read; the other output rows are left as they were.

    ``bias`` (fp32 [fout]) and ``dropout_p`` / ``seed`` (without out_rows / live):
    dropout(act(x @ weight^T + bias)) in the store epilogue (gnn_gcn_transform_epi_f32; act =
    ReLU if ``relu``; element (i, c) kept iff the (seed, i, c) hash clears p, kept values scaled
    by 1 / (1 - p))."""
    _require_device(x, weight)
    if (x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() != 2
            or weight.dim() != 2 or x.shape[1] != weight.shape[1]):
        return None
    lib = _lib.load()
    fout, k = weight.shape
    if not lib.gnn_gcn_transform_supported(k, fout):
        return None
    if fout == 256 and k > 64 and not TRANSFORM_WIDE_MFMA:
        return None
    if out_rows is not None and relu:
        raise ValueError("out_rows= is supported without the ReLU epilogue only")
    epi = bias is not None or dropout_p > 0
    if epi and (out_rows is not None or live is not None):
        raise ValueError("bias= / dropout_p= are supported without out_rows / live only")
    if not 0.0 <= dropout_p < 1.0:
        raise ValueError("dropout_p must be in [0, 1)")
    if bias is not None:
        _require_device(bias)
        if bias.dtype != torch.float32 or bias.numel() != fout:
            raise ValueError("bias must be float32 [fout]")
        bias = bias.contiguous()
        if bias.data_ptr() % 16:
            bias = bias.clone()
    if live is not None:
        _require_device(live)
        if not relu or out_rows is not None:
            raise ValueError("live= is supported with the ReLU epilogue (the SageLayer) only")
        if live.dtype != torch.int64 or live.numel() != 1:
            raise TypeError("live must be a one-element int64 device tensor")
    if x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
        x = x.contiguous()
    w = weight.contiguous()
    m = x.shape[0]
    if out is None:
        out = torch.empty((m, fout), dtype=torch.float32, device=x.device)
    elif (out.dim() != 2 or out.shape[1] != fout or (out_rows is None and out.shape[0] != m)
          or out.dtype != torch.float32 or out.stride(1) != 1
          or out.stride(0) % 4 or out.data_ptr() % 16):
        raise ValueError("out must be float32 [rows, fout], 16-B aligned rows")
    if out_rows is not None:
        _require_device(out_rows)
        if out_rows.dtype != torch.int64 or out_rows.dim() != 1 or out_rows.numel() != m:
            raise TypeError("out_rows must be a 1-D int64 tensor with one id per row of x")
        out_rows = out_rows.contiguous()
        if m == 0:
            return out
        err = torch.zeros(1, dtype=torch.int32, device=x.device)
        _lib.check(lib.gnn_gcn_transform_rows_f32(
            x.data_ptr(), x.stride(0), m, k, w.data_ptr(), fout, out.data_ptr(), out.stride(0),
            out_rows.data_ptr(), out.shape[0], err.data_ptr(), _lib.stream_handle(x.device)),
            "gnn_gcn_transform_rows_f32")
        if check_rows and int(err.item()):
            raise IndexError("gcn_transform: an output row id is out of range")
        return out
    if live is not None:
        _lib.check(lib.gnn_linear_relu_live_f32(
            x.data_ptr(), x.stride(0), x.shape[0], live.data_ptr(), k, w.data_ptr(), fout,
            out.data_ptr(), out.stride(0), _lib.stream_handle(x.device)),
            "gnn_linear_relu_live_f32")
        return out
    if epi:
        _lib.check(lib.gnn_gcn_transform_epi_f32(
            x.data_ptr(), x.stride(0), x.shape[0], k, w.data_ptr(), fout, _lib.ptr(bias),
            1 if relu else 0, float(dropout_p), int(seed) & (2 ** 64 - 1), out.data_ptr(),
            out.stride(0), _lib.stream_handle(x.device)), "gnn_gcn_transform_epi_f32")
        return out
    fn, name = ((lib.gnn_linear_relu_f32, "gnn_linear_relu_f32") if relu else
                (lib.gnn_gcn_transform_f32, "gnn_gcn_transform_f32"))
    _lib.check(fn(x.data_ptr(), x.stride(0), x.shape[0], k, w.data_ptr(), fout, out.data_ptr(),
                  out.stride(0), _lib.stream_handle(x.device)), name)
    return out


def linear_relu_classify(x: torch.Tensor, weight: torch.Tensor, wd: torch.Tensor,
                         bd: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """(y, logits) = (relu(x @ weight^T), y @ wd^T + bd) in ONE launch
    (gnn_linear_relu_cls_f32): the last SageLayer (GraphSAGE/GraphSAGE.py:18-20) with the
    classifier ``self.dense`` (GraphSAGE.py:51-52) in its epilogue. Inference only; None when
    the shape is not covered (more than 4 classes, or a transform shape gcn_transform does not
    take), and the caller then runs the two layers separately."""
    _require_device(x, weight, wd)
    fout, k = weight.shape
    n_cls = wd.shape[0] if wd.dim() == 2 else 0
    if (x.dtype != torch.float32 or weight.dtype != torch.float32 or wd.dtype != torch.float32
            or x.dim() != 2 or x.shape[1] != k or wd.dim() != 2 or wd.shape[1] != fout
            or fout > 128
            or not 1 <= n_cls <= 4 or (bd is not None and (bd.dtype != torch.float32
                                                            or bd.numel() != n_cls))):
        return None
    lib = _lib.load()
    if not lib.gnn_gcn_transform_supported(k, fout) or (fout == 256 and k > 64
                                                         and not TRANSFORM_WIDE_MFMA):
        return None
    if bd is not None:
        _require_device(bd)
        bd = bd.contiguous()
    if x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
        x = x.contiguous()
    w, wdc = weight.contiguous(), wd.contiguous()
    m = x.shape[0]
    if out is None:
        out = torch.empty((m, fout), dtype=torch.float32, device=x.device)
    elif (out.shape != (m, fout) or out.dtype != torch.float32 or out.device != x.device
          or out.stride(1) != 1 or out.stride(0) % 4 or out.data_ptr() % 16):
        raise ValueError("out must be float32 [rows, fout] on x's device, 16-B aligned rows")
    logits = torch.empty((m, n_cls), dtype=torch.float32, device=x.device)
    _lib.check(lib.gnn_linear_relu_cls_f32(
        x.data_ptr(), x.stride(0), m, k, w.data_ptr(), fout, out.data_ptr(), out.stride(0),
        wdc.data_ptr(), _lib.ptr(bd), n_cls, logits.data_ptr(), logits.stride(0),
        _lib.stream_handle(x.device)), "gnn_linear_relu_cls_f32")
    return out, logits


def col_mean(x: torch.Tensor) -> torch.Tensor:
    """Mean over rows (double accumulation) -- the dense GAT layer's edgeless-row output."""
    _require_device(x)
    x = _rows_f32(x, "x")
    lib = _lib.load()
    scratch = torch.empty(max(8, int(lib.gnn_col_mean_scratch_bytes(x.shape[0], x.shape[1]))),
                          dtype=torch.uint8, device=x.device)
    out = torch.empty(x.shape[1], dtype=torch.float32, device=x.device)
    _lib.check(lib.gnn_col_mean_f32(x.data_ptr(), x.stride(0), x.shape[0], x.shape[1],
                                    out.data_ptr(), scratch.data_ptr(),
                                    _lib.stream_handle(x.device)), "gnn_col_mean_f32")
    return out


GAT_SHORT_MAX_DEG = 16  # rows with 2..16 edges take the short-row path (A/B at cfg3: 16 best)
# Packed row tasks for the rows of degree <= GAT_SHORT_MAX_DEG (gnn_gat_csr_tasks_f32,
# gat.hip gat_packed_rows): runs of consecutive low-degree rows, edgeless and one-edge rows
# included, cut at GAT_TASK_COST edges + rows, one wave per task -- in place of the packed
# small rows and gat_short_kernel's four rows per wave. Built, tested, and slower at cfg3:
# aggregation 0.943-0.976 ms (cost 64-256) against 0.779 ms for the row classes
# (tools/gat_tasks_ab.py, profiles/r05b_gat_tasks_ab.log): the small-row path packs the 435K
# edgeless / one-edge rows far more cheaply than a task's per-row flush and per-edge softmax
# update. Opt-in.
GAT_TASKS = False
# er_j recomputed from the gathered Wh_j rows when gat_aggregate is given a_dst, instead of an
# er load per (edge, head group): 1.2 of the 4.1 GB the aggregation fetched at cfg3
# (profiles/r05r_*). In gat_csr_kernel's layouts the recomputation cost what the loads saved
# (0.793 vs 0.783 ms, r05p_gat_ab.log); in the edge-head layout (gat_eh_kernel: each lane holds
# its head's slice of the row) it is a lane-local dot product: 0.631 vs 0.772 ms
# (r05t_gat_ab.log). The backward row pass takes er_j the same way.
GAT_ER_RECOMPUTE = True
GAT_TASK_COST = 128


def _gat_tasks_ok(heads, fh, *ts) -> bool:
    # the task kernel's geometry: one 16-B vector per lane, one chunk of <= 64 lanes per row of a
    # head group (<= 8 heads x fh <= 256 features), a lane's features inside one head
    if not GAT_TASKS or fh % 4 or min(heads, 8) * fh > 256:
        return False
    return all(t is None or (t.data_ptr() % 16 == 0 and (t.dim() == 1 or t.stride(0) % 4 == 0))
               for t in ts)
# XCD-sliced hub staging for GAT (``_gat_xcd``) is built and tested but not the default: at
# cfg3 it loses or ties at every setting (tools/xcd_ab.py --op gat, profiles/r02z_xcd_ab_gat_*:
# single pass 0.79 ms; rows of >= 128 edges 0.88, >= 256 0.86, >= 1024 0.79). The edge
# softmax (8 exps per edge, phase A/B through LDS) hides the gathers that the SpMM waits on.
GAT_XCD = False


def _gat_call(lib, g_rowptr, col, n, wh, el, er, lde, heads, fh, slope, mode, fill, out, ldo,
              seg_len, plan, mid, short, partial, stats, flags, stream, whh, erh, what):
    pa = plan.args()
    _lib.check(lib.gnn_gat_csr_hub_f32(
        g_rowptr.data_ptr(), col.data_ptr(), n, wh.data_ptr(), wh.stride(0), heads, fh,
        el.data_ptr(), er.data_ptr(), lde, float(slope), int(mode), _lib.ptr(fill), 0.0, 0,
        out.data_ptr(), ldo, seg_len, *pa[:6], pa[6], pa[7], pa[9],
        mid.data_ptr() if mid.numel() else pa[10], mid.numel(),
        short.data_ptr() if short is not None and short.numel() else None,
        short.numel() if short is not None else 0, _lib.ptr(partial), _lib.ptr(stats), flags,
        stream, whh.data_ptr(), whh.stride(0), erh.data_ptr(), erh.stride(0)), what)


def _gat_xcd(lib, g: CsrGraph, xp, wh, el, er, heads, fh, slope, mode, fill, out, seg, flags,
             stream):
    """GAT over the XCD-sliced hub plan (graph.XcdHubPlan), inference.

    Pass 1 runs each item (a row's hub edges in one XCD slice) as a row of its own, on XCD
    w % 8 like the SpMM, writing the item's softmax-weighted mean of Wh (no activation) and
    its per-head log-sum-exp L. Pass 2 runs every row's remaining edges plus one pseudo-edge
    per item whose Wh row is that mean and whose logit is L: an edge's logit is
    LeakyReLU(el_i + er_j) (dense; its negation for sparse), so the item's er entry is set
    to LeakyReLU^-1(+-L) - el_i. The online softmax then merges the items exactly as the
    fix-up merges segments (log-sum-exp rule). Both passes are gnn_gat_csr_hub_f32 over
    the staged buffers [hub rows | item rows]."""
    k, n_pos = xp.k, xp.n_pos
    feat = heads * fh
    dev = wh.device
    whb = torch.empty((k + n_pos, feat), dtype=torch.float32, device=dev)
    erb = torch.empty((k + n_pos, heads), dtype=torch.float32, device=dev)
    hp = xp.hub
    for src, dst, w in ((wh, whb, feat), (er, erb, heads)):
        _lib.check(lib.gnn_gather_rows_f32(src.data_ptr(), src.stride(0), src.shape[0],
                                           hp.hub_ids.data_ptr(), k, w, dst.data_ptr(), w,
                                           hp.err.data_ptr(), stream), "gnn_gather_rows_f32")
    el_items = el.index_select(0, xp.item_row)
    lse = torch.empty((n_pos, heads), dtype=torch.float32, device=dev)
    p1 = xp.items.plan(seg)
    if p1.n_seg or p1.n_small:
        raise RuntimeError("XCD hub plan: item rows outside the mid-row class")
    # er is never read in pass 1 (every column is staged): erb stands in with its stride
    _gat_call(lib, xp.items.rowptr, xp.items.col, n_pos, wh, el_items, erb, heads, heads, fh,
              slope, mode, None, whb[k:], feat, seg, p1, p1.mid_row, None, None, lse, 0, stream,
              whb, erb, "gnn_gat_csr_hub_f32 (xcd items)")
    y = lse if mode == GAT_DENSE else -lse
    torch.sub(torch.where(y >= 0, y, y / slope), el_items, out=erb[k:])
    p2 = xp.rest_plan(seg)
    mid, short = p2.gat_split(xp.rest.rowptr, GAT_SHORT_MAX_DEG)
    partial = None
    if p2.n_seg:
        partial = torch.empty((p2.n_seg, feat + 2 * heads), dtype=torch.float32, device=dev)
    _gat_call(lib, xp.rest.rowptr, xp.rest.col, g.n_rows, wh, el, er, el.stride(0), heads, fh,
              slope, mode, fill, out, out.stride(0), seg, p2, mid, short, partial, None, flags,
              stream, whb, erb, "gnn_gat_csr_hub_f32 (xcd rest)")


def gat_aggregate_staged(g: CsrGraph, wh: torch.Tensor, el: torch.Tensor, er: torch.Tensor,
                         whh: torch.Tensor, erh: torch.Tensor, heads: int, fh: int,
                         negative_slope: float, mode: int, activation: str | None = None,
                         out: torch.Tensor | None = None) -> torch.Tensor:
    """``gat_aggregate`` (inference: no dropout, no stats) over a graph whose column c >= 0
    reads Wh / er row c and c < 0 reads row -1-c of the staged tables ``whh`` / ``erh``
    (strided views allowed: e.g. the [Wh | er] rows an edge-cut rank received, used in
    place instead of concatenated). gnn_gat_csr_hub_f32; rows without edges are rejected
    (their dense-mode fill is a mean over every column, own and staged)."""
    _require_device(g.rowptr, wh, el, er, whh, erh, out)
    for t, name in ((wh, "Wh"), (el, "el"), (er, "er"), (whh, "whh"), (erh, "erh")):
        if t.dtype != torch.float32:
            raise TypeError(f"{name} must be float32 (got {t.dtype})")
    feat = heads * fh
    # column range, checked once per graph (one host sync, cached): -1-c must name a row of
    # the staged tables, c a row of Wh -- the hub kernel does not bound-check its reads
    rng_ = g._plans.get("_col_range")
    if rng_ is None and g.nnz:
        rng_ = g._plans["_col_range"] = tuple(int(v) for v in
                                              torch.stack([g.col.min(), g.col.max()]).tolist())
    if rng_ is not None and (rng_[0] < -whh.shape[0] or rng_[1] >= g.n_cols):
        raise IndexError(f"gat_aggregate_staged: column ids span [{rng_[0]}, {rng_[1]}], the "
                         f"tables hold {whh.shape[0]} staged rows and {g.n_cols} rows")
    if wh.shape != (g.n_cols, feat) or wh.stride(1) != 1:
        raise ValueError("Wh must be [n_cols, heads * fh] with unit column stride")
    if whh.shape[1] != feat or erh.shape != (whh.shape[0], heads) or whh.stride(1) != 1 \
            or erh.stride(1) != 1:
        raise ValueError("whh [K, heads * fh] and erh [K, heads] with unit column stride")
    if el.shape != (g.n_rows, heads) or er.shape != (g.n_cols, heads):
        raise ValueError("el must be [n_rows, heads] and er [n_cols, heads]")
    el, er = el.contiguous(), er.contiguous()
    if el.stride(0) != er.stride(0):
        raise ValueError("el / er must share a row stride")
    if g.has_empty_rows():
        raise ValueError("gat_aggregate_staged: the graph has rows without edges")
    if out is None:
        out = torch.empty((g.n_rows, feat), dtype=torch.float32, device=wh.device)
    if g.n_rows == 0:
        return out
    from .graph import staged_plan
    seg = seg_len_for(feat, GAT_SEG_BYTES)
    plan = g.__dict__.setdefault("_staged_plans", {}).get(seg)
    if plan is None:
        plan = g.__dict__["_staged_plans"][seg] = staged_plan(g, seg)
    mid, short = plan.gat_split(g.rowptr, GAT_SHORT_MAX_DEG)
    partial = None
    if plan.n_seg:
        partial = torch.empty((plan.n_seg, feat + 2 * heads), dtype=torch.float32,
                              device=wh.device)
    _gat_call(_lib.load(), g.rowptr, g.col, g.n_rows, wh, el, er, el.stride(0), heads, fh,
              negative_slope, mode, None, out, out.stride(0), seg, plan, mid, short, partial,
              None, _ACT_FLAGS[activation], _lib.stream_handle(wh.device), whh, erh,
              "gnn_gat_csr_hub_f32 (staged)")
    return out


def gat_aggregate(g: CsrGraph, wh: torch.Tensor, el: torch.Tensor, er: torch.Tensor, heads: int,
                  fh: int, negative_slope: float, mode: int, activation: str | None = None,
                  dropout_p: float = 0.0, seed: int = 0, seg_len: int | None = None,
                  out: torch.Tensor | None = None,
                  stats: torch.Tensor | None = None, hubs: int | None = None,
                  xcd: bool | None = None, a_dst: torch.Tensor | None = None) -> torch.Tensor:
    """Fused edge-softmax + neighbour aggregation for all heads (one HIP launch + fix-up).

    ``a_dst`` ([heads * fh], the vector er = Wh . a_dst came from): the kernels recompute er_j
    from the Wh rows they gather instead of loading it (gnn_gat_csr_ex_f32; GAT_ER_RECOMPUTE);
    the same values up to the rounding of er's dot products.

    ``hubs``: Wh / er rows of the highest-degree columns staged into compact tables first
    (gnn_gat_csr_hub_f32; 0 = none, default ``hub_rows_for``); same output bits.

    ``xcd``: XCD-sliced hub staging (``_gat_xcd``; default GAT_XCD and the same size rule
    as the SpMM, inference only: no dropout, no stats, a positive LeakyReLU slope)."""
    _require_device(g.rowptr, wh, el, er, out)
    wh = _rows_f32(wh, "Wh")
    n = g.n_rows
    if wh.shape[0] != g.n_cols or wh.shape[1] != heads * fh:
        raise ValueError("Wh must be [n_cols, heads * fh]")
    if el.shape != (n, heads) or er.shape != (g.n_cols, heads):
        raise ValueError("el must be [n_rows, heads] and er [n_cols, heads]")
    # el / er share one row stride in the C-ABI: strided views of one buffer (gat_project
    # packed=True) pass as they are, anything else is made contiguous
    if not (el.stride(1) == 1 and er.stride(1) == 1 and el.stride(0) == er.stride(0)
            and el.stride(0) >= heads):
        el = el.contiguous()
        er = er.contiguous()
    lde = el.stride(0)
    feat = heads * fh
    if out is None:
        out = torch.empty((n, feat), dtype=torch.float32, device=wh.device)
    if n == 0:
        return out
    fill = None
    if mode == GAT_DENSE and g.has_empty_rows():
        fill = col_mean(wh)
    seg = seg_len if seg_len is not None else seg_len_for(feat, GAT_SEG_BYTES)
    lib = _lib.load()
    if xcd is None:
        xcd = (GAT_XCD and hubs is None and g.nnz >= XCD_MIN_NNZ
               and xcd_hub_rows_for(g.n_cols, feat + heads) > 0)
    if (xcd and g.nnz and dropout_p == 0 and stats is None and negative_slope > 0
            and mode in (GAT_DENSE, GAT_SPARSE)):
        kx = (xcd_hub_rows_for(g.n_cols, feat + heads) if hubs is None
              else min(int(hubs), g.n_cols))
        chunk = min(XCD_CHUNK, seg)
        xp = g.xcd_hub_plan(kx, XCD_MIN_DEG, chunk) if kx >= 8 and chunk >= 4 else None
        if xp is not None:
            _gat_xcd(lib, g, xp, wh, el, er, heads, fh, negative_slope, mode, fill, out, seg,
                     _ACT_FLAGS[activation], _lib.stream_handle(wh.device))
            return out
    plan = g.plan(seg)
    partial = None
    if plan.n_seg:
        partial = torch.empty((plan.n_seg, feat + 2 * heads), dtype=torch.float32,
                              device=wh.device)
    pa = plan.args()  # (seg_row, seg_begin, n_seg, long_row, long_seg_ptr, n_long,
    #                    small_row, small_col, small_val, n_small, mid_row, n_mid)
    mid, short = plan.gat_split(g.rowptr, GAT_SHORT_MAX_DEG)
    stream = _lib.stream_handle(wh.device)
    args = (n, wh.data_ptr(), wh.stride(0), heads, fh,
            el.data_ptr(), er.data_ptr(), lde, float(negative_slope), int(mode), _lib.ptr(fill),
            float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF, out.data_ptr(), out.stride(0),
            plan.seg_len, *pa[:6], pa[6], pa[7], pa[9],
            mid.data_ptr() if mid.numel() else pa[10], mid.numel(),
            short.data_ptr() if short.numel() else None, short.numel(), _lib.ptr(partial),
            _lib.ptr(stats), _ACT_FLAGS[activation], stream)
    k = hub_rows_for(g.n_cols, feat + heads) if hubs is None else min(int(hubs), g.n_cols)
    hp = whh = erh = None
    ldwh = lderh = 0
    if k > 0 and g.nnz:
        hp = g.hub_plan(k)
        if XCD_DIRECT and hp.prefix:  # degree-ordered columns: hub rows read in place
            whh, ldwh, erh, lderh = wh, wh.stride(0), er, lde
        else:
            whh = torch.empty((hp.k, feat), dtype=torch.float32, device=wh.device)
            erh = torch.empty((hp.k, heads), dtype=torch.float32, device=wh.device)
            ldwh, lderh = feat, heads
            for src, dst, w in ((wh, whh, feat), (er, erh, heads)):
                _lib.check(lib.gnn_gather_rows_f32(src.data_ptr(), src.stride(0), src.shape[0],
                                                   hp.hub_ids.data_ptr(), hp.k, w,
                                                   dst.data_ptr(), w, hp.err.data_ptr(), stream),
                           "gnn_gather_rows_f32")
    col = hp.col_hub if hp is not None else g.col
    if _gat_tasks_ok(heads, fh, wh, out, fill, whh):
        tp = g.task_plan(plan.seg_len, GAT_SHORT_MAX_DEG, GAT_TASK_COST)
        b = tp.base
        if b.n_seg and partial is None:
            partial = torch.empty((b.n_seg, feat + 2 * heads), dtype=torch.float32,
                                  device=wh.device)
        rc = lib.gnn_gat_csr_tasks_f32(
            g.rowptr.data_ptr(), col.data_ptr(), n, wh.data_ptr(), wh.stride(0), heads, fh,
            el.data_ptr(), er.data_ptr(), lde, float(negative_slope), int(mode), _lib.ptr(fill),
            float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF, out.data_ptr(), out.stride(0),
            tp.seg_len, _lib.ptr(b.seg_row), _lib.ptr(b.seg_begin), b.n_seg, _lib.ptr(b.long_row),
            b.long_seg_ptr.data_ptr(), b.n_long,
            tp.mid_row.data_ptr() if tp.n_mid else b.long_seg_ptr.data_ptr(), tp.n_mid,
            tp.task_row.data_ptr() if tp.n_task else None, tp.n_task, _lib.ptr(partial),
            _lib.ptr(stats), _ACT_FLAGS[activation], stream, _lib.ptr(whh), ldwh, _lib.ptr(erh),
            lderh)
        if rc != _lib.E_UNSUPPORTED:  # e.g. a 4-float vector path the row pitches do not allow
            _lib.check(rc, "gnn_gat_csr_tasks_f32")
            return out
        # the row-class launch below (same plan, same partial buffer) covers the shape
    if a_dst is not None and GAT_ER_RECOMPUTE:
        a_dst = a_dst.detach().reshape(-1).contiguous().float()
        if a_dst.numel() != feat:
            raise ValueError("a_dst must hold heads * fh values")
        _require_device(a_dst)
        rc = lib.gnn_gat_csr_ex_f32(g.rowptr.data_ptr(), col.data_ptr(), *args, _lib.ptr(whh),
                                    ldwh, _lib.ptr(erh), lderh, a_dst.data_ptr())
        _lib.check(rc, "gnn_gat_csr_ex_f32")
        return out
    if hp is not None:
        rc = lib.gnn_gat_csr_hub_f32(g.rowptr.data_ptr(), hp.col_hub.data_ptr(), *args,
                                     whh.data_ptr(), ldwh, erh.data_ptr(), lderh)
        _lib.check(rc, "gnn_gat_csr_hub_f32")
        return out
    rc = lib.gnn_gat_csr_f32(g.rowptr.data_ptr(), g.col.data_ptr(), *args)
    _lib.check(rc, "gnn_gat_csr_f32")
    return out


# ---------------------------------------------------------------- GraphSAGE
SAGE_MODES = {"MEAN": 0, "MAX": 1}   # GraphSAGE/graph_utils.py Aggregator
# + NeighborAggregator 'sum' (GraphSAGE_Pytorch) and the value max-pool the north star names
# ("mean/max-pool"; torch.max(dim=1).values, GraphSAGE_Pytorch/models/Aggregator.py:23-24)
SAGE_KINDS = {"MEAN": 0, "MAX": 1, "SUM": 2, "MAXPOOL": 3}


_EMPTY_FILL = {0: float("nan"), 2: 0.0}  # k == 0: torch.mean -> NaN, torch.sum -> 0


def _empty_reduction(mode: int) -> None:
    if mode == 1:  # torch.argmax over an empty dim raises
        raise IndexError("argmax(): Expected reduction dim 1 to have non-zero size.")
    if mode == 3:  # so does torch.max(dim=1)
        raise IndexError("max(): Expected reduction dim 1 to have non-zero size.")


def _sage_out(M, F, mode, dev):
    dt = torch.int64 if mode == 1 else torch.float32
    return torch.empty((M, F), dtype=dt, device=dev)


def sage_aggregate(neigh: torch.Tensor, agg_func: str = "MEAN") -> torch.Tensor:
    """Aggregator over a pre-gathered [M, k, F] tensor (GraphSAGE/graph_utils.py:4-11);
    'SUM' is NeighborAggregator's sum (GraphSAGE_Pytorch/models/Aggregator.py:21-22)."""
    if agg_func not in SAGE_KINDS:
        raise RuntimeError(f"unknown agg_func {agg_func!r}")
    _require_device(neigh)
    if neigh.dtype != torch.float32 or neigh.dim() != 3:
        raise TypeError("neigh_feat must be float32 [M, k, F]")
    if neigh.stride(2) != 1:
        neigh = neigh.contiguous()
    M, k, F = neigh.shape
    mode = SAGE_KINDS[agg_func]
    if k == 0:
        _empty_reduction(mode)
        return torch.full((M, F), _EMPTY_FILL[mode], device=neigh.device)
    out = _sage_out(M, F, mode, neigh.device)
    lib = _lib.load()
    _lib.check(lib.gnn_sage_aggregate_f32(neigh.data_ptr(), neigh.stride(1), neigh.stride(0), M, k,
                                          F, mode, out.data_ptr(), F,
                                          _lib.stream_handle(neigh.device)),
               "gnn_sage_aggregate_f32")
    return out


_ERR_SINK: dict = {}


def _err_flag(dev, check: bool) -> torch.Tensor:
    """A zeroed device flag for a checked gather; unchecked (trusted-index) calls share a
    per-device sink that is never read, so they cost no memset and no host sync."""
    if check:
        return torch.zeros(1, dtype=torch.int32, device=dev)
    t = _ERR_SINK.get(dev)
    if t is None:
        t = _ERR_SINK[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return t


def _check_err(err: torch.Tensor, what: str) -> None:
    if int(err.item()) != 0:
        raise IndexError(f"{what}: index out of range in self")


def _sage_dst(out, M, F, mode, dev):
    """The caller's output view (any row stride, unit column stride) or a new tensor."""
    if out is None:
        return _sage_out(M, F, mode, dev)
    want = torch.int64 if mode == 1 else torch.float32
    if out.shape != (M, F) or out.dtype != want or out.stride(1) != 1 or not out.is_cuda:
        raise ValueError(f"out must be a {want} [{M}, {F}] device view with unit column stride")
    return out


def sage_gather_aggregate(table: torch.Tensor, idx: torch.Tensor, agg_func: str = "MEAN",
                          check: bool = True, out: torch.Tensor | None = None) -> torch.Tensor:
    """Aggregator(torch.embedding(table, idx)) fused: [M, k] int64 indices into table [n, F]."""
    if agg_func not in SAGE_KINDS:
        raise RuntimeError(f"unknown agg_func {agg_func!r}")
    _require_device(table, idx)
    table = _rows_f32(table, "table")
    if idx.dim() != 2:
        raise ValueError("idx must be [M, k]")
    idx = idx.to(torch.int64)
    if idx.stride(1) != 1:
        idx = idx.contiguous()
    M, k = idx.shape
    F = table.shape[1]
    mode = SAGE_KINDS[agg_func]
    out = _sage_dst(out, M, F, mode, table.device)
    if k == 0:  # torch.mean over an empty dim is NaN, sum is 0; the caller's view is filled
        _empty_reduction(mode)
        return out.fill_(_EMPTY_FILL[mode])
    err = _err_flag(table.device, check)
    lib = _lib.load()
    _lib.check(lib.gnn_sage_gather_aggregate_f32(
        table.data_ptr(), table.stride(0), table.shape[0], idx.data_ptr(), idx.stride(0), M, k, F,
        mode, out.data_ptr(), out.stride(0), err.data_ptr(), _lib.stream_handle(table.device)),
        "gnn_sage_gather_aggregate_f32")
    if check:
        _check_err(err, "sage_gather_aggregate")
    return out


def sage_gather_concat(table: torch.Tensor, self_idx: torch.Tensor, idx: torch.Tensor,
                       agg_func: str = "MEAN", check: bool = True,
                       out: torch.Tensor | None = None,
                       live: torch.Tensor | None = None) -> torch.Tensor:
    """[M, 2F] = cat[table[self_idx], Aggregator(table[idx])] in one launch
    (gnn_sage_gather_concat_f32): the SageLayer input of GraphSAGE/GraphSAGE.py:17 with the
    gathers of :47-49. ``out`` may be any [M, 2F] float32 view with unit column stride.
    ``live``: a device int64 scalar; rows [0, min(live, M)) only (gnn_sage_gather_concat_live_f32,
    M = the capacity of a sampled batch whose frontier size the host never read).
    'MAX' (torch.argmax over the neighbours, graph_utils.py:8): the index written as fp32, the
    value torch.cat([self, argmax]) promotes it to (GNN_SAGE_ARGMAX_F32)."""
    if agg_func not in ("MEAN", "SUM", "MAXPOOL", "MAX"):
        raise RuntimeError(f"agg_func {agg_func!r} has no concat form")
    mode = 4 if agg_func == "MAX" else SAGE_KINDS[agg_func]
    _require_device(table, self_idx, idx, out)
    table = _rows_f32(table, "table")
    if idx.dim() != 2:
        raise ValueError("idx must be [M, k]")
    idx = idx.to(torch.int64)
    if idx.stride(1) != 1:
        idx = idx.contiguous()
    self_idx = self_idx.to(torch.int64).contiguous().view(-1)
    M, k = idx.shape
    F = table.shape[1]
    if self_idx.numel() != M:
        raise ValueError("self_idx must hold one index per output row")
    if out is None:
        out = torch.empty((M, 2 * F), dtype=torch.float32, device=table.device)
    elif out.shape != (M, 2 * F) or out.dtype != torch.float32 or out.stride(1) != 1:
        raise ValueError(f"out must be a float32 [{M}, {2 * F}] view with unit column stride")
    if M == 0:
        return out
    if k == 0:
        _empty_reduction(SAGE_KINDS[agg_func])
        out[:, :F].copy_(gather_rows(table, self_idx, check=check))
        out[:, F:].fill_(_EMPTY_FILL[SAGE_KINDS[agg_func]])
        return out
    if live is not None:
        _require_device(live)
        if live.dtype != torch.int64 or live.numel() != 1:
            raise TypeError("live must be a one-element int64 device tensor")
    err = _err_flag(table.device, check)
    lib = _lib.load()
    _lib.check(lib.gnn_sage_gather_concat_live_f32(
        table.data_ptr(), table.stride(0), table.shape[0], self_idx.data_ptr(), idx.data_ptr(),
        idx.stride(0), M, _lib.ptr(live), k, F, mode, out.data_ptr(),
        out.stride(0), out[:, F:].data_ptr(), out.stride(0), err.data_ptr(),
        _lib.stream_handle(table.device)), "gnn_sage_gather_concat_live_f32")
    if check:
        _check_err(err, "sage_gather_concat")
    return out


# The fused layer is opt-in (set SAGE_FUSED_MIN_ROWS to the smallest frontier to fuse): at
# cfg4 it gains 2-3 % on layer 0 (62,479 rows: 110 vs 112 us) and loses on the 8,192-row
# layer 1 (33 vs 25 us) -- its gathers and MFMAs do not overlap, so it costs about their
# sum, while the unfused gather-mean and hipBLASLt GEMM each run near their own roofline.
# A producer/consumer form (8 gather + 8 MFMA waves, double-buffered LDS tiles) was slower
# still (129 us). tools/sage_layer_ab.py, profiles/r02z_sage_layer_ab*.log.
SAGE_FUSED_MIN_ROWS = None


def _rows16(t: torch.Tensor) -> bool:
    return (t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1
            and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0)


def sage_layer(table: torch.Tensor, nbr_idx: torch.Tensor, weight: torch.Tensor,
               self_src: torch.Tensor, self_idx: torch.Tensor | None = None,
               check: bool = True) -> torch.Tensor | None:
    """relu(W . cat[self, mean_j table[nbr_idx[:, j]]]) in ONE launch (gnn_sage_layer_f32):
    the inference SageLayer (GraphSAGE/GraphSAGE.py:15-20) fused with its MEAN Aggregator and
    input gathers (graph_utils.py:6, GraphSAGE.py:47-49). self = self_src[self_idx] or, with
    no index, self_src itself. None when the shape is not covered (the caller then runs the
    gather-mean + GEMM launches)."""
    _require_device(table, nbr_idx, weight, self_src, self_idx)
    if nbr_idx.dim() != 2 or weight.dim() != 2 or not (_rows16(table) and _rows16(self_src)):
        return None
    M, k = nbr_idx.shape
    feat = table.shape[1]
    H = weight.shape[0]
    if (SAGE_FUSED_MIN_ROWS is None or M < SAGE_FUSED_MIN_ROWS or k == 0
            or self_src.shape[1] != feat or weight.shape[1] != 2 * feat):
        return None
    if self_idx is None and self_src.shape[0] != M:
        return None
    lib = _lib.load()
    if not lib.gnn_sage_layer_supported(feat, H):
        return None
    w = weight.detach().to(torch.float32).contiguous()
    nbr_idx = nbr_idx.to(torch.int64)
    if nbr_idx.stride(1) != 1:
        nbr_idx = nbr_idx.contiguous()
    if self_idx is not None:
        self_idx = self_idx.to(torch.int64).contiguous().view(-1)
        if self_idx.numel() != M:
            raise ValueError("self_idx must hold one index per output row")
    out = torch.empty((M, H), dtype=torch.float32, device=table.device)
    err = _err_flag(table.device, check)
    _lib.check(lib.gnn_sage_layer_f32(
        table.data_ptr(), table.stride(0), table.shape[0], self_src.data_ptr(),
        self_src.stride(0), self_src.shape[0], _lib.ptr(self_idx), nbr_idx.data_ptr(),
        nbr_idx.stride(0), M, k, feat, w.data_ptr(), H, out.data_ptr(), H, err.data_ptr(),
        _lib.stream_handle(table.device)), "gnn_sage_layer_f32")
    if check:
        _check_err(err, "sage_layer")
    return out


def gather_rows(x: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None,
                check: bool = True) -> torch.Tensor:
    """out[i] = x[idx[i]] (torch.embedding semantics, one HIP launch)."""
    _require_device(x, idx, out)
    x = _rows_f32(x, "x")
    idx = idx.to(torch.int64).contiguous().view(-1)
    n, F = idx.numel(), x.shape[1]
    if out is None:
        out = torch.empty((n, F), dtype=torch.float32, device=x.device)
    err = _err_flag(x.device, check)
    lib = _lib.load()
    _lib.check(lib.gnn_gather_rows_f32(x.data_ptr(), x.stride(0), x.shape[0], idx.data_ptr(), n, F,
                                       out.data_ptr(), out.stride(0), err.data_ptr(),
                                       _lib.stream_handle(x.device)), "gnn_gather_rows_f32")
    if check:
        _check_err(err, "gather_rows")
    return out


# ---------------------------------------------------------------- GAT backward
# The GAT backward as two passes (gnn_gat_backward_rows_f32: prep + del, per-row statistics;
# gnn_gat_backward_nodes_recompute_f32: the transposed aggregation recomputing the edge
# weights) instead of three (prep, edge pass writing w / ds per (edge, head), node pass reading
# them back); the three-pass path serves the shapes the two-pass kernels refuse.
GAT_BWD_RECOMPUTE = True
GAT_BWD_SHORT_DEG = 8   # rows with <= 8 edges: several per wave in both passes


def _short_split(plan, rowptr, max_deg):
    """(rows of more than max_deg edges, rows of at most max_deg edges incl. the plan's
    small rows) of a plan's non-segmented rows, cached on the plan."""
    cache = plan.__dict__.setdefault("_bwd_short", {})
    if max_deg not in cache:
        mid, short = plan.gat_split(rowptr, max_deg)
        cache[max_deg] = (mid, torch.cat([short, plan.small_row]).contiguous())
    return cache[max_deg]


def _bwd_recompute_ok(heads: int, fh: int, ldw: int) -> bool:
    """The shapes gnn_gat_backward_rows_f32 / _nodes_recompute_f32 take (16-B aligned tensors):
    the row pass's LDS (2 feat + heads <= 1152 floats) and the node pass's lane layout (fh / VW
    lanes per head a power of two, feat <= 256 VW; VW = 4 when fh and the Wh pitch are
    multiples of 4)."""
    feat = heads * fh
    vw = 4 if fh % 4 == 0 and ldw % 4 == 0 else 1
    lanes = fh // vw
    nv = -(-feat // vw)
    lpr = 0 if nv > 256 else (64 if nv > 64 else 1 << max(0, (nv - 1).bit_length()))
    return (2 * feat + heads <= 1152 and fh % vw == 0 and lanes & (lanes - 1) == 0
            and 0 < lanes <= lpr)


def _gat_backward_recompute(g, wh, el, er, stats, y, dy, a_src, a_dst, heads, fh,
                            negative_slope, mode, elu, dropout_p, seed, seg_len, mark,
                            dy_dropout=None):
    """The two-pass backward; None when the kernels refuse the shape (GNN_E_UNSUPPORTED)."""
    n = g.n_rows
    feat = heads * fh
    if not _bwd_recompute_ok(heads, fh, wh.stride(0)):
        return None
    dev = wh.device
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    f32 = dict(dtype=torch.float32, device=dev)
    sl = seg_len if seg_len is not None else seg_len_for(feat, GAT_SEG_BYTES)
    plan = g.plan(sl)
    short_ok = 8 * (2 * feat + heads) <= 1152
    rows, short = (_short_split(plan, g.rowptr, GAT_BWD_SHORT_DEG) if short_ok
                   else (plan.row_list(), plan.small_row[:0]))
    a_src = a_src.detach().reshape(-1).contiguous().float()
    a_dst = a_dst.detach().reshape(-1).contiguous().float()
    dout = torch.empty((n, feat), **f32)
    nstat = torch.empty((n, heads, 4), **f32)  # {el, lse, D, 0} per (row, head)
    dl = torch.empty((n, heads), **f32)
    del_part = torch.empty((max(plan.n_seg, 1), heads), **f32)
    seed64 = int(seed) & 0xFFFFFFFFFFFFFFFF
    mark("rows")

    def rows_pass(dy, dp, ds):
        return lib.gnn_gat_backward_rows_ex_f32(
            g.rowptr.data_ptr(), g.col.data_ptr(), n, wh.data_ptr(), wh.stride(0), heads, fh,
            el.data_ptr(), er.data_ptr(), stats.data_ptr(), dy.data_ptr(), y.data_ptr(), feat,
            int(elu), float(negative_slope), int(mode), float(dropout_p), seed64,
            dout.data_ptr(), nstat.data_ptr(), dl.data_ptr(), plan.seg_len,
            _lib.ptr(plan.seg_row), _lib.ptr(plan.seg_begin), plan.n_seg,
            _lib.ptr(plan.long_row), plan.long_seg_ptr.data_ptr(), plan.n_long, _lib.ptr(rows),
            rows.numel(), _lib.ptr(short), short.numel(), del_part.data_ptr(),
            a_dst.data_ptr() if GAT_ER_RECOMPUTE else None, float(dp),
            int(ds) & 0xFFFFFFFFFFFFFFFF, stream)

    if dy_dropout is not None:  # the upstream mask inside the prep where it takes the shape
        rc = rows_pass(dy, dy_dropout[0], dy_dropout[1])
        if rc == _lib.E_UNSUPPORTED:
            rc = rows_pass(dropout_rows(dy, dy_dropout[0], dy_dropout[1]), 0.0, 0)
    else:
        rc = rows_pass(dy, 0.0, 0)
    if rc == _lib.E_UNSUPPORTED:  # (_bwd_recompute_ok passed: an unaligned view)
        mark(None)
        return None
    _lib.check(rc, "gnn_gat_backward_rows_ex_f32")
    if g.symmetric and dropout_p == 0.0:
        # A^T = A: node j's in-edges are row j's (ascending sources); no edge ids needed
        rowptr_t, src_t, eid_t, gt = g.rowptr, g.col, None, g
    else:
        rowptr_t, src_t, eid_t, gt = g.transpose_eid()
    pt = gt.plan(sl)
    rows_t, short_t = _short_split(pt, rowptr_t, GAT_BWD_SHORT_DEG)
    dwh = torch.empty((n, feat), **f32)
    der = torch.empty((n, heads), **f32)
    part = torch.empty((max(pt.n_seg, 1), feat + heads), **f32)
    mark("nodes")
    rc = lib.gnn_gat_backward_nodes_recompute_f32(
        rowptr_t.data_ptr(), src_t.data_ptr(), _lib.ptr(eid_t), n, heads, fh, dout.data_ptr(),
        nstat.data_ptr(), wh.data_ptr(), wh.stride(0), er.data_ptr(), dl.data_ptr(),
        a_src.data_ptr(), a_dst.data_ptr(), float(negative_slope), int(mode), float(dropout_p),
        seed64, dwh.data_ptr(), der.data_ptr(), pt.seg_len, _lib.ptr(pt.seg_row),
        _lib.ptr(pt.seg_begin), pt.n_seg, _lib.ptr(pt.long_row), pt.long_seg_ptr.data_ptr(),
        pt.n_long, _lib.ptr(rows_t), rows_t.numel(), _lib.ptr(short_t), short_t.numel(),
        part.data_ptr(), stream)
    if rc == _lib.E_UNSUPPORTED:
        # the row pass's outputs are the three-pass path's prep + edge outputs but for w / ds:
        # start over there (a shape both refuse is one the three-pass kernels also cover)
        mark(None)
        return None
    _lib.check(rc, "gnn_gat_backward_nodes_recompute_f32")
    mark(None)
    return dwh, dout, dl, der


def gat_backward(g: CsrGraph, wh: torch.Tensor, el: torch.Tensor, er: torch.Tensor,
                 stats: torch.Tensor, y: torch.Tensor, dy: torch.Tensor, a_src: torch.Tensor,
                 a_dst: torch.Tensor, heads: int, fh: int, negative_slope: float, mode: int,
                 elu: bool, dropout_p: float = 0.0, seed: int = 0,
                 seg_len: int | None = None, timings: list | None = None,
                 dy_dropout: tuple | None = None):
    """dWh (incl. the el/er terms), del, der for one GAT layer: two HIP passes (row pass,
    recomputing node pass; GAT_BWD_RECOMPUTE) or, for the shapes those refuse, three.

    Returns (dwh [N, H*fh], dout [N, H*fh], del [N, H], der [N, H]). ``timings`` (a list):
    (pass name, start event, end event) of each pass on the current stream is appended
    (bench.py's per-kernel backward times). ``dy_dropout`` = (p, seed): dy is the gradient of
    ``dropout_rows(y, p, seed)`` (the hidden dropout fused into the layer); its mask is applied
    to dy here -- inside the backward prep where the two-pass kernels take the shape."""
    _require_device(wh, dy)
    n = g.n_rows
    feat = heads * fh
    dev = wh.device
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    dy = dy.contiguous()
    y = y.contiguous()

    def mark(name):
        if timings is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream(dev))
            if timings and timings[-1][2] is None:
                timings[-1] = (timings[-1][0], timings[-1][1], ev)
            if name:
                timings.append((name, ev, None))

    if GAT_BWD_RECOMPUTE:
        r = _gat_backward_recompute(g, wh, el, er, stats, y, dy, a_src, a_dst, heads, fh,
                                    negative_slope, mode, elu, dropout_p, seed, seg_len, mark,
                                    dy_dropout)
        if r is not None:
            return r
    if dy_dropout is not None:
        dy = dropout_rows(dy, dy_dropout[0], dy_dropout[1])
    dout = torch.empty((n, feat), dtype=torch.float32, device=dev)
    D = torch.empty((n, heads), dtype=torch.float32, device=dev)
    mark("prep")
    _lib.check(lib.gnn_gat_backward_prep_f32(dy.data_ptr(), y.data_ptr(), feat, n, heads, fh,
                                             int(elu), dout.data_ptr(), D.data_ptr(), stream),
               "gnn_gat_backward_prep_f32")
    sl = seg_len if seg_len is not None else seg_len_for(feat, GAT_SEG_BYTES)
    plan = g.plan(sl)
    E = g.nnz
    w_edge = torch.empty((max(E, 1), heads), dtype=torch.float32, device=dev)
    ds_edge = torch.empty((max(E, 1), heads), dtype=torch.float32, device=dev)
    dl = torch.zeros((n, heads), dtype=torch.float32, device=dev)
    del_part = torch.empty((max(plan.n_seg, 1), heads), dtype=torch.float32, device=dev)
    rows = plan.row_list()
    mark("edges")
    _lib.check(lib.gnn_gat_backward_edges_f32(
        g.rowptr.data_ptr(), g.col.data_ptr(), n, wh.data_ptr(), wh.stride(0), heads, fh,
        el.data_ptr(), er.data_ptr(), stats.data_ptr(), dout.data_ptr(), D.data_ptr(),
        float(negative_slope), int(mode), float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF,
        w_edge.data_ptr(), ds_edge.data_ptr(), dl.data_ptr(), plan.seg_len,
        _lib.ptr(plan.seg_row), _lib.ptr(plan.seg_begin), plan.n_seg, _lib.ptr(plan.long_row),
        plan.long_seg_ptr.data_ptr(), plan.n_long, _lib.ptr(rows), rows.numel(),
        del_part.data_ptr(), stream), "gnn_gat_backward_edges_f32")
    rowptr_t, src_t, eid_t, gt = g.transpose_eid()
    pt = gt.plan(sl)
    rows_t = pt.row_list()
    dwh = torch.empty((n, feat), dtype=torch.float32, device=dev)
    der = torch.zeros((n, heads), dtype=torch.float32, device=dev)
    part = torch.empty((max(pt.n_seg, 1), feat + heads), dtype=torch.float32, device=dev)
    a_src = a_src.contiguous().float()
    a_dst = a_dst.contiguous().float()
    # one node pass for every head (the kernel sums der over groups of 8 heads itself)
    mark("nodes")
    _lib.check(lib.gnn_gat_backward_nodes_f32(
        rowptr_t.data_ptr(), src_t.data_ptr(), eid_t.data_ptr(), n, heads, fh,
        dout.data_ptr(), w_edge.data_ptr(), ds_edge.data_ptr(), dl.data_ptr(),
        a_src.data_ptr(), a_dst.data_ptr(), dwh.data_ptr(), der.data_ptr(), pt.seg_len,
        _lib.ptr(pt.seg_row), _lib.ptr(pt.seg_begin), pt.n_seg, _lib.ptr(pt.long_row),
        pt.long_seg_ptr.data_ptr(), pt.n_long, _lib.ptr(rows_t), rows_t.numel(),
        part.data_ptr(), stream), "gnn_gat_backward_nodes_f32")
    mark(None)
    return dwh, dout, dl, der
