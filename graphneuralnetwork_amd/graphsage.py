"""Drop-in GraphSAGE modules (reference: GraphSAGE/GraphSAGE.py, GraphSAGE/graph_utils.py).

Same names, constructor arguments, 9-argument ``forward`` and state_dict keys
(``sage_blocks.sage_layer{i}.weight.weight`` [H, 2F or F], ``dense.weight`` /
``dense.bias``) as the reference.

Hot path on gfx950:

* ``Aggregator`` (graph_utils.py:4-11) -> one HIP launch (mean, or torch.argmax's
  int64 first-max indices, bit-exact; plus 'MAXPOOL', the value max-pool of the north star);
* the re-gathers of GraphSAGE.py:47-49 (``torch.embedding(feats, map)`` followed
  by the next layer's ``Aggregator``) -> ONE fused gather-aggregate launch that
  never materialises the [M, k, H] neighbour tensor, plus one row-gather
  launch for the centre rows;
* ``SageLayer``'s ``Linear(cat[self, agg])`` -> two accumulating MFMA GEMMs on
  the two halves of W (no concatenated copy).
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn.functional as F
from torch import nn

from .graph import from_coo
from .ops import (gather_rows, gcn_transform, linear_relu_classify, sage_aggregate,
                  sage_gather_aggregate, sage_gather_concat, sage_layer, spmm_forward)

# the inference SageLayer GEMM relu([self | agg] @ W^T) runs on the hand-written MFMA kernel
# (gnn_linear_relu_f32). With the split-bf16 arithmetic (the default, ops.set_transform_precision)
# it beats hipBLASLt at every size (K=256, N=128, tools/transform_prec_ab.py,
# profiles/r03w_transform_prec_ab.log: 8192 rows 11.0 vs 19.9 us, 61771 rows 32.6 vs 40.1,
# 200000 rows 90.2 vs 136.5); on the fp32-MFMA arithmetic it ran up to SAGE_MFMA_MAX_SMALL rows and
# from SAGE_MFMA_MIN_LARGE rows up, hipBLASLt in between (62479 rows 46.8 vs 41.0 us,
# profiles/r03f_gemm_ab.log).
SAGE_MFMA_MAX_SMALL = 16384
SAGE_MFMA_MIN_LARGE = 131072


def _sage_gemm_on_mfma(rows: int) -> bool:
    from .ops import transform_precision
    if transform_precision() == "split-bf16":
        return True
    return rows <= SAGE_MFMA_MAX_SMALL or rows >= SAGE_MFMA_MIN_LARGE


class Gathered(NamedTuple):
    """A feature tensor given as (table, index): ``table[index]`` without materialising it.

    Accepted by ``GraphSAGE.forward`` in place of the pre-gathered
    ``center_feats_data`` ([M] index) / ``center_neigh_feats_data`` ([M, k] index)
    the reference's collate_fn builds with torch.embedding
    (GraphSAGE/data_utils.py:161-162); see ``sampler.sample_batch``.
    ``trusted``: the indices are known to be in range (built by the device
    sampler), so the gather skips its index check and the host sync it costs.
    ``live``: a device int64 scalar -- only ``index[:live]`` is real (a batch from
    ``sample_batch(..., sync=False)``, whose sizes the host never read; ``index`` is then
    the buffer at its capacity). The fused inference layer runs on it as it is; any other
    path reads the count back and slices.
    """
    table: torch.Tensor
    index: torch.Tensor
    trusted: bool = False
    live: torch.Tensor | None = None


def _trim(g):
    """A Gathered with a device row count as an ordinary one (one host read)."""
    if not isinstance(g, Gathered) or g.live is None:
        return g
    return Gathered(g.table, g.index[:int(g.live.item())], g.trusted)


def trust_map(t: torch.Tensor) -> torch.Tensor:
    """Mark an index map as -1-free and in range (the device sampler's maps): the
    forward then skips the reference's ``map != -1`` filtering and the index check,
    i.e. every host synchronisation."""
    t._gnn_trusted = True
    return t


def _trusted(t) -> bool:
    return bool(getattr(t, "_gnn_trusted", False))


def _scatter_rows(g: torch.Tensor, idx: torch.Tensor, n: int, scale: float) -> torch.Tensor:
    """out[t] = scale * sum of g[m] over the (m, j) with idx[m, j] == t  (the adjoint of a
    row gather), as the HIP SpMM over the transposed index map: deterministic, no atomics.
    ``idx`` was bounds-checked by the forward gather."""
    M = idx.shape[0]
    k = idx.numel() // max(M, 1)
    rows = idx.reshape(-1)
    cols = torch.arange(M, device=idx.device, dtype=torch.int64).repeat_interleave(k)
    at = from_coo(rows, cols, torch.full((rows.numel(),), scale, dtype=torch.float32,
                                         device=idx.device), n, M, check=False)
    return spmm_forward(at, g.contiguous())


class _MeanAgg(torch.autograd.Function):
    """Pre-gathered MEAN / SUM with autograd (d neigh = d out (/ k) broadcast over k)."""

    @staticmethod
    def forward(ctx, neigh, kind="MEAN"):
        ctx.k = neigh.shape[1]
        ctx.kind = kind
        return sage_aggregate(neigh, kind)

    @staticmethod
    def backward(ctx, g):
        g = g / ctx.k if ctx.kind == "MEAN" else g
        return g.unsqueeze(1).expand(-1, ctx.k, -1), None


class _GatherMeanAgg(torch.autograd.Function):
    """Fused gather + MEAN / SUM with autograd w.r.t. the table (scatter of d out (/ k))."""

    @staticmethod
    def forward(ctx, table, idx, kind="MEAN", check=True):
        ctx.save_for_backward(idx)
        ctx.n = table.shape[0]
        ctx.kind = kind
        return sage_gather_aggregate(table, idx, kind, check=check)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        scale = 1.0 / idx.shape[1] if ctx.kind == "MEAN" else 1.0
        return _scatter_rows(g, idx, ctx.n, scale), None, None, None


class _MaxPoolAgg(torch.autograd.Function):
    """Value max-pool over a pre-gathered [M, k, F] tensor with autograd: the gradient goes
    to the first maximal neighbour of every (row, feature) -- the argmax kernel's index."""

    @staticmethod
    def forward(ctx, neigh):
        arg = sage_aggregate(neigh, "MAX")
        ctx.save_for_backward(arg)
        ctx.k = neigh.shape[1]
        return sage_aggregate(neigh, "MAXPOOL")

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        M, F = g.shape
        out = torch.zeros((M, ctx.k, F), dtype=g.dtype, device=g.device)
        return out.scatter_(1, arg.unsqueeze(1), g.unsqueeze(1))


class _GatherMaxPoolAgg(torch.autograd.Function):
    """Fused gather + value max-pool with autograd w.r.t. the table (the gradient of each
    (row, feature) lands on the table row of its first maximal neighbour)."""

    @staticmethod
    def forward(ctx, table, idx, check=True):
        arg = sage_gather_aggregate(table, idx, "MAX", check=check)
        ctx.save_for_backward(idx, arg)
        ctx.n = table.shape[0]
        return sage_gather_aggregate(table, idx, "MAXPOOL", check=False)

    @staticmethod
    def backward(ctx, g):
        idx, arg = ctx.saved_tensors
        rows = idx.to(torch.int64).gather(1, arg)                     # [M, F] table rows
        cols = torch.arange(g.shape[1], device=g.device).expand_as(rows)
        out = torch.zeros((ctx.n, g.shape[1]), dtype=g.dtype, device=g.device)
        return out.index_put_((rows, cols), g, accumulate=True), None, None


class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx, check=True):
        ctx.save_for_backward(idx)
        ctx.n = x.shape[0]
        return gather_rows(x, idx, check=check)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return _scatter_rows(g, idx.reshape(-1, 1), ctx.n, 1.0), None, None


def Aggregator(neigh_feat, agg_func='MEAN'):
    """GraphSAGE/graph_utils.py:4-11 on the device ('MEAN' -> fp32, 'MAX' -> int64 argmax).

    Extension beyond the reference: 'MAXPOOL' -> the fp32 value max-pool the north star
    names (torch.max(neigh_feat, dim=1).values); the reference's own names keep their
    meaning, and any other name prints and raises as the reference does."""
    if agg_func not in ('MEAN', 'MAX', 'MAXPOOL'):
        print('请选择合适的聚合函数')  # the reference prints this, then a bare raise
        raise RuntimeError("No active exception to reraise")
    return reduce_neighbors(neigh_feat, agg_func)


def _gather_aggregate(table, idx, agg_func, trusted=False):
    if agg_func in ('MEAN', 'SUM') and torch.is_grad_enabled() and table.requires_grad:
        return _GatherMeanAgg.apply(table, idx, agg_func, not trusted)
    if agg_func == 'MAXPOOL' and torch.is_grad_enabled() and table.requires_grad:
        return _GatherMaxPoolAgg.apply(table, idx, not trusted)
    return sage_gather_aggregate(table, idx, agg_func, check=not trusted)


def reduce_neighbors(neigh_feat, kind='MEAN'):
    """MEAN / SUM / MAX(argmax) / MAXPOOL over dim 1 of a pre-gathered [M, k, F] tensor or a
    ``Gathered`` (table, [M, k] index), with autograd for MEAN / SUM / MAXPOOL."""
    if isinstance(neigh_feat, Gathered):
        return _gather_aggregate(neigh_feat.table, neigh_feat.index, kind, neigh_feat.trusted)
    if kind in ('MEAN', 'SUM') and torch.is_grad_enabled() and neigh_feat.requires_grad:
        return _MeanAgg.apply(neigh_feat, kind)
    if kind == 'MAXPOOL' and torch.is_grad_enabled() and neigh_feat.requires_grad:
        return _MaxPoolAgg.apply(neigh_feat)
    return sage_aggregate(neigh_feat, kind)


def _gather(x, idx, trusted=False):
    if torch.is_grad_enabled() and x.requires_grad:
        return _GatherRows.apply(x, idx, not trusted)
    return gather_rows(x, idx, check=not trusted)


class SageLayer(nn.Module):
    """GraphSAGE/GraphSAGE.py:7-20: relu(W . cat[self, agg]) (or relu(W . agg) in gcn mode)."""

    def __init__(self, input_size, output_size, gcn=False, **kwargs):
        super().__init__(**kwargs)
        self.input_size = input_size
        self.output_size = output_size
        self.gcn = gcn
        self.weight = nn.Linear(self.input_size if self.gcn else 2 * self.input_size, self.output_size, bias=False)

    def forward(self, self_feats, aggregate_feats):
        W = self.weight.weight
        if self.gcn:  # the reference feeds the aggregate straight into Linear (int64 argmax fails there too)
            return F.relu(self.weight(aggregate_feats))
        if aggregate_feats.dtype != torch.float32:  # MAX mode: argmax indices promote like torch.cat
            aggregate_feats = aggregate_feats.to(torch.float32)
        if self_feats.dtype != torch.float32:
            self_feats = self_feats.to(torch.float32)
        n = self.input_size
        # cat([self, agg]) @ W^T == self @ W[:, :n]^T + agg @ W[:, n:]^T (no concat copy)
        part = F.linear(self_feats, W[:, :n])
        if torch.is_grad_enabled() and (W.requires_grad or self_feats.requires_grad
                                        or aggregate_feats.requires_grad):
            return F.relu(torch.addmm(part, aggregate_feats, W[:, n:].t()))
        # inference: ReLU in the GEMM epilogue (hipBLASLt), one kernel fewer
        return torch._addmm_activation(part, aggregate_feats, W[:, n:].t())


def _fused_sage_layer(block, center, neigh: Gathered, dense: nn.Linear | None = None,
                      agg: str = 'MEAN'):
    """Inference SageLayer on a (table, index map) aggregate.

    ``agg`` 'MAX' / 'MAXPOOL' (centre and neighbours Gathered from one table): the concat
    launch writes the argmax index as fp32 (the value torch.cat([self, argmax]) promotes it
    to) / the value max-pool into the [self | agg] buffer, then the same GEMM.

    Covered shapes (``ops.sage_layer``): ONE launch gathers the centre rows and the
    neighbour mean into an LDS tile and multiplies it by W on the matrix cores, ReLU fused.
    Otherwise the centre rows and the fused gather-mean write the two halves of ONE
    [M, 2F] buffer (the reference's torch.cat, never copied), then a single K=2F GEMM with
    the ReLU in the hipBLASLt epilogue: GraphSAGE.py:18-20 + the gathers of :47-49 as 3
    launches instead of 7; with the centre rows and the neighbours drawn from the same table
    (the sampler's Gathered maps) the two halves come from ONE launch
    (``ops.sage_gather_concat``), then the GEMM: 2 launches.

    ``dense`` (the last layer of a supervised net): the classifier of GraphSAGE.py:51-52 runs in
    the GEMM's epilogue when the MFMA kernel takes the shape (``ops.linear_relu_classify``);
    the return value is then ``(y, logits)``, else ``y`` alone."""
    live = neigh.live
    if live is not None:
        # a device row count: the concat gather + MFMA GEMM run on the buffers' capacity and
        # read the count themselves (no host round trip); other shapes / the classifier
        # epilogue read it back and slice
        W = block.weight.weight
        if (dense is not None or not isinstance(center, Gathered) or center.table is not neigh.table
                or center.live is None or not _sage_gemm_on_mfma(neigh.index.shape[0])
                or W.dtype != torch.float32):
            center, neigh, live = _trim(center), _trim(neigh), None
    if isinstance(center, Gathered):
        self_src, self_idx, trusted = center.table, center.index, center.trusted
    else:
        self_src, self_idx, trusted = center, None, True
    y = None
    if live is None and agg == 'MEAN':
        y = sage_layer(neigh.table, neigh.index, block.weight.weight, self_src, self_idx,
                       check=not (trusted and neigh.trusted))
    if y is not None:
        return y
    M, n = neigh.index.shape[0], block.input_size
    dev = neigh.table.device
    buf = torch.empty((M, 2 * n), dtype=torch.float32, device=dev)
    if live is not None:
        sage_gather_concat(neigh.table, center.index, neigh.index, agg,
                           check=not (center.trusted and neigh.trusted), out=buf, live=live)
        y = gcn_transform(buf, block.weight.weight, relu=True, live=live)
        if y is not None:
            return y
        # the transform does not take the shape: the rows past the count are never read
        buf = buf[:int(live.item())]
        M = buf.shape[0]
    elif isinstance(center, Gathered) and center.table is neigh.table:
        # both halves of cat[self, agg] in one launch (gnn_sage_gather_concat_f32)
        sage_gather_concat(neigh.table, center.index, neigh.index, agg,
                           check=not (center.trusted and neigh.trusted), out=buf)
    else:
        if isinstance(center, Gathered):
            gather_rows(center.table, center.index, out=buf[:, :n], check=not center.trusted)
        else:
            buf[:, :n].copy_(center)
        sage_gather_aggregate(neigh.table, neigh.index, "MEAN", check=not neigh.trusted,
                              out=buf[:, n:])
    W = block.weight.weight
    if dense is not None and _sage_gemm_on_mfma(M):
        yl = linear_relu_classify(buf, W, dense.weight, dense.bias)
        if yl is not None:
            return yl
    if _sage_gemm_on_mfma(M):  # relu(buf @ W^T) on the hand-written fp32-MFMA kernel
        y = gcn_transform(buf, W, relu=True)
        if y is not None:
            return y
    # the addmm's bias operand: a zero vector cached on the block (not a registered buffer,
    # so state_dict keys stay the reference's); a fresh torch.zeros cost a 5 us fill launch
    # per call (profiles/r03k_sage_trace_summary.txt)
    zero = block.__dict__.get("_zero_bias")
    if zero is None or zero.device != W.device or zero.dtype != W.dtype or \
            zero.numel() != W.shape[0]:
        zero = torch.zeros(W.shape[0], dtype=W.dtype, device=W.device)
        block.__dict__["_zero_bias"] = zero
    return torch._addmm_activation(zero, buf, W.t())


class GraphSAGE(nn.Module):
    """GraphSAGE/GraphSAGE.py:23-61 with the same 9-argument forward."""

    def __init__(self, num_layers, input_size, out_size, gcn=False, agg_func='MEAN', Unsupervised=True, class_size=None,
                 **kwargs):
        super().__init__(**kwargs)
        self.num_layers = num_layers
        self.gcn = gcn
        self.agg_func = agg_func
        self.sage_blocks = nn.Sequential()
        for index in range(0, num_layers):
            layer_size = out_size if index != 0 else input_size
            self.sage_blocks.add_module('sage_layer' + str(index), SageLayer(layer_size, out_size, gcn=self.gcn))
        self.Unsupervised = Unsupervised
        if not Unsupervised:
            self.dense = nn.Linear(out_size, class_size)

    def _fused_ok(self, block, center, neigh) -> bool:
        if torch.is_grad_enabled() or block.gcn or not isinstance(neigh, Gathered):
            return False
        if self.agg_func == 'MEAN':
            return True
        # MAX / MAXPOOL: the one-launch concat form (centre and neighbours from one table)
        return (self.agg_func in ('MAX', 'MAXPOOL') and isinstance(center, Gathered)
                and center.table is neigh.table and neigh.table.dtype == torch.float32)

    def forward(self, center_feats_data, center_nodes_map, center_neigh_feats_data, center_neigh_nodes_map,
                contexts_negatives_feats_data, contexts_negatives_nodes_map, contexts_negatives_neigh_feats_data,
                contexts_negatives_neigh_nodes_map, contexts_negatives_shape):
        if contexts_negatives_feats_data is None:
            center = center_feats_data         # tensor, or Gathered (table, [M] index)
            neigh = center_neigh_feats_data    # [M, k, F] tensor, or Gathered (table, [M, k] index)
            feats_data = classes = None
            for i, block in enumerate(self.sage_blocks):
                if self._fused_ok(block, center, neigh):
                    last = i == self.num_layers - 1 and not self.Unsupervised
                    feats_data = _fused_sage_layer(block, center, neigh,
                                                   self.dense if last else None, self.agg_func)
                    if isinstance(feats_data, tuple):  # the classifier ran in the epilogue
                        feats_data, classes = feats_data
                else:
                    center, neigh = _trim(center), _trim(neigh)
                    if isinstance(center, Gathered):
                        center = _gather(center.table, center.index, center.trusted)
                    feats_data = block(center, Aggregator(neigh, self.agg_func))
                if i != self.num_layers - 1:
                    cm = center_nodes_map[i]
                    nm = center_neigh_nodes_map[i]
                    if _trusted(cm) and _trusted(nm):  # device-sampler maps: no -1, in range
                        lv = getattr(cm, "_gnn_live", None)  # sync=False batch: device size
                        center = Gathered(feats_data, cm, True, lv)
                        neigh = Gathered(feats_data, nm, True, lv)
                    else:                              # GraphSAGE.py:56-57 (-1 padding dropped)
                        center = Gathered(feats_data, cm[cm != -1], False)
                        neigh = Gathered(feats_data, nm[nm[:, 0] != -1, :], False)
            if not self.Unsupervised and classes is None:
                classes = self.dense(feats_data)
            return feats_data, classes
        center_feats_data, _ = self(center_feats_data, center_nodes_map, center_neigh_feats_data,
                                    center_neigh_nodes_map, None, None, None, None, None)
        contexts_negatives_feats_data, _ = self(contexts_negatives_feats_data, contexts_negatives_nodes_map,
                                                contexts_negatives_neigh_feats_data,
                                                contexts_negatives_neigh_nodes_map, None, None, None, None, None)
        contexts_negatives_feats_data = contexts_negatives_feats_data.reshape(*contexts_negatives_shape, -1)
        return center_feats_data, torch.bmm(center_feats_data.unsqueeze(1), contexts_negatives_feats_data.permute(0, 2, 1))
