"""Drop-in GAT modules (reference: GAT/models/layers.py, GAT/models/GAT.py).

Same class names, constructor arguments, parameter shapes/initialisation and
``forward(h, adj)`` signatures as the reference:

* ``GraphAttentionLayer``   -- W [in, out] xavier_uniform(gain 1.414), a [2*out, 1]
  (layers.py:6-40); edges are ``adj > 0``; softmax attention.
* ``SpGraphAttentionLayer`` -- W [in, out] xavier_normal(gain 1.414), a [1, 2*out]
  (layers.py:72-134); edges are ``adj.nonzero()``; exp(-LeakyReLU) weights
  with no max subtraction, exactly the reference arithmetic (incl. its NaN
  assert for edgeless rows).
* ``GAT`` / ``SpGAT`` (GAT.py:7-38) -- ``attentions.AttentionHead{i}`` + ``out_att``
  state_dict keys.  The reference module cannot even be imported (GAT.py:4
  imports the missing ``models.HAN``); these are usable.

Where the reference materialises an N x N x 2F tensor per head (dense) or
E x 2F per head (sparse) and loops over heads in Python, here every
attention layer is: one pass for the feature transform of all heads
(X @ [W_1 | ... | W_H]) with the attention logits fused into its epilogue
(gnn_gat_project_f32, fp32 MFMA; torch.mm + gnn_gat_logits_f32 for shapes it
does not cover or when autograd needs the GEMM), and one HIP launch for the
fused edge-softmax + aggregation (+ ELU) over the CSR adjacency.  ``adj`` may be the
reference's dense tensor, a torch sparse tensor or a ``CsrGraph``.

At inference on graphs whose Wh is hub-staged, the layer runs over the column-degree-ordered
graph A P^T (``_AttentionBase._ordered``): the projection writes Wh / er in that column order
and the aggregation reads their hub rows in place (no per-call staging copies).

Training: the aggregation is an autograd Function whose backward is two more
HIP passes (gat_bwd.hip: a row pass -- ELU / softmax backward and the SDDMM
edge gradients summed per row -- and a node pass that recomputes the edge
weights over A^T), with the forward's per-row log-sum-exp and dropout seed
saved instead of the attention matrix; dropout masks are recomputed. On large
symmetric graphs the model trains over the degree-ordered graph P A P^T
(``GATBase.forward``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import ops as _ops
from .graph import as_csr
from .ops import (GAT_DENSE, GAT_SPARSE, PermuteRows, _bwd_recompute_ok, _transform_or_mm,
                  gat_aggregate, gat_backward, gat_column_order, gat_logits, gat_project,
                  gat_train_order, gemm_tn, model_dropout, dropout_rows,
                  hashed_dropout_ok as HASHED_DROPOUT_OK)

# The reference asserts ``not torch.isnan(...).any()`` in the sparse layer
# (layers.py:102,109,119,124).  Kept on by default for identical error
# behaviour; each check is one device reduction + host sync.
SPARSE_NAN_CHECK = True
# the GAT model's hidden dropout (GAT.py:17) inside the heads' autograd op: the forward applies
# the hashed mask to the layer's output, the backward prep applies it to the upstream gradient
# (no separate dropout backward pass)
GAT_FUSE_OUT_DROPOUT = True


class _GatLayerFn(torch.autograd.Function):
    """Fused attention layer: Wh, a_src, a_dst -> act(edge-softmax aggregation)."""

    @staticmethod
    def forward(ctx, Wh, a_src, a_dst, g, heads, fh, slope, mode, activation, drop_p, seed,
                out_drop=None):
        el, er = gat_logits(Wh, heads, fh, a_src, a_dst)
        stats = torch.empty((g.n_rows, heads), dtype=torch.float32, device=Wh.device)
        out = gat_aggregate(g, Wh, el, er, heads, fh, slope, mode, activation,
                            dropout_p=drop_p, seed=seed, stats=stats, a_dst=a_dst)
        ctx.save_for_backward(Wh, a_src, a_dst, el, er, stats, out)
        ctx.cfg = (g, heads, fh, slope, mode, activation, drop_p, seed, out_drop)
        if out_drop is not None:
            # the model's hidden F.dropout (GAT.py:17) on the layer's output; its backward runs
            # inside this layer's backward prep (gat_backward dy_dropout)
            return dropout_rows(out, out_drop[0], out_drop[1])
        return out

    @staticmethod
    def backward(ctx, dy):
        Wh, a_src, a_dst, el, er, stats, out = ctx.saved_tensors
        g, heads, fh, slope, mode, activation, drop_p, seed, out_drop = ctx.cfg
        dwh, dout, dl, der = gat_backward(g, Wh, el, er, stats, out, dy, a_src, a_dst, heads, fh,
                                          slope, mode, activation == "elu", drop_p, seed,
                                          dy_dropout=out_drop)
        n = Wh.shape[0]
        da_src, da_dst = _attention_vector_grads(Wh.detach(), dl, der, heads, fh)
        if mode == GAT_DENSE and g.has_empty_rows():
            # an edgeless row is the uniform average of every row (layers.py:29-32)
            empty = (g.rowptr[1:] - g.rowptr[:-1]) == 0
            dwh = dwh + dout[empty].sum(0) / n
        return dwh, da_src, da_dst, None, None, None, None, None, None, None, None, None


def _padded_fh(heads: int, fh: int, Wh) -> int:
    """fh, or the head width to zero-pad to when the two-pass backward refuses fh but takes the
    next power of two (>= 4: 16-B rows): 3 -> 4, 7 -> 8, 12 -> 16."""
    if not Wh.is_cuda or _bwd_recompute_ok(heads, fh, Wh.stride(0)):
        return fh
    fp = max(4, 1 << (fh - 1).bit_length())
    return fp if _bwd_recompute_ok(heads, fp, heads * fp) else fh


def _attention_vector_grads(Wh, dl, der, heads, fh):
    """d a_src[h, f] = sum_n dl[n, h] Wh[n, h, f] (el = a_src . Wh) and likewise d a_dst with der:
    the diagonal [h, h*fh:(h+1)*fh] blocks of dl^T Wh and der^T Wh -- both from ONE pass over
    Wh ([dl | der]^T Wh, gnn_gemm_tn_f32) where the shape is covered, else one pass each, else
    the torch reduction."""
    both = gemm_tn(torch.cat([dl, der], 1), Wh)
    if both is not None:
        c = both[0].view(2, heads, heads, fh)
        idx = torch.arange(heads, device=Wh.device)
        return c[0, idx, idx].reshape(-1), c[1, idx, idx].reshape(-1)
    out = []
    for g in (dl, der):
        r = gemm_tn(g, Wh)
        if r is None:
            out.append((g.unsqueeze(-1) * Wh.view(-1, heads, fh)).sum(0).reshape(-1))
        else:
            c = r[0].view(heads, heads, fh)
            out.append(c[torch.arange(heads), torch.arange(heads)].reshape(-1))
    return out[0], out[1]


class _ProjectFn(torch.autograd.Function):
    """Wh = x W (layers.py:23 / :97, all heads side by side) on the MFMA transform (torch.mm where
    it does not cover the shape) with the weight gradient dW = x^T dWh by gnn_gemm_tn_f32 (a
    K = N reduction; hipBLASLt parallelises it badly)."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return _transform_or_mm(x, W.t())  # the MFMA transform (x W = x (W^T)^T)

    @staticmethod
    def backward(ctx, dwh):
        x, W = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _transform_or_mm(dwh, W)
        if ctx.needs_input_grad[1]:
            r = gemm_tn(x, dwh.contiguous())
            dw = r[0] if r is not None else torch.mm(x.t(), dwh)
        return dx, dw


def _project(x, W, heads, fh, a_src, a_dst):
    """(Wh, (el, er) or None): the fused MFMA transform + logits kernel at inference when
    the shape is covered (gnn_gat_project_f32), else torch.mm (autograd) and logits later."""
    if not (torch.is_grad_enabled() and (x.requires_grad or W.requires_grad
                                         or a_src.requires_grad or a_dst.requires_grad)) \
            and x.is_cuda:
        r = gat_project(x, W, heads, fh, a_src, a_dst)
        if r is not None:
            return r[0], (r[1], r[2])
    if x.is_cuda and x.dtype == torch.float32 and W.dtype == torch.float32 \
            and torch.is_grad_enabled() and (x.requires_grad or W.requires_grad):
        return _ProjectFn.apply(x, W), None
    return torch.mm(x, W), None


def _inference(x, *params) -> bool:
    return x.is_cuda and not (torch.is_grad_enabled() and
                              (x.requires_grad or any(p.requires_grad for p in params)))


def _dropout_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _AttentionBase(nn.Module):
    MODE = GAT_DENSE
    PREDICATE = "positive"

    def _a_parts(self):
        a = self.a.reshape(-1)
        F_ = self.out_features
        return a[:F_], a[F_:]

    def _aggregate(self, Wh, adj, heads, fh, a_src, a_dst, activation, dropout_p, logits=None,
                   out_drop=0.0):
        """The layer's output, followed by F.dropout(., out_drop) when out_drop > 0 (the GAT
        model's hidden dropout: fused into the layer's autograd op on the hashed kernel, whose
        mask the backward prep applies; else model_dropout on the output)."""
        g = as_csr(adj, self.PREDICATE)
        p = dropout_p if self.training else 0.0
        seed = _dropout_seed() if p > 0 else 0
        if torch.is_grad_enabled() and (Wh.requires_grad or a_src.requires_grad
                                        or a_dst.requires_grad):
            fp = _padded_fh(heads, fh, Wh)
            if fp != fh:
                # head width the two-pass backward cannot lay out (e.g. a 7-class out_att):
                # zero-pad each head to fp features -- zero a-weights, so the logits and the
                # first fh output columns are unchanged -- and slice the output back
                n = Wh.shape[0]
                whp = F.pad(Wh.reshape(n, heads, fh), (0, fp - fh)).reshape(n, heads * fp)
                asp = F.pad(a_src.reshape(heads, fh), (0, fp - fh)).reshape(-1)
                adp = F.pad(a_dst.reshape(heads, fh), (0, fp - fh)).reshape(-1)
                out = _GatLayerFn.apply(whp, asp, adp, g, heads, fp, self.alpha, self.MODE,
                                        activation, p, seed)
                out = out.view(n, heads, fp)[:, :, :fh].reshape(n, heads * fh)
            else:
                od = None
                if out_drop > 0 and GAT_FUSE_OUT_DROPOUT and HASHED_DROPOUT_OK(Wh, out_drop):
                    od = (float(out_drop), _ops.dropout_seed())  # after the attention's seed
                out = _GatLayerFn.apply(Wh, a_src, a_dst, g, heads, fh, self.alpha, self.MODE,
                                        activation, p, seed, od)
                if od is not None:
                    out_drop = 0.0  # applied
        else:
            el, er = logits if logits is not None else gat_logits(Wh, heads, fh, a_src, a_dst)
            out = gat_aggregate(g, Wh, el, er, heads, fh, self.alpha, self.MODE, activation,
                                dropout_p=p, seed=seed, a_dst=a_dst)
        if self.MODE == GAT_SPARSE and SPARSE_NAN_CHECK:
            assert not torch.isnan(out).any()  # dropout keeps NaNs (x * 0): same verdict
        if out_drop > 0:
            out = model_dropout(out, out_drop, True)
        return out

    def _ordered(self, x, W, heads, fh, a_src, a_dst, adj, activation):
        """Inference over the column-degree-ordered graph A P^T (ops.gat_column_order): the
        projection writes Wh / er in its column order (el in place) and the aggregation reads
        the hub rows of Wh / er in place. Same values, output rows in the original order.
        None when it does not apply (training, dropout, small graph, uncovered shape)."""
        if self.training or not _inference(x, W, a_src, a_dst):
            return None
        g = as_csr(adj, self.PREDICATE)
        if g.n_rows != x.shape[0] or g.n_cols != x.shape[0]:
            return None
        order = gat_column_order(g, heads, fh)
        if order is None:
            return None
        r = gat_project(x, W, heads, fh, a_src, a_dst, col_rows=order.inv)
        if r is None:
            return None
        Wh, el, er = r
        if self.MODE == GAT_SPARSE and SPARSE_NAN_CHECK:
            assert not torch.isnan(Wh).any()
        out = gat_aggregate(order.graph, Wh, el, er, heads, fh, self.alpha, self.MODE, activation,
                            a_dst=a_dst)
        if self.MODE == GAT_SPARSE and SPARSE_NAN_CHECK:
            assert not torch.isnan(out).any()
        return out

    def forward(self, h, adj, activation: str | None = "__concat__"):
        if activation == "__concat__":
            activation = "elu" if self.concat else None
        a_src, a_dst = self._a_parts()
        out = self._ordered(h, self.W, 1, self.out_features, a_src, a_dst, adj, activation)
        if out is not None:
            return out
        Wh, logits = _project(h, self.W, 1, self.out_features, a_src, a_dst)
        if self.MODE == GAT_SPARSE and SPARSE_NAN_CHECK:
            assert not torch.isnan(Wh).any()
        return self._aggregate(Wh, adj, 1, self.out_features, a_src, a_dst, activation,
                               self._drop_p(), logits)

    def __repr__(self):
        return self.__class__.__name__ + ' (' + str(self.in_features) + ' -> ' + str(self.out_features) + ')'


class GraphAttentionLayer(_AttentionBase):
    """GAT/models/layers.py:6-40 (dense attention, edges = adj > 0)."""

    MODE = GAT_DENSE
    PREDICATE = "positive"

    def __init__(self, in_features, out_features, dropout, alpha, concat=True, **kwargs):
        super().__init__(**kwargs)
        self.dropout = dropout
        self.in_features = in_features
        self.out_features = out_features
        self.alpha = alpha
        self.concat = concat
        self.W = nn.Parameter(torch.empty(size=(in_features, out_features)))
        nn.init.xavier_uniform_(self.W.data, gain=1.414)
        self.a = nn.Parameter(torch.empty(size=(2 * out_features, 1)))
        nn.init.xavier_uniform_(self.a.data, gain=1.414)
        self.leakyrelu = nn.LeakyReLU(self.alpha)

    def _drop_p(self):
        return float(self.dropout)


class SpGraphAttentionLayer(_AttentionBase):
    """GAT/models/layers.py:72-134 (sparse attention, edges = adj.nonzero())."""

    MODE = GAT_SPARSE
    PREDICATE = "nonzero"

    def __init__(self, in_features, out_features, dropout, alpha, concat=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.alpha = alpha
        self.concat = concat
        self.W = nn.Parameter(torch.zeros(size=(in_features, out_features)))
        nn.init.xavier_normal_(self.W.data, gain=1.414)
        self.a = nn.Parameter(torch.zeros(size=(1, 2 * out_features)))
        nn.init.xavier_normal_(self.a.data, gain=1.414)
        self.dropout = nn.Dropout(dropout)
        self.leakyrelu = nn.LeakyReLU(self.alpha)

    def _drop_p(self):
        return float(self.dropout.p)


class _HeadParams(torch.autograd.Function):
    """The H heads' parameters side by side: W = [W_1 | ... | W_H] ([in, H fh]), a_src / a_dst
    = the heads' a[:fh] / a[fh:] concatenated (GAT.py:16 runs the heads as one layer here).
    Backward hands every head its gradients as contiguous views of two buffers -- dW
    regrouped per head by one copy, [da_src | da_dst] per head by one -- which AccumulateGrad
    takes as they are: two kernels per step where torch.cat / slicing autograd took ~40 tiny
    copies, fills and adds (~0.2 ms at cfg3, profiles/r06f_*)."""

    @staticmethod
    def forward(ctx, n_heads, *params):
        Ws, As = params[:n_heads], params[n_heads:]
        fh = Ws[0].shape[1]
        ctx.shapes = (n_heads, Ws[0].shape[0], fh, [a.shape for a in As])
        a = torch.stack([t.reshape(-1) for t in As])  # [H, 2 fh]
        return (torch.cat(Ws, dim=1), a[:, :fh].reshape(-1).contiguous(),
                a[:, fh:].reshape(-1).contiguous())

    @staticmethod
    def backward(ctx, dW, da_src, da_dst):
        H, fin, fh, a_shapes = ctx.shapes
        dWs = dW.reshape(fin, H, fh).permute(1, 0, 2).contiguous()          # [H, in, fh]
        da = torch.cat([da_src.reshape(H, fh), da_dst.reshape(H, fh)], dim=1)  # [H, 2 fh]
        return (None, *[dWs[h] for h in range(H)],
                *[da[h].view(a_shapes[h]) for h in range(H)])


class GATBase(nn.Module):
    """GAT/models/GAT.py:7-18: dropout -> concat(heads) -> dropout -> ELU(out_att).

    Training on a large symmetric graph runs the whole model over P A P^T (``gat_train_order``:
    nodes relabelled once by degree): x is permuted once on entry and the logits once on exit,
    so every attention layer's forward and both backward passes read their hub rows at the top
    of Wh / er / dout. Same function; the dropout draws fall on the relabelled rows / edges.
    In training the two F.dropout calls run as hashed element masks that are never stored
    (``ops.model_dropout``: (seed, row, column) hash, the first fused with the relabelling)."""

    def __init__(self, dropout, **kwargs):
        super().__init__(**kwargs)
        self.dropout = dropout
        self.attentions = nn.ModuleList()
        self.out_att = None

    def _heads(self, x, adj, out_drop: float = 0.0):
        """concat(heads) (GAT.py:16) followed by F.dropout(., out_drop) (GAT.py:17; 0 = none)."""
        heads = list(self.attentions)
        first = heads[0]
        uniform = all(type(m) is type(first) and m.concat and m.alpha == first.alpha
                      and m.out_features == first.out_features
                      and m._drop_p() == first._drop_p() for m in heads)
        if not uniform:
            return model_dropout(torch.cat([att(x, adj) for att in heads], dim=1), out_drop,
                                 out_drop > 0)
        fh = first.out_features
        W, a_src, a_dst = _HeadParams.apply(len(heads), *[m.W for m in heads],
                                            *[m.a for m in heads])  # [in, H*fh], [H*fh] x 2
        out = first._ordered(x, W, len(heads), fh, a_src, a_dst, adj, "elu")
        if out is not None:
            return model_dropout(out, out_drop, out_drop > 0)
        Wh, logits = _project(x, W, len(heads), fh, a_src, a_dst)  # one MFMA pass, all heads
        if first.MODE == GAT_SPARSE and SPARSE_NAN_CHECK:
            assert not torch.isnan(Wh).any()
        return first._aggregate(Wh, adj, len(heads), fh, a_src, a_dst, "elu", first._drop_p(),
                                logits, out_drop=out_drop)

    def _train_order(self, x, adj):
        """The node order training runs in (None: the graph's own, e.g. at inference, where
        ``_ordered`` takes the column order instead)."""
        if not (x.is_cuda and torch.is_grad_enabled()
                and (x.requires_grad or any(p.requires_grad for p in self.parameters()))):
            return None
        heads = list(self.attentions)  # keys AttentionHead{i}: no integer indexing
        if not heads:
            return None
        g = as_csr(adj, heads[0].PREDICATE)
        if g.n_rows != x.shape[0]:
            return None
        return gat_train_order(g, len(heads), heads[0].out_features)

    def forward(self, x, adj):
        order = self._train_order(x, adj)
        if order is not None:  # relabel and drop out in one pass
            x = model_dropout(x, self.dropout, self.training, order.perm, order.inv)
            adj = order.graph
        else:
            x = model_dropout(x, self.dropout, self.training)
        x = self._heads(x, adj, self.dropout if self.training else 0.0)  # + F.dropout (GAT.py:17)
        out = self.out_att(x, adj, activation="elu")  # F.elu(out_att(x)) fused (concat=False)
        if order is not None:
            out = PermuteRows.apply(out, order.inv, order.perm)
        return out


class GAT(GATBase):
    """GAT/models/GAT.py:21-28 (dense version)."""

    def __init__(self, nfeat, nhid, nclass, dropout, alpha, nheads, **kwargs):
        super().__init__(dropout, **kwargs)
        for i in range(nheads):
            self.attentions.add_module(f'AttentionHead{i}',
                                       GraphAttentionLayer(nfeat, nhid, dropout=dropout, alpha=alpha, concat=True))
        self.out_att = GraphAttentionLayer(nhid * nheads, nclass, dropout=dropout, alpha=alpha, concat=False)


class SpGAT(GATBase):
    """GAT/models/GAT.py:31-38 (sparse version)."""

    def __init__(self, nfeat, nhid, nclass, dropout, alpha, nheads, **kwargs):
        super().__init__(dropout, **kwargs)
        for i in range(nheads):
            self.attentions.add_module(f'AttentionHead{i}',
                                       SpGraphAttentionLayer(nfeat, nhid, dropout=dropout, alpha=alpha, concat=True))
        self.out_att = SpGraphAttentionLayer(nhid * nheads, nclass, dropout=dropout, alpha=alpha, concat=False)
