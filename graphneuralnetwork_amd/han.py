"""Drop-in HAN modules on the GAT kernels (reference: HAN/models/NodeAttention.py,
HAN/models/SemanticAttention.py, HAN/models/HAN.py) -- SURVEY 8f row 4.

Same class names, constructor arguments, ``forward`` signatures and state_dict
keys (``layers.{l}.gat_layers.meta_path_model{m}.attentions.AttentionHead{i}.W``
/ ``.a``, ``layers.{l}.semantic_attention.project.{0,2}.*``, ``predict.*``).

The node-level attention of each metapath graph is the dense GAT layer of
``GAT/models/layers.py`` (HAN/models/NodeAttention.py:6-40 is the same layer),
so every ``GATConv`` runs as one GEMM for all heads + one logits launch + one
fused edge-softmax/aggregation launch over the metapath's CSR (built once per
adjacency tensor and cached), instead of the reference's N x N x 2F
``a_input`` per head.  At inference a ``HANLayer`` goes further: the M metapath
graphs are interleaved into ONE block-diagonal CSR (row n*M + m = node n in
metapath m), so all metapaths x heads take one GEMM and one aggregation launch,
and the result is already the [N, M, H*F] stack the semantic attention reads.
The semantic attention over the M metapath embeddings is a few small dense ops
and stays in PyTorch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .gat import GATBase, GraphAttentionLayer, _project
from .graph import as_csr, from_coo
from .ops import GAT_DENSE, gat_aggregate, gat_logits

# one aggregation launch for all metapaths at inference (HANLayer._batched)
BATCH_METAPATHS = True


class GATConv(GATBase):
    """HAN/models/NodeAttention.py:44-62: dropout -> concat of ELU'd heads -> dropout ->
    ELU(out_att) when ``num_class`` is given, else ELU of the concat (applied a second
    time, exactly like the reference)."""

    def __init__(self, feat_size, hidden_size, dropout, num_heads, alpha=0.2, num_class=None,
                 **kwargs):
        super().__init__(dropout, **kwargs)
        for i in range(num_heads):
            self.attentions.add_module(f'AttentionHead{i}',
                                       GraphAttentionLayer(feat_size, hidden_size, dropout=dropout,
                                                           alpha=alpha, concat=True))
        self.num_class = num_class
        if num_class is not None:
            self.out_att = GraphAttentionLayer(hidden_size * num_heads, num_class, dropout=dropout,
                                               alpha=alpha, concat=False)
        else:
            del self.out_att   # no such submodule / attribute in the reference

    def forward(self, x, adj):
        x = F.dropout(x, self.dropout, training=self.training)
        x = self._heads(x, adj)
        x = F.dropout(x, self.dropout, training=self.training)
        if self.num_class is not None:
            return self.out_att(x, adj, activation="elu")  # F.elu(out_att(x)) fused
        return F.elu(x)


class SemanticAttention(nn.Module):
    """HAN/models/SemanticAttention.py:5-20 (metapath-level attention)."""

    def __init__(self, in_size, hidden_size=128):
        super().__init__()
        self.project = nn.Sequential(nn.Linear(in_size, hidden_size), nn.Tanh(),
                                     nn.Linear(hidden_size, 1, bias=False))

    def forward(self, z):
        beta = torch.softmax(self.project(z).mean(0), dim=0)      # (M, 1)
        return (beta.unsqueeze(0) * z).sum(1)                      # (N, D * K)


class HANLayer(nn.Module):
    """HAN/models/HAN.py:7-23: one GATConv per metapath graph + semantic attention."""

    def __init__(self, num_meta_paths, in_size, out_size, layer_num_heads, dropout, **kwargs):
        super().__init__(**kwargs)
        self.gat_layers = nn.ModuleList()
        for i in range(num_meta_paths):
            self.gat_layers.add_module(f'meta_path_model{i}',
                                       GATConv(in_size, out_size, dropout, layer_num_heads))
        self.semantic_attention = SemanticAttention(in_size=out_size * layer_num_heads)

    def forward(self, gs, h):
        z = self._batched(gs, h) if self._batch_ok(gs, h) else None
        if z is None:
            z = torch.stack([gat(h, g).flatten(1) for g, gat in zip(gs, self.gat_layers)], dim=1)
        return self.semantic_attention(z)

    def _batch_ok(self, gs, h) -> bool:
        if not (BATCH_METAPATHS and not self.training and not torch.is_grad_enabled()
                and h.is_cuda and len(gs) == len(self.gat_layers) and len(gs) > 1):
            return False
        convs = list(self.gat_layers)     # keys are meta_path_model{i}: no integer indexing
        first = next(iter(convs[0].attentions))
        return all(type(m) is GraphAttentionLayer and m.concat and m.alpha == first.alpha
                   and m.alpha > 0 and m.out_features == first.out_features
                   and len(conv.attentions) == len(convs[0].attentions)
                   and conv.num_class is None
                   for conv in convs for m in conv.attentions)

    def _block_graph(self, gs, n):
        """The M metapath CSRs interleaved: edge (i, j) of metapath m becomes
        (i*M + m, j*M + m); each row keeps its metapath's edge order. Cached against the
        metapath CsrGraphs (themselves cached per adjacency tensor by as_csr). None when a
        metapath graph has an edgeless row (its uniform-average fill is per metapath, not
        over the block)."""
        csrs = [as_csr(g, "positive") for g in gs]
        cached = getattr(self, "_block_cache", None)
        if cached is not None and len(cached[0]) == len(csrs) \
                and all(a is b for a, b in zip(cached[0], csrs)):
            return cached[1]
        M = len(gs)
        rows, cols = [], []
        block = None
        if all(c.n_rows == n and c.n_cols == n and not c.has_empty_rows() for c in csrs):
            for m, c in enumerate(csrs):
                r = torch.repeat_interleave(torch.arange(n, device=c.device), c.rowptr[1:] - c.rowptr[:-1])
                rows.append(r * M + m)
                cols.append(c.col.to(torch.int64) * M + m)
            r, cc = torch.cat(rows), torch.cat(cols)
            block = from_coo(r, cc, torch.ones(r.numel(), device=r.device), n * M, n * M,
                             check=False)
        self._block_cache = (csrs, block)
        return block

    def _batched(self, gs, h):
        """[N, M, H*F] for all metapaths: one GEMM, the logits, one aggregation launch over
        the block graph (ELU per head), then GATConv's own second ELU
        (HAN/models/NodeAttention.py:58-62 applied to every metapath at once)."""
        n, M = h.shape[0], len(gs)
        gb = self._block_graph(gs, n)
        if gb is None:
            return None
        heads = [list(conv.attentions) for conv in self.gat_layers]
        H, fh = len(heads[0]), heads[0][0].out_features
        flat = [m for hs in heads for m in hs]                               # head m*H + i
        W = torch.cat([m.W for m in flat], dim=1)                            # [in, M*H*fh]
        a_src = torch.cat([m._a_parts()[0] for m in flat])
        a_dst = torch.cat([m._a_parts()[1] for m in flat])
        wh, logits = _project(h, W, M * H, fh, a_src, a_dst)                 # [N, M*H*fh]
        if logits is None:
            logits = gat_logits(wh, M * H, fh, a_src, a_dst)
        el, er = (t.reshape(n * M, H) for t in logits)
        out = gat_aggregate(gb, wh.view(n * M, H * fh), el, er, H, fh, heads[0][0].alpha,
                            GAT_DENSE, "elu")
        return F.elu(out.view(n, M, H * fh))


class HANModel(nn.Module):
    """HAN/models/HAN.py:26-41."""

    def __init__(self, num_mate_paths, in_size, hidden_size, out_size, num_heads, dropout,
                 **kwargs):
        super().__init__(**kwargs)
        self.layers = nn.ModuleList()
        self.layers.append(HANLayer(num_mate_paths, in_size, hidden_size, num_heads[0], dropout))
        for layer in range(1, len(num_heads)):
            self.layers.append(HANLayer(num_mate_paths, hidden_size * num_heads[layer - 1],
                                        hidden_size, num_heads[layer], dropout))
        self.predict = nn.Linear(hidden_size * num_heads[-1], out_size)

    def forward(self, g, h):
        for gnn in self.layers:
            h = gnn(g, h)
        return self.predict(h)
