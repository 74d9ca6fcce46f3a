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
``a_input`` per head.  The semantic attention over the M metapath embeddings is
a few small dense ops and stays in PyTorch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .gat import GATBase, GraphAttentionLayer


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
        z = torch.stack([gat(h, g).flatten(1) for g, gat in zip(gs, self.gat_layers)], dim=1)
        return self.semantic_attention(z)


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
