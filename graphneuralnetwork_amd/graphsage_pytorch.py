"""Drop-in GraphSAGE_Pytorch modules on the SAGE kernels (reference:
GraphSAGE_Pytorch/models/{Aggregator,SageGCN,GraphSage}.py and
GraphSAGE_Pytorch/sample_utils.py) -- SURVEY 8f row 4.

Same class names, constructor arguments, ``forward`` signatures and state_dict
keys (``gcn.{l}.weight``, ``gcn.{l}.aggregator.weight`` / ``.bias``).

* ``NeighborAggregator`` 'mean' / 'sum' -> one HIP reduction launch
  (gnn_sage_aggregate_f32, GNN_SAGE_MEAN / GNN_SAGE_SUM) + the MFMA GEMM;
  'max' keeps the reference's behaviour (``Tensor.max(dim=1)`` is a
  (values, indices) pair and ``torch.matmul`` rejects it with a TypeError).
* ``SageGCN`` 'sum' hidden: ``src @ W + agg @ W_agg`` as one addmm (no separate
  add); 'concat' as in the reference.
* ``GraphSage.forward`` takes the reference's list of per-hop feature tensors;
  any hop may instead be a ``Gathered(table, ids)`` (see ``multihop_sampling``),
  in which case the hop's neighbour rows are reduced straight from the table
  (fused gather + reduction) and never materialised.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .graph import CsrGraph
from .graphsage import Gathered, _gather, reduce_neighbors

_KINDS = {"mean": "MEAN", "sum": "SUM"}


def _nbr_view(feat, n_src: int, k: int):
    """hidden[hop + 1].view(n_src, k, -1), for a tensor or a Gathered hop."""
    if isinstance(feat, Gathered):
        return Gathered(feat.table, feat.index.reshape(n_src, k), feat.trusted)
    return feat.view((n_src, k, -1))


def _rows(feat):
    """A hop's feature rows as a tensor (row gather for a Gathered hop)."""
    return _gather(feat.table, feat.index.reshape(-1), feat.trusted) if isinstance(feat, Gathered) else feat


def _len(feat) -> int:
    return feat.index.numel() if isinstance(feat, Gathered) else len(feat)


class NeighborAggregator(nn.Module):
    """GraphSAGE_Pytorch/models/Aggregator.py:5-37."""

    def __init__(self, input_dim, output_dim, use_bias=False, aggr_method="mean", **kwargs):
        super().__init__()
        self.input_dim = input_dim
        self.output_dim = output_dim
        self.use_bias = use_bias
        self.aggr_method = aggr_method
        self.weight = nn.Parameter(torch.Tensor(input_dim, output_dim))
        nn.init.xavier_uniform_(self.weight)
        if self.use_bias:
            self.bias = nn.Parameter(torch.zeros(self.output_dim))

    def aggregate(self, neighbor_feature):
        if self.aggr_method in _KINDS:
            return reduce_neighbors(neighbor_feature, _KINDS[self.aggr_method])
        if self.aggr_method == "max":
            feats = neighbor_feature
            if isinstance(feats, Gathered):
                feats = feats.table[feats.index]
            return feats.max(dim=1)  # (values, indices): the reference's matmul then fails
        raise ValueError("Unknown aggr type, expected sum, max, or mean, but got {}"
                         .format(self.aggr_method))

    def forward(self, neighbor_feature):
        aggr_neighbor = self.aggregate(neighbor_feature)
        if self.use_bias:
            return torch.addmm(self.bias, aggr_neighbor, self.weight)
        return torch.matmul(aggr_neighbor, self.weight)

    def extra_repr(self):
        return 'in_features={}, out_features={}, aggr_method={}'.format(
            self.input_dim, self.output_dim, self.aggr_method)


class SageGCN(nn.Module):
    """GraphSAGE_Pytorch/models/SageGCN.py:7-41."""

    def __init__(self, input_dim, hidden_dim, activation=F.relu, aggr_neighbor_method="mean",
                 aggr_hidden_method="sum", **kwargs):
        super().__init__(**kwargs)
        assert aggr_neighbor_method in ["mean", "sum", "max"]
        assert aggr_hidden_method in ["sum", "concat"]
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.aggr_neighbor_method = aggr_neighbor_method
        self.aggr_hidden_method = aggr_hidden_method
        self.activation = activation
        self.aggregator = NeighborAggregator(input_dim, hidden_dim,
                                             aggr_method=aggr_neighbor_method)
        self.weight = nn.Parameter(torch.Tensor(input_dim, hidden_dim))
        nn.init.xavier_uniform_(self.weight)

    def forward(self, src_node_features, neighbor_node_features):
        src = _rows(src_node_features)
        agg = self.aggregator
        if self.aggr_hidden_method == "sum" and agg.aggr_method in _KINDS and not agg.use_bias:
            # self_hidden + neighbor_hidden as ONE GEMM accumulation
            hidden = torch.addmm(torch.matmul(src, self.weight),
                                 agg.aggregate(neighbor_node_features), agg.weight)
        else:
            neighbor_hidden = agg(neighbor_node_features)
            self_hidden = torch.matmul(src, self.weight)
            if self.aggr_hidden_method == "sum":
                hidden = self_hidden + neighbor_hidden
            else:
                hidden = torch.cat([self_hidden, neighbor_hidden], dim=1)
        return self.activation(hidden) if self.activation else hidden

    def extra_repr(self):
        output_dim = self.hidden_dim if self.aggr_hidden_method == "sum" else self.hidden_dim * 2
        return 'in_features={}, out_features={}, aggr_hidden_method={}'.format(
            self.input_dim, output_dim, self.aggr_hidden_method)


class GraphSage(nn.Module):
    """GraphSAGE_Pytorch/models/GraphSage.py:5-34."""

    def __init__(self, input_dim, hidden_dim, num_neighbors_list):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.num_neighbors_list = num_neighbors_list
        self.num_layers = len(num_neighbors_list)
        self.gcn = nn.ModuleList()
        self.gcn.append(SageGCN(input_dim, hidden_dim[0]))
        for index in range(0, len(hidden_dim) - 2):
            self.gcn.append(SageGCN(hidden_dim[index], hidden_dim[index + 1]))
        self.gcn.append(SageGCN(hidden_dim[-2], hidden_dim[-1], activation=None))

    def forward(self, node_features_list):
        hidden = node_features_list
        for layer in range(self.num_layers):
            gcn = self.gcn[layer]
            nxt = []
            for hop in range(self.num_layers - layer):
                n_src = _len(hidden[hop])
                nbr = _nbr_view(hidden[hop + 1], n_src, self.num_neighbors_list[hop])
                nxt.append(gcn(hidden[hop], nbr))
            hidden = nxt
        return hidden[0]

    def extra_repr(self):
        return 'in_features={}, num_neighbors_list={}'.format(self.input_dim,
                                                              self.num_neighbors_list)


def multihop_sampling(src_nodes, sample_nums, adj: CsrGraph, seed: int = 0):
    """Device form of GraphSAGE_Pytorch/sample_utils.py:22-35: hop k+1 = ``sample_nums[k]``
    neighbours of every hop-k node (random.sample without replacement when the node has
    enough neighbours, random.choices with replacement otherwise), flattened in node
    order like the reference's ``results.extend``.  Returns int64 id tensors."""
    from .sampler import sample_neighbors
    hops = [torch.as_tensor(src_nodes, dtype=torch.int64, device=adj.device).reshape(-1)]
    for k, n in enumerate(sample_nums):
        hops.append(sample_neighbors(adj, hops[k], int(n), seed, layer=k).reshape(-1))
    return hops
