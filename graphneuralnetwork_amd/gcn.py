"""Drop-in GCN modules (reference: GCN/GCN.py).

Same class names, constructor arguments, parameter names/shapes
(``gcn_blocks.gcn{i}.dense.weight`` [out, in], ``gcn_blocks.gcn{i}.bias`` [out])
and ``forward(X, adj)`` signature as the reference, so reference checkpoints
load unchanged.  ``GCN_Model.forward`` dispatches on the class-name string
exactly like GCN/GCN.py:23, which is why the layer class keeps the name
``Graph_conv_layer``.

The aggregation ``torch.spmm(adj, support) + bias`` (GCN/GCN.py:43-45) runs
as ONE gfx950 kernel launch (CSR SpMM with the bias fused into its epilogue);
the feature transform ``support = dense(X)`` is an fp32 MFMA GEMM: the hand-written
``gnn_gcn_transform_f32`` for the shapes it covers (F_in/F_out 64-256), otherwise nn.Linear
on hipBLASLt. Under autograd the layer is one differentiable op (``ops.gcn_layer``): the same
forward, and a backward of the SpMM over A^T (A itself: the normalised adjacency is
symmetric), the MFMA transform for dX and the tall-skinny A^T B kernel (gnn_gemm_tn_f32) for
dW and d bias in one pass. ``adj`` may be the
reference's sparse COO tensor, a sparse CSR tensor, a dense tensor or a prebuilt ``CsrGraph``;
the CSR form is cached on the adjacency tensor.

On graphs large enough for the XCD-sliced hub staging, the inference layer runs over the
column-degree-ordered graph A P^T (``ops.column_order``): the transform writes the support
rows in that order and the SpMM reads the hub rows in place, with no per-call staging copy.
Training ``GCN_Model`` on such a (symmetric) graph runs every layer over P A P^T
(``ops.gcn_train_order``: X permuted once on entry, the logits once on exit), so the backward
SpMM dS = A dY reads its hub rows in place too. In training, a layer with in_features <=
out_features runs as (A X) W^T + b (ops._GcnLayerFn), and a Graph_conv_layer -> ReLU ->
Dropout triple of such a layer as one op: ReLU and (hashed) dropout in the transform's store
epilogue, their backward folded into the weight-gradient pass (``_fuse_train``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .graph import as_csr
from . import ops
from .ops import (PermuteRows, column_order, dropout_seed, fuses_relu_dropout, gcn_layer,
                  gcn_train_order, gcn_transform, row_order_graph, spmm, spmm_forward)


class GCN_Model(nn.Module):
    """GCN/GCN.py:5-27."""

    def __init__(self, num_features, num_hidden, num_classes, num_layers, dropout, **kwargs):
        super().__init__(**kwargs)
        self.gcn_blocks = nn.Sequential()
        for i in range(num_layers):
            if i == 0:
                self.gcn_blocks.add_module(f'gcn{i}', Graph_conv_layer(num_features, num_hidden))
                self.gcn_blocks.add_module(f'relu{i}', nn.ReLU())
                self.gcn_blocks.add_module(f'dropout{i}', nn.Dropout(dropout))
            elif i == num_layers - 1:
                self.gcn_blocks.add_module(f'gcn{i}', Graph_conv_layer(num_hidden, num_classes))
            else:
                self.gcn_blocks.add_module(f'gcn{i}', Graph_conv_layer(num_hidden, num_hidden))
                self.gcn_blocks.add_module(f'relu{i}', nn.ReLU())
                self.gcn_blocks.add_module(f'dropout{i}', nn.Dropout(dropout))

    def _train_order(self, X, adj):
        """The degree-ordered graph P A P^T training runs over (ops.gcn_train_order), or None
        (inference -- the layers take the column order there -- or a graph it does not pay
        for)."""
        if not (isinstance(X, torch.Tensor) and X.is_cuda and torch.is_grad_enabled()
                and (X.requires_grad or any(p.requires_grad for p in self.parameters()))):
            return None
        layers = [m for m in self.gcn_blocks if isinstance(m, Graph_conv_layer)]
        if not layers:
            return None
        g = as_csr(adj)
        if g.n_cols != X.shape[0]:
            return None
        return gcn_train_order(g, layers[0].out_features)

    def forward(self, X, adj):
        order = self._train_order(X, adj)
        first = None
        if order is not None:
            # training over P A P^T: X in on its rows once, the logits back out once; every
            # layer's SpMM (forward, and dS = A dY in backward) reads its hub rows in place. A
            # first layer over features without gradient reads X as it is through P A instead
            # (its output rows land in the degree order all the same)
            if self._first_rows(X, order.graph):
                first = row_order_graph(as_csr(adj))
            else:
                X = PermuteRows.apply(X, order.perm, order.inv)
            adj = order.graph
        X = self._blocks(X, adj, first)
        if order is not None:
            X = PermuteRows.apply(X, order.inv, order.perm)
        return X

    def _first_rows(self, X, g) -> bool:
        blocks = list(self.gcn_blocks)
        b = blocks[0] if blocks else None
        return (ops.GCN_FIRST_ROWS and not X.requires_grad and isinstance(b, Graph_conv_layer)
                and not (b._forward_hooks or b._forward_pre_hooks)
                and ops._reassociate(X, b.dense.weight, g))

    def _blocks(self, X, adj, first=None):
        """The Sequential's modules in order (GCN/GCN.py:22-27), with the fusions above; the
        first Graph_conv_layer runs over ``first`` when given (P A, see forward)."""
        blocks = list(self.gcn_blocks)
        i = 0
        while i < len(blocks):
            gcn_block = blocks[i]
            if gcn_block._get_name() == 'Graph_conv_layer':
                g_i = first if (i == 0 and first is not None) else adj
                nxt = blocks[i + 1] if i + 1 < len(blocks) else None
                span = _fuse_train(gcn_block, nxt, blocks[i + 2] if i + 2 < len(blocks) else None,
                                   X, g_i)
                if span:
                    # Graph_conv_layer -> ReLU (-> Dropout) in training: one op, ReLU and dropout
                    # in the transform's epilogue (GCN/GCN.py:12-14)
                    drop = blocks[i + 2] if span == 3 else None
                    p = drop.p if drop is not None and drop.training else 0.0
                    X = gcn_layer(as_csr(g_i), X, gcn_block.dense.weight, gcn_block.bias,
                                  relu_dropout=(p, dropout_seed() if p > 0 else 0))
                    i += span
                    continue
                if _fuse_relu(gcn_block, nxt, X):
                    # the ReLU in the SpMM's store epilogue (GNN_EPI_RELU): one pass over the
                    # [n, hidden] activations fewer at inference
                    X = gcn_block._forward(X, g_i, 'relu')
                    i += 2
                    continue
                X = gcn_block(X, g_i)
            else:
                X = gcn_block(X)
            i += 1
        return X


def _no_hooks(*mods) -> bool:
    return not any(m._forward_hooks or m._forward_pre_hooks for m in mods)


def _fuse_train(block, nxt, nxt2, X, adj) -> int:
    """How many modules from ``block`` run as one training op (0: none): 3 for
    Graph_conv_layer -> nn.ReLU -> nn.Dropout, 2 for Graph_conv_layer -> nn.ReLU (a Dropout
    with hooks runs on its own), when the layer trains in the reassociated form on a transform
    shape (ops.fuses_relu_dropout) and none of the fused modules has hooks (they would not run).
    """
    if not (isinstance(block, Graph_conv_layer) and type(nxt) is nn.ReLU
            and isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.float32
            and torch.is_grad_enabled() and _no_hooks(block, nxt)):
        return 0
    if not (X.requires_grad or any(p.requires_grad for p in block.parameters())):
        return 0
    g = as_csr(adj)
    if X.dim() != 2 or X.shape[1] != block.in_features or not fuses_relu_dropout(
            X, block.dense.weight, g):
        return 0
    return 3 if type(nxt2) is nn.Dropout and _no_hooks(nxt2) else 2


def _fuse_relu(block, nxt, X) -> bool:
    """Graph_conv_layer followed by nn.ReLU (GCN/GCN.py:12-13) at inference, no hooks on
    either module: the pair runs as one layer with the ReLU epilogue."""
    return (isinstance(block, Graph_conv_layer) and type(nxt) is nn.ReLU and isinstance(X, torch.Tensor)
            and X.is_cuda and not torch.is_grad_enabled()
            and not (block._forward_hooks or block._forward_pre_hooks or nxt._forward_hooks
                     or nxt._forward_pre_hooks))


class Graph_conv_layer(nn.Module):
    """GCN/GCN.py:30-52: support = X W^T ; out = A_hat support + bias (one HIP launch)."""

    def __init__(self, in_features, out_features, is_bias=True, **kwargs):
        super().__init__(**kwargs)
        self.in_features = in_features
        self.out_features = out_features
        self.dense = nn.Linear(in_features, out_features, bias=False)
        if is_bias:
            self.bias = nn.Parameter(torch.zeros(out_features))
        else:
            self.register_parameter('bias', None)

    def forward(self, X_input, adj):
        return self._forward(X_input, adj, None)

    def _forward(self, X_input, adj, activation):
        """forward, with ``activation`` ('relu' or None) in the SpMM's epilogue at inference."""
        g = as_csr(adj)
        support = None
        training = torch.is_grad_enabled() and (
            X_input.requires_grad or self.dense.weight.requires_grad
            or (self.bias is not None and self.bias.requires_grad))
        if X_input.is_cuda and training and X_input.dtype == torch.float32 \
                and X_input.shape[0] == g.n_cols:
            # one differentiable op: MFMA transform + SpMM forward, SpMM + MFMA transform +
            # dW GEMM backward (ops._GcnLayerFn)
            y = gcn_layer(g, X_input, self.dense.weight, self.bias)
            return F.relu(y) if activation == 'relu' else y
        if X_input.is_cuda and not training:
            order = column_order(g, self.out_features)
            if order is not None and X_input.shape[0] == g.n_cols:
                # support rows in the column-degree order of A P^T: the SpMM then reads its hub
                # rows in place; A P^T (P X W^T) = A X W^T, rows in the original order
                support = gcn_transform(X_input, self.dense.weight, out_rows=order.inv,
                                        check_rows=False)
                if support is not None:
                    return spmm_forward(order.graph, support, self.bias, activation=activation)
            support = gcn_transform(X_input, self.dense.weight)  # MFMA kernel (inference)
            if support is not None:
                return spmm_forward(g, support, self.bias, activation=activation)
        if support is None:
            support = self.dense(X_input)
        y = spmm(g, support, self.bias)
        return F.relu(y) if activation == 'relu' else y

    def __repr__(self):
        return self.__class__.__name__ + ' (' \
               + str(self.in_features) + ' -> ' \
               + str(self.out_features) + ')'
