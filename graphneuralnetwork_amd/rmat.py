"""Synthetic power-law graphs (Graph500 R-MAT) for benchmarks and scale tests.

Recipe: a=0.57, b=0.19, c=0.19, d=0.05,
scale = ceil(log2 N); for every bit, LSB first, draw u then v from
``np.random.default_rng(seed)``: the row bit is ``u > a + b``; the column bit
is ``v < d/(c+d)`` when the row bit is set, else ``v < b/(a+b)``.  Node ids
are taken mod N.  With N = 2^20 nodes / 10M edges this yields, after the
reference GCN pipeline (symmetrise, +I, normalise), nnz = 20,073,500.
"""
from __future__ import annotations

import math

import numpy as np

A, B, C, D = 0.57, 0.19, 0.19, 0.05


def rmat_edges(n_nodes: int, n_edges: int, seed: int = 0, chunk: int = 1 << 24):
    """Directed R-MAT edge list (src, dst) as int64 numpy arrays."""
    scale = max(1, math.ceil(math.log2(max(2, n_nodes))))
    rng = np.random.default_rng(seed)
    src = np.zeros(n_edges, np.int64)
    dst = np.zeros(n_edges, np.int64)
    p_row1 = D / (C + D)
    p_row0 = B / (A + B)
    for bit in range(scale):
        u = rng.random(n_edges)
        v = rng.random(n_edges)
        rb = u > A + B
        cb = np.where(rb, v < p_row1, v < p_row0)
        src |= rb.astype(np.int64) << bit
        dst |= cb.astype(np.int64) << bit
        del u, v, rb, cb
    if n_nodes != (1 << scale):
        src %= n_nodes
        dst %= n_nodes
    return src, dst


def permute_ids(src, dst, n_nodes: int, seed: int = 1):
    """Optional seeded relabelling (leaves nnz unchanged)."""
    perm = np.random.default_rng(seed).permutation(n_nodes)
    return perm[src], perm[dst]
