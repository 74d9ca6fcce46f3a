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


def _rmat_chunk(seed: int, n_edges: int, scale: int, e0: int, e1: int, src, dst) -> None:
    """Edges [e0, e1) of the stream: for bit b the u draws are outputs b*2E + e (0 <= e < E)
    of the seeded PCG64 stream and the v draws b*2E + E + e (Generator.random takes one
    64-bit output per double), so every chunk starts from its own advanced copy of the
    generator and the result equals one sequential pass bit for bit."""
    p_row1 = D / (C + D)
    p_row0 = B / (A + B)
    m = e1 - e0
    s = np.zeros(m, np.int64)
    d = np.zeros(m, np.int64)
    for bit in range(scale):
        bu = np.random.PCG64(seed)
        bu.advance(bit * 2 * n_edges + e0)
        u = np.random.Generator(bu).random(m)
        bv = np.random.PCG64(seed)
        bv.advance(bit * 2 * n_edges + n_edges + e0)
        v = np.random.Generator(bv).random(m)
        rb = u > A + B
        cb = np.where(rb, v < p_row1, v < p_row0)
        s |= rb.astype(np.int64) << bit
        d |= cb.astype(np.int64) << bit
    src[e0:e1] = s
    dst[e0:e1] = d


def rmat_edges(n_nodes: int, n_edges: int, seed: int = 0, chunk: int = 1 << 22,
               threads: int | None = None):
    """Directed R-MAT edge list (src, dst) as int64 numpy arrays.

    The stream is the one of ``np.random.default_rng(seed)`` drawn u then v per bit over
    all edges; chunks of ``chunk`` edges are generated on a thread pool (numpy fills
    releases the GIL) from advanced generator copies, with the same result."""
    scale = max(1, math.ceil(math.log2(max(2, n_nodes))))
    src = np.zeros(n_edges, np.int64)
    dst = np.zeros(n_edges, np.int64)
    bounds = list(range(0, n_edges, chunk)) + [n_edges]
    jobs = [(bounds[i], bounds[i + 1]) for i in range(len(bounds) - 1)]
    if threads is None:
        import os
        threads = min(16, len(os.sched_getaffinity(0)))
    if len(jobs) <= 1 or threads <= 1:
        for e0, e1 in jobs:
            _rmat_chunk(seed, n_edges, scale, e0, e1, src, dst)
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda j: _rmat_chunk(seed, n_edges, scale, j[0], j[1], src, dst), jobs))
    if n_nodes != (1 << scale):
        src %= n_nodes
        dst %= n_nodes
    return src, dst


def permute_ids(src, dst, n_nodes: int, seed: int = 1):
    """Optional seeded relabelling (leaves nnz unchanged)."""
    perm = np.random.default_rng(seed).permutation(n_nodes)
    return perm[src], perm[dst]
