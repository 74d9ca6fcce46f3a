"""CPython-exact GraphSAGE sampler: native (csrc/pysample.cpp) vs the reference algorithm.

Builds the 1M-node / 10M-pair R-MAT adjacency both ways (native restatement of
read_pubmed_data's set construction vs real Python sets), checks the neighbour orders
are identical, then times get_layer_adj_nodes (2 layers, k=10) natively against the
oracle restatement that runs the reference algorithm on CPython sets / random, and
checks maps and generator state are identical.  Host only (no GPU).

    python tools/pysampler_bench.py
"""
import sys, time, random
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import numpy as np
from collections import defaultdict
from graphneuralnetwork_amd.rmat import rmat_edges
from graphneuralnetwork_amd.pysampler import PyAdjacency, get_layer_adj_nodes
from oracle import gnn_oracle as O
n = 1_000_000
s, d = rmat_edges(n, 10_000_000, 0)
pa = PyAdjacency.from_pairs(s, d, n)
t = time.perf_counter()
adj = defaultdict(set)
for a, b in zip(s.tolist(), d.tolist()):
    adj[a].add(b); adj[b].add(a)
print("python adj build", time.perf_counter() - t, flush=True)
t = time.perf_counter(); pb = PyAdjacency.from_adj_lists(adj, n); print("read python sets", time.perf_counter()-t)
print("adjacency order identical:", np.array_equal(pa.nbr, pb.nbr), np.array_equal(pa.rowptr, pb.rowptr), flush=True)
deg = np.diff(pa.rowptr); cand = np.flatnonzero(deg > 0)
rs = np.random.default_rng(0)
for B in (128, 512, 2048):
    nodes = rs.choice(cand, B, replace=False).tolist()
    r = random.Random(1)
    t = time.perf_counter(); nm, cm = get_layer_adj_nodes(nodes, pa, 2, 10, False, rng=r); tn = time.perf_counter() - t
    r0 = random.Random(1)
    t = time.perf_counter(); ref = O.sage_layer_adj_nodes(nodes, adj, 2, 10, False, r0); to = time.perf_counter() - t
    print(f"B={B}: native {tn*1e3:.1f} ms, reference algorithm {to*1e3:.0f} ms, maps {tuple(nm.shape)}, equal:",
          np.array_equal(np.asarray(ref[0]), nm.numpy()) and np.array_equal(np.asarray(ref[1]), cm.numpy()) and r.getstate()==r0.getstate(), flush=True)
nodes = rs.choice(cand, 8192, replace=False).tolist()
t = time.perf_counter(); nm, cm = get_layer_adj_nodes(nodes, pa, 2, 10, False, rng=random.Random(2)); print(f"native B=8192: {(time.perf_counter()-t)*1e3:.1f} ms {tuple(nm.shape)}")
