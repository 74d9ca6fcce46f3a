"""Would a locality partition cut the edge-cut exchange? Balanced label propagation
(nodes move to the part most of their neighbours are in, capacity 1.03x mean cost) against
the contiguous nnz-balanced blocks, on the weak-scaling RMAT graph of W ranks. Prints, per
iteration: (max rows a part receives, total distinct (part, remote column) pairs, total
distinct (remote part, row) pairs, cut-edge fraction, max/mean cost).

    python tools/lp_partition_probe.py W [iterations]      (CPU only)
"""
import sys, time, numpy as np, torch
sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parent.parent))
from graphneuralnetwork_amd.rmat import rmat_edges
from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
import graphneuralnetwork_amd.distributed as D
W = int(sys.argv[1]); n, e = 1_000_000 * W, 10_000_000 * W
t=time.time(); s, d = rmat_edges(n, e, 0); g = gcn_normalized_csr(s, d, n); del s, d
rp = g.rowptr.numpy(); col = g.col.numpy().astype(np.int64)
row = np.repeat(np.arange(n), np.diff(rp)); print("graph", time.time()-t, g.nnz, flush=True)
deg = np.diff(rp)
def volume(part):
    # gather volume: distinct (part[row], col) with part[col] != part[row]
    pr = part[row]; pc = part[col]; m = pr != pc
    key = np.unique(pr[m] * n + col[m])
    per = np.bincount(key // n, minlength=W)
    # partial-sum alt: distinct (part[col], row) pairs
    key2 = np.unique(pc[m] * n + row[m]); per2 = np.bincount(key2 // n, minlength=W)
    cost = np.bincount(part, weights=deg + 1, minlength=W)
    return per.max(), per.sum(), per2.sum(), m.mean(), cost.max() / cost.mean()
bounds = D.nnz_balanced_bounds(g.rowptr, W)
part0 = np.zeros(n, np.int64)
for r in range(W): part0[bounds[r]:bounds[r+1]] = r
print("contiguous", volume(part0), flush=True)
rng = np.random.default_rng(0)
part = part0.copy()
w = (deg + 1).astype(np.float64); cap = w.sum() / W * 1.03
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 8):
    cnt = np.bincount(row * W + part[col], minlength=n * W).reshape(n, W).astype(np.float64)
    load = np.bincount(part, weights=w, minlength=W)
    cur = cnt[np.arange(n), part]
    best = cnt.argmax(1); gain = cnt.max(1) - cur
    cand = np.nonzero((gain > 0) & (best != part))[0]
    cand = cand[rng.random(cand.size) < 0.5]
    # capacity: admit moves into each target until it would exceed cap (highest gain first)
    order = cand[np.argsort(-gain[cand], kind='stable')]
    moved = 0
    out = np.bincount(part[order], weights=w[order], minlength=W)
    for p in range(W):
        sel = order[best[order] == p]
        room = cap - load[p] + 0  # ignore outflow for safety
        cs = np.cumsum(w[sel]); ok = sel[cs <= max(room, 0) + 0]
        part[ok] = p; moved += ok.size
    print(it, "moved", moved, volume(part), flush=True)
