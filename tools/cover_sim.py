"""Exchanged-row statistics of the edge-cut exchanges (feature rows only vs cover) on the
weak-scaling RMAT graphs, by running the real partition builders for all ranks in one
process (threads stand in for ranks; the all-to-all-v is an in-memory exchange).

    python tools/cover_sim.py 2 4 8      (CPU only; ~2 min for 8 ranks)
"""
import sys, threading, time, numpy as np, torch
sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parent.parent))
import graphneuralnetwork_amd.distributed as D
from graphneuralnetwork_amd.rmat import rmat_edges
from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
torch.set_num_threads(1)
class Sim:
    def __init__(self, W):
        self.W = W; self.bar = threading.Barrier(W); self.box = {}
    def a2a(self, out, inp, out_splits, in_splits, group=None):
        r = threading.current_thread().rank
        offs = np.concatenate([[0], np.cumsum(in_splits)])
        self.box[r] = [inp[offs[k]:offs[k+1]] for k in range(self.W)]
        self.bar.wait()
        parts = [self.box[k][r] for k in range(self.W)]
        torch.cat(parts, out=out) if out.numel() else None
        self.bar.wait()
for W in [int(a) for a in sys.argv[1:]]:
    n, e = 1_000_000 * W, 10_000_000 * W
    s, d = rmat_edges(n, e, 0); g = gcn_normalized_csr(s, d, n); del s, d
    sim = Sim(W); D._all_to_all_v = sim.a2a
    bounds = D.nnz_balanced_bounds(g.rowptr, W)
    res = {}
    def run(r):
        threading.current_thread().rank = r
        for kind in ("gather", "cover"):
            t = time.time()
            p = D.build_partition(g, r, W, bounds=bounds) if kind == "gather" else D.build_cover_exchange(g, r, W, bounds=bounds)
            res[(kind, r)] = (p.n_halo, sum(p.send_counts), p.nnz if kind == "gather" else (p.interior.nnz, p.send_p.nnz, p.halo_x.nnz + p.halo_p.nnz), time.time() - t)
    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    [t.start() for t in th]; [t.join() for t in th]
    for kind in ("gather", "cover"):
        rv = [res[(kind, r)] for r in range(W)]
        print(f"W={W} {kind}: recv rows {[x[0] for x in rv]} max {max(x[0] for x in rv)}; send max {max(x[1] for x in rv)}; work {[x[2] for x in rv]}; build s {max(x[3] for x in rv):.1f}", flush=True)
