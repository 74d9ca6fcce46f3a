"""Per-rank compute phases of the edge-cut SpMM at world size W, measured on ONE GPU.

    python tools/rank_sim.py [W=8] [--feat 128] [--exchange cover|gather]

Builds the weak-scaling graph (W x the 1M / 10M R-MAT, as bench.py --gpus W), runs the
real partition builders for every rank in one process (threads stand in for ranks; the
all-to-all-v is an in-memory copy on the device), then times each rank's kernels with
the exchange removed: the send-side work, the interior SpMM and the halo SpMMs, plus
the bytes each rank sends and receives per aggregation. The exchange itself (RCCL over
xGMI) is not modelled here -- only what runs around it.
"""
import argparse
import json
import statistics
import sys
import threading
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


class _Sim:
    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.box = {}

    def a2a(self, out, inp, out_splits, in_splits, group=None):
        r = threading.current_thread().rank
        offs = [0]
        for v in in_splits:
            offs.append(offs[-1] + int(v))
        self.box[r] = [inp[offs[k]:offs[k + 1]] for k in range(self.world)]
        self.bar.wait()
        parts = [self.box[k][r] for k in range(self.world)]
        if out.numel():
            torch.cat(parts, out=out)
        self.bar.wait()

    def all_gather_floats(self, v, world, device, group=None):
        r = threading.current_thread().rank
        self.box[r] = list(v)
        self.bar.wait()
        out = torch.tensor([self.box[k] for k in range(self.world)], dtype=torch.float64)
        self.bar.wait()
        return out

    def global_sum(self, v, device, group=None):
        r = threading.current_thread().rank
        self.box[r] = int(v)
        self.bar.wait()
        tot = sum(self.box[k] for k in range(self.world))
        self.bar.wait()
        return tot


def _time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("world", nargs="?", type=int, default=8)
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--exchange", default="cover", choices=["cover", "gather", "balanced"])
    ap.add_argument("--chunks", type=int, default=1,
                    help="time the halo_x pass split into this many column chunks "
                         "(EdgeCutSpmm chunks=, the chunked feature-row exchange)")
    ap.add_argument("--strong", action="store_true",
                    help="cfg5: the fixed 10M / 100M graph cut W ways (default: W x 1M / 10M)")
    args = ap.parse_args()
    import graphneuralnetwork_amd.distributed as D
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gather_rows, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    _lib.load()
    dev = torch.device("cuda:0")
    W, F = args.world, args.feat
    nodes, edges = (10_000_000, 100_000_000) if args.strong else (1_000_000 * W, 10_000_000 * W)
    s, d = rmat_edges(nodes, edges, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), nodes, device=dev)
    del s, d
    sim = _Sim(W)
    D._all_to_all_v = sim.a2a
    D._global_sum = sim.global_sum
    D._all_gather_floats = sim.all_gather_floats
    bounds = D.nnz_balanced_bounds(g.rowptr, W)
    parts = {}

    def build(r):
        threading.current_thread().rank = r
        if args.exchange == "balanced":
            parts[r], hist = D.build_cover_exchange_balanced(g, r, W)
            if r == 0:
                print(json.dumps({"balance_history_max_mean": hist,
                                  "bounds": parts[r].bounds}), flush=True)
        else:
            parts[r] = (D.build_cover_exchange(g, r, W, bounds=bounds) if args.exchange == "cover"
                        else D.build_partition(g, r, W, bounds=bounds))
        torch.cuda.synchronize()

    th = [threading.Thread(target=build, args=(r,)) for r in range(W)]
    [t.start() for t in th]
    [t.join() for t in th]
    print(json.dumps({"world": W, "feat": F, "nnz": g.nnz, "exchange": args.exchange,
                      "halo_chunks": args.chunks}), flush=True)
    rows = []
    for r in range(W):
        p = parts[r]
        x = torch.randn(p.n_own, F, device=dev)
        out = torch.empty(p.n_own, F, device=dev)
        ph = {}
        if args.exchange != "gather":
            sx = torch.empty(sum(p.send_x_counts), F, device=dev)
            sp = torch.empty(sum(p.send_p_counts), F, device=dev)
            rx = torch.randn(sum(p.recv_x_counts), F, device=dev)
            rp = torch.randn(sum(p.recv_p_counts), F, device=dev)
            if sx.shape[0]:
                ph["gather_send_x"] = _time(lambda: gather_rows(x, p.send_x_idx, out=sx,
                                                                check=False))
            if sp.shape[0]:
                ph["spmm_send_p"] = _time(lambda: spmm_forward(p.send_p, x, None, out=sp))
            ph["spmm_interior"] = _time(lambda: spmm_forward(p.interior, x, None, out=out))
            if rx.shape[0] and args.chunks > 1:
                hx = D.split_halo_chunks(p.halo_x, p.recv_x_counts, args.chunks)
                offs = [0]
                for gk in hx:
                    offs.append(offs[-1] + gk.n_cols)

                def halo_chunks():
                    for k, gk in enumerate(hx):
                        if gk.nnz:
                            spmm_forward(gk, rx[offs[k]:offs[k + 1]], None, out=out,
                                         accumulate=True)
                ph["spmm_halo_x"] = _time(halo_chunks)
            elif rx.shape[0]:
                ph["spmm_halo_x"] = _time(lambda: spmm_forward(p.halo_x, rx, None, out=out,
                                                               accumulate=True))
            if rp.shape[0]:
                ph["spmm_halo_p"] = _time(lambda: spmm_forward(p.halo_p, rp, None, out=out,
                                                               accumulate=True))
            send_rows = sx.shape[0] + sp.shape[0]
            recv_rows = rx.shape[0] + rp.shape[0]
            work = {"interior": p.interior.nnz, "send_p": p.send_p.nnz,
                    "halo_x": p.halo_x.nnz, "halo_p": p.halo_p.nnz}
        else:
            sb = torch.empty(sum(p.send_counts), F, device=dev)
            rb = torch.randn(p.n_halo, F, device=dev)
            if sb.shape[0]:
                ph["gather_send"] = _time(lambda: gather_rows(x, p.send_idx, out=sb, check=False))
            ph["spmm_interior"] = _time(lambda: spmm_forward(p.interior, x, None, out=out))
            ph["spmm_halo"] = _time(lambda: spmm_forward(p.halo, rb, None, out=out,
                                                         accumulate=True))
            send_rows, recv_rows = sb.shape[0], rb.shape[0]
            work = {"interior": p.interior.nnz, "halo": p.halo.nnz}
        rows.append({"rank": r, "own_rows": p.n_own, "phases_ms": ph,
                     **({"model_cost": D.cover_cost(p)} if args.exchange != "gather" else {}),
                     "compute_ms": sum(ph.values()), "send_MB": send_rows * 4 * F / 1e6,
                     "recv_MB": recv_rows * 4 * F / 1e6, "nnz": work})
        print(json.dumps(rows[-1]), flush=True)
        del x, out
        torch.cuda.empty_cache()
    print(json.dumps({"max_compute_ms": max(r["compute_ms"] for r in rows),
                      "mean_compute_ms": statistics.mean(r["compute_ms"] for r in rows),
                      "max_send_MB": max(r["send_MB"] for r in rows),
                      "max_recv_MB": max(r["recv_MB"] for r in rows)}), flush=True)


if __name__ == "__main__":
    main()
