"""Runs the cfg4 GraphSAGE forward (degree-ordered dataset, 8192 seeds, [25, 10]) REPS times
after warm-up, for a rocprofv3 --kernel-trace of its kernels; ``--batch``: whole batches
instead (sample_batch(..., sync=False) + the forward, no host read inside a batch):

    rocprofv3 --kernel-trace -d gpurun_out/sage_trace -o run --output-format csv -- python3 tools/sage_forward_trace.py [--batch]
    python3 tools/sage_forward_trace.py --summarize gpurun_out/sage_trace/.../run_kernel_trace.csv
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main(batch: bool = False):
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import degree_ordered, sample_batch, symmetric_adjacency
    dev = torch.device("cuda:0")
    n, F = 10_000_000, 128
    s, d = rmat_edges(n, 100_000_000, 0)
    adj, _, _ = degree_ordered(symmetric_adjacency(s, d, n, device=dev))
    del s, d
    gen = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(n, F, device=dev, generator=gen)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    cand = torch.nonzero(deg > 0).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    b = sample_batch(adj, seeds, (25, 10), seed=0)
    net = GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    fa = b.forward_args(table)
    import time
    if batch:
        def one():
            p = sample_batch(adj, seeds, (25, 10), seed=0, sync=False)
            net(*p.forward_args(table), None, None, None, None, None)
            return p
    else:
        def one():
            return net(*fa, None, None, None, None, None)
    with torch.no_grad():
        for _ in range(10):
            one()
        torch.cuda.synchronize()
        # host enqueue time per forward (no sync inside) vs the wall time until the GPU is done:
        # equal = the eager forward is paced by the host, not by its kernels
        t0 = time.perf_counter()
        kept = [one() for _ in range(50)]
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for p in kept if batch else ():
            p.check()
    what = "batch" if batch else "forward"
    print(f"done frontier {b.frontier.numel()}: host enqueue {(t1 - t0) / 50 * 1e6:.1f} us per "
          f"{what}, wall {(t2 - t0) / 50 * 1e6:.1f} us per {what}", flush=True)


def summarize(csv_path: str, per: int = 0, last: int = 50) -> None:
    """Median duration per kernel position of the last ``last`` forwards (``per`` kernels each,
    default: inferred from the repeating kernel-name cycle) and the median gap before it."""
    import csv
    import statistics
    rows = sorted((r for r in csv.DictReader(open(csv_path))
                   if not r["Kernel_Name"].startswith("__amd_rocclr")),  # the checks' readbacks
                  key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    if not per:
        for p in range(1, 20):
            if names[-p:] == names[-2 * p:-p] and names[-p:] == names[-3 * p:-2 * p]:
                per = p
                break
    tail = rows[-per * last:]
    print(f"{per} kernels per forward, last {last} forwards")
    tot = 0.0
    for i in range(per):
        ks = tail[i::per]
        d = statistics.median((int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3 for k in ks)
        prev = [tail[(i - 1) % per + per * j] if i else (tail[per * j - 1] if j else None)
                for j in range(last)]
        g = statistics.median((int(k["Start_Timestamp"]) - int(pv["End_Timestamp"])) / 1e3
                              for k, pv in zip(ks, prev) if pv is not None)
        tot += d
        print(f"  {d:7.1f} us (gap {g:5.1f})  {ks[0]['Kernel_Name'][:110]}")
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3 / last
    print(f"sum of kernels {tot:.1f} us per forward; first start to last end {span:.1f} us per forward")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        main(batch="--batch" in sys.argv)
