"""Does the SpMM's streaming traffic evict the hub rows from the Infinity Cache (MALL)?

The north-star step streams ~5 GB of output rows and ~1 GB of CSR through the memory side while
it gathers a 128 MiB hub table; a table stays MALL-resident only while everything touched
between two of its uses fits ~256 MiB (MI355X_MICROARCH.md "Infinity Cache"). This probe
allocates the output Y (and optionally the pass-2 CSR arrays) with hipExtMallocWithFlags
(uncached / fine-grained) so that those streams cannot allocate in the caches, and times the
same XCD-sliced SpMM (same graph, same X) against the default allocation, in one process.

    python tools/mall_probe.py [--workload ns|cfg2] [--reps 20]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

FLAGS = {"default": 0x0, "finegrained": 0x1, "uncached": 0x3}


class _Raw:
    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def hip_alloc(hip, nbytes, flag):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flag))
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags({flag}) failed: {rc}")
    return p.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ns", choices=["ns", "cfg2"])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    n, m = (10_000_000, 100_000_000) if a.workload == "ns" else (1_000_000, 10_000_000)
    F = 128
    s, d = rmat_edges(n, m, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    ga = column_order(g, F).graph
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, F, device=dev, generator=gen)
    b = torch.randn(F, device=dev, generator=gen)
    ref = spmm_forward(ga, X, b)
    torch.cuda.synchronize()
    outs = {}
    for name, flag in FLAGS.items():
        if flag == 0:
            outs[name] = torch.empty(n, F, device=dev)
        else:
            p = hip_alloc(hip, n * F * 4, flag)
            outs[name] = torch.as_tensor(_Raw(p, (n, F), "<f4"), device=dev)
    res = {}
    for rnd in range(3):  # interleaved rounds
        for name, Y in outs.items():
            spmm_forward(ga, X, b, out=Y)
            torch.cuda.synchronize()
            if rnd == 0:
                assert torch.equal(Y, ref), name
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record()
                spmm_forward(ga, X, b, out=Y)
                e1.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).extend(e0.elapsed_time(e1) for e0, e1 in ev)
    print(json.dumps({"workload": a.workload, "Y_alloc_ms": {k: round(statistics.median(v), 4)
                                                            for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
