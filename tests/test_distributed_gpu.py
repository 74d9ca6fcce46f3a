"""Edge-cut aggregation with the HIP kernels: 2 ranks sharing cuda:0, gloo exchange
(host-staged). Checks the pack kernel, interior SpMM and accumulating halo SpMM
against the single-GPU aggregation. (RCCL itself runs in bench.py --gpus N.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _collect(procs, q, n, timeout=600):
    """Results from n workers; fails fast when a worker dies instead of waiting for the timeout."""
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < n:
        try:
            out.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > timeout:
                for p in procs:
                    p.kill()
                raise AssertionError(f"worker failed (exit codes {dead}) or timed out")
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph(n, dev):
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(n, 10 * n, 5)
    return gcn_normalized_csr(s, d, n, device=dev)


def _worker(rank, world, port, n, F, q, kind="gather"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import (EdgeCutSpmm, build_cover_exchange,
                                                        build_cover_exchange_balanced,
                                                        build_partition)
        dev = torch.device("cuda:0")
        g = _graph(n, dev)
        if kind.endswith("_xcd"):  # every sub-SpMM through the XCD-sliced hub staging
            from graphneuralnetwork_amd import ops
            ops.XCD_MIN_NNZ, ops.HUB_MIN_X_BYTES, ops.XCD_MIN_DEG, ops.XCD_CHUNK = 1, 0, 8, 16
            kind = kind[:-4]
        if kind == "balanced":  # what bench.py --gpus N uses
            part, _ = build_cover_exchange_balanced(g, rank, world)
        else:
            build = build_cover_exchange if kind == "cover" else build_partition
            part = build(g, rank, world)
        X = torch.from_numpy(np.random.default_rng(1).standard_normal((n, F)).astype(np.float32)).to(dev)
        b = torch.linspace(-1, 1, F, device=dev)
        r0, r1 = part.bounds[rank], part.bounds[rank + 1]
        run = EdgeCutSpmm(part, F, dev)
        y = run(X[r0:r1].contiguous(), b, activation="relu")
        prof = run.profile(X[r0:r1].contiguous(), b, activation="relu")  # bench.py's breakdown
        assert prof["total_ms"] > 0 and prof["spmm_interior_ms"] >= 0
        assert any(k.startswith("a2a") for k in prof) and any(k.startswith("wait") for k in prof)
        y = run(X[r0:r1].contiguous(), b, activation="relu")  # later calls reuse buffers
        torch.cuda.synchronize()
        q.put((rank, r0, r1, y.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "gather"), (2, "cover"), (3, "cover"),
                                        (2, "balanced"), (3, "balanced_xcd")])
def test_edge_cut_hip_path_matches_single_gpu(dev, world, kind):
    from graphneuralnetwork_amd.ops import spmm_forward
    n, F = 20000, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, F, q, kind))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(_collect(procs, q, world), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = _graph(n, dev)
    X = torch.from_numpy(np.random.default_rng(1).standard_normal((n, F)).astype(np.float32)).to(dev)
    ref = spmm_forward(g, X, torch.linspace(-1, 1, F, device=dev), activation="relu",
                       hubs=0).cpu().numpy()
    for rank, r0, r1, y in res:
        np.testing.assert_allclose(y, ref[r0:r1], rtol=1e-5, atol=1e-5)


def _gat_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import EdgeCutGat, build_partition
        dev = torch.device("cuda:0")
        g = _graph(n, dev)
        part = build_partition(g, rank, world)
        gen = torch.Generator().manual_seed(0)
        Wh = (torch.randn(n, 64, generator=gen) * 0.5).to(dev)
        a_s = (torch.randn(64, generator=gen) * 0.3).to(dev)
        a_d = (torch.randn(64, generator=gen) * 0.3).to(dev)
        r0, r1 = part.bounds[rank], part.bounds[rank + 1]
        layer = EdgeCutGat(part, 8, 8, dev)
        assert layer._staged is not None  # received rows read in place (gat_aggregate_staged)
        y = layer(Wh[r0:r1].contiguous(), a_s, a_d, 0.2, 0, "elu")
        torch.cuda.synchronize()
        q.put((rank, r0, r1, y.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_gat_edge_cut_hip_path_matches_single_gpu(dev):
    from graphneuralnetwork_amd.ops import GAT_DENSE, gat_aggregate, gat_logits
    n, world = 20000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gat_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(_collect(procs, q, world), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = _graph(n, dev)
    gen = torch.Generator().manual_seed(0)
    Wh = (torch.randn(n, 64, generator=gen) * 0.5).to(dev)
    a_s = (torch.randn(64, generator=gen) * 0.3).to(dev)
    a_d = (torch.randn(64, generator=gen) * 0.3).to(dev)
    el, er = gat_logits(Wh, 8, 8, a_s, a_d)
    ref = gat_aggregate(g, Wh, el, er, 8, 8, 0.2, GAT_DENSE, "elu").cpu().numpy()
    for rank, r0, r1, y in res:
        np.testing.assert_allclose(y, ref[r0:r1], rtol=1e-5, atol=1e-5)


def _sage_setup(dev):
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import symmetric_adjacency
    n, F = 20000, 64
    s, d = rmat_edges(n, 10 * n, 9)
    adj = symmetric_adjacency(s, d, n, device=dev)
    gen = torch.Generator().manual_seed(3)
    table = torch.randn(n, F, generator=gen).to(dev)
    torch.manual_seed(4)
    net = GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False, class_size=5)
    net = net.to(dev).eval()
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu()
    seeds = torch.nonzero(deg > 0).view(-1)[:1001].to(dev)
    return net, adj, table, seeds


def _sage_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import sage_forward_sharded
        dev = torch.device("cuda:0")
        net, adj, table, seeds = _sage_setup(dev)
        with torch.no_grad():
            emb, logits = sage_forward_sharded(net, adj, table, seeds, rank, world, seed=7,
                                               gather=True)
        torch.cuda.synchronize()
        q.put((rank, emb.cpu().numpy(), logits.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_sage_sharded_forward_matches_per_shard_runs(dev):
    """GraphSAGE data parallelism: 2 ranks on cuda:0 each sample their seed
    shard and run the drop-in forward; every rank ends with all shards' embeddings and
    logits in seed order, bit-identical to running each shard's batch in one process."""
    from graphneuralnetwork_amd.distributed import rank_sample_seed, shard_seeds
    from graphneuralnetwork_amd.sampler import sample_batch
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sage_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(_collect(procs, q, world), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    net, adj, table, seeds = _sage_setup(dev)
    embs, logs = [], []
    with torch.no_grad():
        for r in range(world):
            b = sample_batch(adj, shard_seeds(seeds, r, world), (25, 10),
                             seed=rank_sample_seed(7, r))
            e, lg = net(*b.forward_args(table), None, None, None, None, None)
            embs.append(e.cpu().numpy())
            logs.append(lg.cpu().numpy())
    emb_ref, log_ref = np.concatenate(embs), np.concatenate(logs)
    assert emb_ref.shape[0] == seeds.numel()
    for _, emb, logits in res:
        np.testing.assert_array_equal(emb, emb_ref)
        np.testing.assert_array_equal(logits, log_ref)


def _run_ranks(world, fn):
    """fn(rank) on `world` threads of this process (distributed.LocalGroup ranks)."""
    import threading
    errs = []

    def main(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)
            _run_ranks.comm._bar.abort()

    th = [threading.Thread(target=main, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    if errs:
        raise errs[0]


@pytest.mark.timeout(900)
def test_cfg5_eight_ranks_full_size():
    """BASELINE configs[4] rehearsed on one GPU: the 8 cover-exchange partitions of the full
    10M / 207M-entry graph (build_cover_exchange_balanced, three builds with the cost re-cut,
    what bench.py --gpus 8 --workload cfg5 runs on every rank), each rank's EdgeCutSpmm at
    F = 256 with the RCCL all-to-all-v replaced by device copies between the ranks' buffers
    (distributed.LocalGroup: the 8 ranks are threads of this process). The concatenated
    output must equal the single-GPU aggregation: row samples (every hub row included)
    against the single-GPU kernel and the C oracle, plus the all-row checksum
    1^T (A X + 1 b^T) v = (1^T A)(X v) + n (b . v). Per-rank setup times are printed."""
    import time
    from graphneuralnetwork_amd import distributed as D
    from graphneuralnetwork_amd.ops import spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    from oracle import c_oracle
    dev = torch.device("cuda:0")
    W, F, n = 8, 256, 10_000_000
    t0 = time.perf_counter()
    s, d = rmat_edges(n, 100_000_000, 0)
    t_edges = time.perf_counter() - t0
    t0 = time.perf_counter()
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    torch.cuda.synchronize()
    t_adj = time.perf_counter() - t0
    del s, d
    assert g.nnz == 206_948_698
    comm = D.LocalGroup(W)
    _run_ranks.comm = comm
    parts, setup = [None] * W, [dict() for _ in range(W)]

    def build(r):
        comm.bind(r)
        t = time.perf_counter()
        parts[r], hist = D.build_cover_exchange_balanced(
            g, r, W, group=comm,
            progress=lambda it, mx, mean, sec: setup[r].__setitem__(f"build{it}_s", round(sec, 2)))
        torch.cuda.synchronize()
        setup[r]["cover_total_s"] = round(time.perf_counter() - t, 2)
        setup[r]["max_mean_cost"] = [round(a / b, 3) for a, b in hist]
        print(f"  rank {r} partition built in {setup[r]['cover_total_s']}s", flush=True)

    t0 = time.perf_counter()
    _run_ranks(W, build)
    t_parts = time.perf_counter() - t0
    bounds = parts[0].bounds
    assert all(p.bounds == bounds for p in parts) and bounds[0] == 0 and bounds[-1] == n
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, F, device=dev, generator=gen)
    b = torch.randn(F, device=dev, generator=gen)
    Y = torch.empty(n, F, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(W)]

    def step(r):
        comm.bind(r)
        r0, r1 = bounds[r], bounds[r + 1]
        with torch.cuda.stream(streams[r]):
            run = D.EdgeCutSpmm(parts[r], F, dev, group=comm)
            x = X[r0:r1].contiguous()
            t = time.perf_counter()
            run(x, b)                     # the first call also builds every sub-SpMM's plans
            torch.cuda.synchronize()
            setup[r]["first_step_s"] = round(time.perf_counter() - t, 2)
            Y[r0:r1].copy_(run(x, b))
            torch.cuda.synchronize()

    _run_ranks(W, step)
    print(f"\ncfg5 8-rank rehearsal: rmat edges {t_edges:.1f}s, gcn_adjacency {t_adj:.2f}s, "
          f"8 x build_cover_exchange_balanced (concurrent threads) {t_parts:.1f}s")
    for r in range(W):
        p = parts[r]
        print(f"  rank {r}: rows {p.n_own} interior {p.interior.nnz} send_p {p.send_p.nnz} "
              f"halo_x {p.halo_x.nnz} halo_p {p.halo_p.nnz} send {sum(p.send_counts)} recv "
              f"{p.n_halo} rows; setup {setup[r]}")
    ref = spmm_forward(g, X, b)
    rowptr = g.rowptr.cpu().numpy()
    deg = np.diff(rowptr)
    rng = np.random.default_rng(4)
    rows = np.unique(np.concatenate([rng.choice(n, 1500, replace=False), np.argsort(-deg)[:32],
                                     np.array(bounds[1:-1]) - 1, np.array(bounds[:-1])]))
    ri = torch.from_numpy(rows).to(dev)
    got, want = Y[ri].cpu().numpy(), ref[ri].cpu().numpy()
    scale = float(np.abs(want).max())
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-5 * scale)
    col, val = g.col.cpu().numpy(), g.val.cpu().numpy()
    Xn = X.cpu().numpy()
    oracle = np.concatenate([c_oracle.spmm_csr(rowptr, col, val, Xn, b.cpu().numpy(), r, r + 1)
                             for r in rows[:400]])
    np.testing.assert_allclose(got[:400], oracle, rtol=1e-4, atol=1e-5 * scale)
    v = np.random.default_rng(2).standard_normal(F)
    lhs = float((Y.double() @ torch.from_numpy(v).to(dev)).sum())
    colsum = np.bincount(col, weights=val.astype(np.float64), minlength=n)
    xv = Xn.astype(np.float64) @ v
    rhs = float(colsum @ xv) + n * float(b.cpu().double().numpy() @ v)
    assert abs(lhs - rhs) <= 1e-4 * float(np.abs(colsum) @ np.abs(xv)), (lhs, rhs)


def _gat_graph(n, dev, self_loops):
    """R-MAT graph with unit values, with or without self-loops (without: rows whose every
    edge is remote, one-edge rows pointing at a halo slot, long hub rows)."""
    from graphneuralnetwork_amd.graph import from_coo
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(n, 12 * n, 11)
    s, d = torch.from_numpy(s), torch.from_numpy(d)
    keep = s != d
    s, d = s[keep], d[keep]
    key = torch.unique(torch.cat([s * n + d, d * n + s]))
    r, c = key // n, key % n
    if self_loops:
        r = torch.cat([r, torch.arange(n)])
        c = torch.cat([c, torch.arange(n)])
    else:  # every row needs an edge: isolated rows get one to node 0 (a remote hub)
        deg = torch.bincount(r, minlength=n)
        iso = torch.nonzero(deg == 0).view(-1)
        r = torch.cat([r, iso])
        c = torch.cat([c, torch.zeros_like(iso)])
    return from_coo(r.to(dev), c.to(dev), torch.ones(r.numel(), device=dev), n, n)


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("self_loops,heads,fh", [(True, 8, 8), (False, 8, 8), (False, 1, 64)])
def test_gat_edge_cut_overlapped_two_pass(dev, world, mode, self_loops, heads, fh):
    """EdgeCutGat on the HIP path (ranks as LocalGroup threads): the interior pass during the
    exchange + the halo pass with the interior result as a log-sum-exp pseudo-edge equals
    the single-GPU layer (dense and sparse semantics, ELU), with and without self-loops
    (rows without interior edges), and heads=1 x 64 (row stride 65 of the [Wh | er]
    buffer); and equals the blocking one-pass path."""
    from graphneuralnetwork_amd import distributed as D
    from graphneuralnetwork_amd.ops import gat_aggregate, gat_logits
    n = 6000
    g = _gat_graph(n, dev, self_loops)
    gen = torch.Generator().manual_seed(world + mode)
    F = heads * fh
    Wh = (torch.randn(n, F, generator=gen) * 0.5).to(dev)
    a_s = (torch.randn(F, generator=gen) * 0.3).to(dev)
    a_d = (torch.randn(F, generator=gen) * 0.3).to(dev)
    el, er = gat_logits(Wh, heads, fh, a_s, a_d)
    ref = gat_aggregate(g, Wh, el, er, heads, fh, 0.2, mode, "elu").cpu().numpy()
    comm = D.LocalGroup(world)
    _run_ranks.comm = comm
    outs = {}

    def rank_main(r):
        comm.bind(r)
        part = D.build_partition(g, r, world, group=comm)
        r0, r1 = part.bounds[r], part.bounds[r + 1]
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for overlap in (True, False):
                layer = D.EdgeCutGat(part, heads, fh, dev, group=comm, overlap=overlap)
                assert (layer._halo_pass is not None) == overlap
                y = layer(Wh[r0:r1].contiguous(), a_s, a_d, 0.2, mode, "elu")
                y2 = layer(Wh[r0:r1].contiguous(), a_s, a_d, 0.2, mode, "elu",
                           el=el[r0:r1], er=er[r0:r1])
                torch.cuda.synchronize()
                outs[(r, overlap)] = (r0, r1, y.cpu().numpy(), y2.cpu().numpy())

    _run_ranks(world, rank_main)
    for (r, overlap), (r0, r1, y, y2) in outs.items():
        np.testing.assert_allclose(y, ref[r0:r1], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(y2, y, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("heads,fh", [(8, 8), (1, 64), (2, 5)])
def test_gat_aggregate_staged_matches_concatenated(dev, mode, heads, fh):
    """gat_aggregate_staged over [own | staged-view] tables == gat_aggregate over
    the concatenated tables -- one-edge rows whose only edge is staged, long rows cut into
    segments, both modes, a (F + heads) % 4 != 0 row stride."""
    from graphneuralnetwork_amd.graph import CsrGraph, from_coo
    from graphneuralnetwork_amd.ops import gat_aggregate, gat_aggregate_staged
    rng = np.random.default_rng(heads * 10 + fh + mode)
    n, k = 3000, 700
    F = heads * fh
    rows = np.concatenate([rng.integers(0, n, 20000), np.arange(200), np.full(2500, 7)])
    cols = np.concatenate([rng.integers(0, n + k, 20000), n + rng.integers(0, k, 200),
                           rng.integers(0, n + k, 2500)])
    present = np.zeros(n, bool)
    present[rows] = True
    rows = np.concatenate([rows, np.flatnonzero(~present)])
    cols = np.concatenate([cols, np.full((~present).sum(), n)])
    gcat = from_coo(torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev),
                    torch.ones(rows.size, device=dev), n, n + k)
    buf = torch.randn(k, F + heads + 1, device=dev)[:, 1:]   # a strided [Wh | er] view
    wh = torch.randn(n, F, device=dev)
    er = torch.randn(n, heads, device=dev)
    el = torch.randn(n, heads, device=dev)
    whh, erh = buf[:, :F], buf[:, F:]
    ref = gat_aggregate(gcat, torch.cat([wh, whh]), el, torch.cat([er, erh]), heads, fh, 0.2,
                        mode, "elu")
    c = gcat.col.to(torch.int64)
    gst = CsrGraph(gcat.rowptr, torch.where(c < n, c, n - 1 - c).to(torch.int32).contiguous(),
                   gcat.val, n, n)
    got = gat_aggregate_staged(gst, wh, el, er, whh, erh, heads, fh, 0.2, mode, "elu")
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    with pytest.raises(TypeError):
        gat_aggregate_staged(gst, wh, el, er, whh.double(), erh, heads, fh, 0.2, mode)
    with pytest.raises(IndexError):
        gat_aggregate_staged(gst, wh, el, er, whh[:k - 5], erh[:k - 5], heads, fh, 0.2, mode)


@pytest.mark.parametrize("unsup", [False, True])
def test_sage_sharded_empty_shard(dev, unsup):
    """fewer seeds than ranks -- the empty shard still joins the gather with
    placeholders of the right widths (supervised and unsupervised nets), and the gathered
    result equals the single-process forward of the one non-empty shard (LocalGroup ranks)."""
    from graphneuralnetwork_amd import distributed as D
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    net, adj, table, seeds = _sage_setup(dev)
    if unsup:
        torch.manual_seed(4)
        net = GraphSAGE(2, table.shape[1], table.shape[1], False, agg_func="MEAN",
                        Unsupervised=True).to(dev).eval()
    one = seeds[:1]
    world = 2
    comm = D.LocalGroup(world)
    _run_ranks.comm = comm
    res = {}

    def rank_main(r):
        comm.bind(r)
        with torch.no_grad():
            res[r] = D.sage_forward_sharded(net, adj, table, one, r, world, seed=7, group=comm,
                                            gather=True)

    _run_ranks(world, rank_main)
    owner = [r for r in range(world) if D.shard_seeds(one, r, world).numel()][0]
    from graphneuralnetwork_amd.sampler import sample_batch
    with torch.no_grad():
        b = sample_batch(adj, one, (25, 10), seed=D.rank_sample_seed(7, owner))
        emb, logits = net(*b.forward_args(table), None, None, None, None, None)
    for r in range(world):
        e, lg = res[r]
        assert e.shape == (1, emb.shape[1])
        torch.testing.assert_close(e, emb)
        if unsup:
            assert lg is None
        else:
            assert lg.shape == (1, net.dense.out_features)
            torch.testing.assert_close(lg, logits)


def test_edge_cut_out_property_and_profile(dev):
    """EdgeCutSpmm.out is the tensor the last call wrote (also a caller's ``out``),
    and profile() neither changes it nor uses up a turn of the internal double buffer."""
    from graphneuralnetwork_amd import distributed as D
    n, F = 3000, 32
    g = _graph(n, dev)
    comm = D.LocalGroup(1)
    comm.bind(0)
    part = D.build_cover_exchange(g, 0, 1, group=comm)
    run = D.EdgeCutSpmm(part, F, dev, group=comm)
    x = torch.randn(n, F, device=dev)
    y1 = run(x)
    assert run.out is y1
    mine = torch.empty(n, F, device=dev)
    y2 = run(x, out=mine)
    assert y2 is mine and run.out is mine
    run.profile(x)
    assert run.out is mine
    y3 = run(x)
    assert y3 is not y1 and y3.data_ptr() != y1.data_ptr()  # the other internal buffer
    torch.testing.assert_close(y3, y1)


def test_halo_alltoallv_c_abi_single_rank(dev):
    """gnn_halo_alltoallv_f32 on a one-rank RCCL communicator made with the same librccl the
    entry resolves (ncclCommInitAll over device 0): the all-to-all-v of one rank is a copy."""
    import ctypes
    from graphneuralnetwork_amd import _lib
    lib = _lib.load()
    path = ctypes.create_string_buffer(4096)
    assert lib.gnn_halo_rccl_path(path, 4096) == 0
    rccl = ctypes.CDLL(path.value.decode())
    comm = (ctypes.c_void_p * 1)()
    devs = (ctypes.c_int * 1)(dev.index or 0)
    assert rccl.ncclCommInitAll(comm, 1, devs) == 0
    try:
        F, n = 24, 1000
        send = torch.randn(n, F, device=dev)
        recv = torch.empty(n, F, device=dev)
        cnt = (ctypes.c_int64 * 1)(n)
        s = torch.cuda.current_stream(dev)
        rc = lib.gnn_halo_alltoallv_f32(send.data_ptr(), cnt, recv.data_ptr(), cnt, F, 1,
                                        comm[0], s.cuda_stream)
        assert rc == 0, _lib.error_string(rc)
        torch.cuda.synchronize(dev)
        assert torch.equal(recv, send)
    finally:
        rccl.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        rccl.ncclCommDestroy(comm[0])


@pytest.mark.parametrize("chunks", [1, 2, 3])
def test_chunked_halo_exchange_two_ranks(dev, chunks):
    """The cover SpMM with its feature rows in `chunks` all-to-all-v's (EdgeCutSpmm chunks=,
    VERDICT r3 next #4): 2 LocalGroup ranks on one GPU equal the single-GPU SpMM (bias, ReLU on
    the last pass), and profile() reports when the first halo chunk started against when the
    last chunk landed."""
    from graphneuralnetwork_amd import distributed as D
    from graphneuralnetwork_amd.ops import spmm_forward
    W, n, F = 2, 20000, 64
    g = _graph(n, dev)
    comm = D.LocalGroup(W)
    _run_ranks.comm = comm
    parts = [None] * W

    def build(r):
        comm.bind(r)
        parts[r] = D.build_cover_exchange(g, r, W, group=comm)

    _run_ranks(W, build)
    X = torch.randn(n, F, device=dev)
    b = torch.randn(F, device=dev)
    Y = torch.empty(n, F, device=dev)
    profs = [None] * W
    streams = [torch.cuda.Stream(dev) for _ in range(W)]

    def step(r):
        comm.bind(r)
        r0, r1 = parts[r].bounds[r], parts[r].bounds[r + 1]
        with torch.cuda.stream(streams[r]):
            run = D.EdgeCutSpmm(parts[r], F, dev, group=comm, chunks=chunks)
            assert len(run.halo_x_chunks) == chunks
            x = X[r0:r1].contiguous()
            Y[r0:r1].copy_(run(x, b, activation="relu"))
            profs[r] = run.profile(x, b, activation="relu")
            torch.cuda.synchronize()

    _run_ranks(W, step)
    ref = torch.relu(spmm_forward(g, X, b))
    torch.testing.assert_close(Y, ref, rtol=1e-4, atol=1e-5 * float(ref.abs().max()))
    for p in profs:
        assert p["total_ms"] > 0
        if chunks > 1 and parts[0].any_x:
            assert {"halo_x0_start_at_ms", "a2a_x_last_end_at_ms",
                    "halo_before_last_recv_ms"} <= set(p)
            assert all(f"a2a_x{k}_ms" in p for k in range(chunks))


def test_rccl_world1_zero_and_chunked_all_to_all(dev):
    """The nccl (= RCCL) backend at world 1 (one GPU cannot host two RCCL ranks): the
    all-to-all-v calls the edge-cut path makes -- a zero-row chunk, a non-empty one, int64 and
    float64 handshakes, the float all-gather -- run through torch.distributed on RCCL."""
    from graphneuralnetwork_amd import distributed as D
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=dev)
    try:
        for rows in (0, 5, 1000):
            inp = torch.randn(rows, 64, device=dev)
            out = torch.empty_like(inp)
            D._all_to_all_v(out, inp, [rows], [rows])
            torch.cuda.synchronize()
            assert torch.equal(out, inp)
        for dt in (torch.int64, torch.float64):
            inp = torch.arange(12, device=dev).to(dt)
            out = torch.empty_like(inp)
            D._all_to_all_v(out, inp, [12], [12])
            assert torch.equal(out, inp)
        g = D._all_gather_floats([1.5, -2.0], 1, dev)
        assert g.tolist() == [[1.5, -2.0]]
        assert D._global_sum(7, dev) == 7
    finally:
        dist.destroy_process_group()
