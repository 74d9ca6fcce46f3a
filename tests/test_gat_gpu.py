"""GAT fused edge-softmax + aggregation on the GPU vs the reference's golden vectors and the oracle.

Tolerance: fp32 within 1e-4 relative (atol scaled by max |out|)."""
import numpy as np
import pytest
import torch

from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu


def close(a, b, rtol=1e-4):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.nanmax(np.abs(b)))) if b.size else 1.0
    np.testing.assert_allclose(a, b, rtol=rtol, atol=2e-5 * scale)


def _dense(g, prefix, n):
    A = np.zeros((n, n), np.float32)
    A[g[f"{prefix}_row"], g[f"{prefix}_col"]] = g[f"{prefix}_val"]
    return A


def _load_heads(model, g, kind):
    sd = {}
    H = g[f"{kind}_W"].shape[0]
    for i in range(H):
        sd[f"attentions.AttentionHead{i}.W"] = torch.from_numpy(g[f"{kind}_W"][i])
        a = g[f"{kind}_a"][i]
        sd[f"attentions.AttentionHead{i}.a"] = torch.from_numpy(a.reshape(-1, 1) if kind == "dense" else a.reshape(1, -1))
    sd["out_att.W"] = torch.from_numpy(g[f"{kind}_outW"])
    a = g[f"{kind}_outa"]
    sd["out_att.a"] = torch.from_numpy(a.reshape(-1, 1) if kind == "dense" else a.reshape(1, -1))
    model.load_state_dict(sd, strict=True)


@pytest.mark.parametrize("kind", ["dense", "sparse"])
@pytest.mark.parametrize("adj_form", ["dense", "sparse_coo"])
def test_golden_gat_models(golden, dev, kind, adj_form):
    from graphneuralnetwork_amd.gat import GAT, SpGAT
    g = golden("gat")
    n = int(g["n"])
    A = torch.from_numpy(_dense(g, "adj", n))
    adj = A.to(dev) if adj_form == "dense" else A.to_sparse().to(dev)
    model = (GAT if kind == "dense" else SpGAT)(64, 8, 7, 0.6, float(g["alpha"]), 8)
    _load_heads(model, g, kind)
    model.to(dev).eval()
    h = torch.from_numpy(g["h"]).to(dev)
    with torch.no_grad():
        logits = model(h, adj).cpu().numpy()
        head0 = model.attentions.AttentionHead0(h, adj).cpu().numpy()
    close(head0, g[f"{kind}_head0"])
    close(logits, g[f"{kind}_logits"])


def test_golden_edge_predicates_and_isolated_rows(golden, dev):
    from graphneuralnetwork_amd.gat import GraphAttentionLayer, SpGraphAttentionLayer
    g = golden("gat")
    n = int(g["n"])
    alpha = float(g["alpha"])
    h = torch.from_numpy(g["h"]).to(dev)
    dl = GraphAttentionLayer(64, 8, 0.0, alpha, True)
    sl = SpGraphAttentionLayer(64, 8, 0.0, alpha, True)
    dl.load_state_dict({"W": torch.from_numpy(g["neg_dense_W"]),
                        "a": torch.from_numpy(g["neg_dense_a"].reshape(-1, 1))})
    sl.load_state_dict({"W": torch.from_numpy(g["neg_sparse_W"]),
                        "a": torch.from_numpy(g["neg_sparse_a"].reshape(1, -1))})
    dl.to(dev).eval()
    sl.to(dev).eval()
    An = torch.from_numpy(_dense(g, "neg", n)).to(dev)
    with torch.no_grad():
        close(dl(h, An).cpu().numpy(), g["neg_dense_out"])   # edges: adj > 0
        close(sl(h, An).cpu().numpy(), g["neg_sparse_out"])  # edges: adj != 0
        Ai = _dense(g, "adj", n)
        Ai[int(g["iso_row"]), :] = 0
        Ai = torch.from_numpy(Ai).to(dev)
        close(dl(h, Ai).cpu().numpy(), g["iso_dense_out"])   # uniform average row
        with pytest.raises(AssertionError):                  # reference: NaN assert
            sl(h, Ai)


def _rand_csr(n, e, seed, hub=0):
    rng = np.random.default_rng(seed)
    s = np.concatenate([rng.integers(0, n, e), np.full(hub, 1)])
    d = np.concatenate([rng.integers(0, n, e), rng.integers(0, n, hub)])
    key = np.unique(s * n + d)
    rowptr, col, _ = O.coo_to_csr(key // n, key % n, np.ones(key.size, np.float32), n)
    return rowptr, col


@pytest.mark.parametrize("heads,fh", [(8, 8), (1, 7), (3, 5), (4, 16), (12, 4), (2, 64), (1, 200)])
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("seg_len", [None, 40])
def test_gat_aggregate_vs_oracle(dev, heads, fh, sparse, seg_len):
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, GAT_SPARSE, gat_aggregate, gat_logits
    n = 1500
    rowptr, col = _rand_csr(n, 12 * n, heads * 100 + fh, hub=900)
    rng = np.random.default_rng(fh)
    wh = (rng.standard_normal((n, heads * fh)) * 0.5).astype(np.float32)
    a_s = (rng.standard_normal(heads * fh) * 0.3).astype(np.float32)
    a_d = (rng.standard_normal(heads * fh) * 0.3).astype(np.float32)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    whd = torch.from_numpy(wh).to(dev)
    el, er = gat_logits(whd, heads, fh, torch.from_numpy(a_s).to(dev), torch.from_numpy(a_d).to(dev))
    el_o, er_o = O.gat_logits(wh, heads, fh, a_s, a_d)
    close(el.cpu().numpy(), el_o)
    close(er.cpu().numpy(), er_o)
    out = gat_aggregate(g, whd, el, er, heads, fh, 0.2, GAT_SPARSE if sparse else GAT_DENSE,
                        seg_len=seg_len).cpu().numpy()
    ref = O.gat_csr(rowptr, col, wh, el.cpu().numpy(), er.cpu().numpy(), heads, fh, 0.2, sparse)
    close(out, ref)


@pytest.mark.parametrize("heads,fh", [(8, 8), (3, 5), (12, 4)])
@pytest.mark.parametrize("sparse", [False, True])
def test_gat_hub_staging_bitexact(dev, heads, fh, sparse):
    """gnn_gat_csr_hub_f32 (staged Wh / er rows of the hub columns) reproduces the unstaged
    kernel bit for bit: outputs, log-sum-exp stats and dropout masks, in every row class
    (small, short, mid, long-row segments) and head group (12 heads = two launches)."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, GAT_SPARSE, gat_aggregate
    n = 2000
    rowptr, col = _rand_csr(n, 6 * n, heads + fh, hub=1500)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    wh = torch.randn(n, heads * fh, device=dev) * 0.5
    el, er = torch.randn(n, heads, device=dev), torch.randn(n, heads, device=dev)
    mode = GAT_SPARSE if sparse else GAT_DENSE
    for seg_len, p in ((None, 0.0), (24, 0.0), (24, 0.4)):
        st0 = torch.empty(n, heads, device=dev)
        ref = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, activation="elu", seg_len=seg_len,
                            dropout_p=p, seed=5, stats=st0, hubs=0)
        for k in (1, 50, n):
            st = torch.empty(n, heads, device=dev)
            out = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, activation="elu",
                                seg_len=seg_len, dropout_p=p, seed=5, stats=st, hubs=k)
            assert torch.equal(out, ref) or (torch.isnan(ref).any() and torch.equal(
                torch.nan_to_num(out, 1.5), torch.nan_to_num(ref, 1.5))), (seg_len, p, k)
            assert torch.equal(torch.nan_to_num(st, 1.5), torch.nan_to_num(st0, 1.5))


@pytest.mark.parametrize("heads,fh", [(8, 8), (12, 4), (1, 64), (2, 128)])
@pytest.mark.parametrize("sparse", [False, True])
def test_gat_packed_tasks_vs_short_rows(dev, heads, fh, sparse, monkeypatch):
    """gnn_gat_csr_tasks_f32 (low-degree rows as packed tasks; opt-in through ops.GAT_TASKS,
    measured slower than the row classes at cfg3)
    against the row-class path it replaces (packed small rows + gat_short_kernel) and the
    oracle: edgeless rows (dense: column mean; sparse: NaN), one-edge rows, runs longer than a
    task, long-row segments, two head groups (12 heads), hub staging, dropout (the same
    (edge, head) masks), ELU and the log-sum-exp stats."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    n = 3000
    rng = np.random.default_rng(heads * fh)
    deg = rng.integers(0, 14, n)
    deg[rng.integers(0, n, 40)] = rng.integers(17, 400, 40)
    deg[200:330] = 0                       # a run of edgeless rows longer than a task
    deg[600:700] = 1
    rowptr = np.zeros(n + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(n, d, replace=False)) for d in deg]).astype(np.int32)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    wh = torch.randn(n, heads * fh, device=dev) * 0.5
    el, er = torch.randn(n, heads, device=dev) * 0.7, torch.randn(n, heads, device=dev) * 0.7
    mode = ops.GAT_SPARSE if sparse else ops.GAT_DENSE
    ref_o = O.gat_csr(rowptr, col, wh.cpu().numpy(), el.cpu().numpy(), er.cpu().numpy(), heads,
                      fh, 0.2, sparse)
    for seg_len, p, hubs in ((None, 0.0, 0), (32, 0.0, 0), (32, 0.0, 100), (None, 0.3, 0)):
        outs = {}
        for tasks in (True, False):
            monkeypatch.setattr(ops, "GAT_TASKS", tasks)
            st = torch.empty(n, heads, device=dev)
            out = ops.gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, activation="elu",
                                    seg_len=seg_len, dropout_p=p, seed=11, stats=st, hubs=hubs)
            outs[tasks] = (out.cpu().numpy(), st.cpu().numpy())
        (a, sa), (b, sb) = outs[True], outs[False]
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
        close(np.nan_to_num(a), np.nan_to_num(b), rtol=1e-5)
        close(np.nan_to_num(sa, neginf=-1e30), np.nan_to_num(sb, neginf=-1e30), rtol=1e-5)
        if p == 0.0:
            elu = np.where(ref_o > 0, ref_o, np.expm1(np.minimum(ref_o, 0)))
            np.testing.assert_array_equal(np.isnan(a), np.isnan(elu))
            close(np.nan_to_num(a), np.nan_to_num(elu))


def _xcd_gat_graph(n, seed):
    """Edge set with hub columns 0..79 of strictly decreasing in-degree (hub rank = id), a
    hub row, one-edge rows into hub 0 (rows 0-99), edgeless rows (100-109), and rows whose
    edges all go to hubs of one XCD slice (110-119 -> columns 8, 16, ..., 64)."""
    rng = np.random.default_rng(seed)
    s = [rng.integers(130, n, 8 * n), np.full(1500, 1)]
    d = [rng.integers(0, n, 8 * n), rng.integers(0, n, 1500)]
    for c in range(80):
        s.append(rng.choice(np.arange(130, n), 1000 - 10 * c, replace=False))
        d.append(np.full(1000 - 10 * c, c))
    s += [np.arange(100), np.repeat(np.arange(110, 120), 8)]
    d += [np.zeros(100, np.int64), np.tile(np.arange(8, 72, 8), 10)]
    s, d = np.concatenate(s), np.concatenate(d)
    key = np.unique(s * n + d)
    rowptr, col, _ = O.coo_to_csr(key // n, key % n, np.ones(key.size, np.float32), n)
    return rowptr, col


@pytest.mark.parametrize("heads,fh", [(8, 8), (3, 5), (12, 4)])
@pytest.mark.parametrize("sparse", [False, True])
def test_gat_xcd_hub_staging(dev, heads, fh, sparse, monkeypatch):
    """XCD-sliced GAT (items per (row, XCD slice) merged as pseudo-edges with their
    log-sum-exp logit): equal to the single-pass kernel within fp32 rounding in every row
    class and head group, reproducible; dropout / stats requests keep the bit-exact path."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, GAT_SPARSE, gat_aggregate
    monkeypatch.setattr(ops, "XCD_MIN_DEG", 4)
    monkeypatch.setattr(ops, "XCD_CHUNK", 8)
    n = 2000
    rowptr, col = _xcd_gat_graph(n, heads + fh)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    wh = torch.randn(n, heads * fh, device=dev) * 0.5
    el, er = torch.randn(n, heads, device=dev), torch.randn(n, heads, device=dev)
    mode = GAT_SPARSE if sparse else GAT_DENSE
    for seg_len in (None, 24):
        ref = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", seg_len=seg_len, hubs=0)
        for k in (64, 200, n):  # (k = 8: one hub per slice, an edge set has no 2-edge item)
            out = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", seg_len=seg_len,
                                hubs=k, xcd=True)
            assert any(isinstance(key, tuple) and key[0] == "_xcd" and key[1] == k and v
                       for key, v in g._plans.items()), k
            close(out.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5)
            again = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", seg_len=seg_len,
                                  hubs=k, xcd=True)
            assert torch.equal(torch.nan_to_num(out, 1.5), torch.nan_to_num(again, 1.5))
    whn, eln, ern = (t.cpu().numpy().astype(np.float64) for t in (wh, el, er))
    o = O.gat_csr(rowptr, col, whn, eln, ern, heads, fh, 0.2, sparse)
    o = np.where(o > 0, o, np.expm1(np.minimum(o, 0)))
    ok = ~np.isnan(o).any(1)
    out = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", hubs=n, xcd=True)
    close(out.cpu().numpy()[ok], o[ok])
    # training requests (dropout, stats for the backward) take the bit-exact single pass
    st0, st1 = torch.empty(n, heads, device=dev), torch.empty(n, heads, device=dev)
    a = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", dropout_p=0.3, seed=2,
                      stats=st0, hubs=64, xcd=True)
    b = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", dropout_p=0.3, seed=2,
                      stats=st1, hubs=0)
    assert torch.equal(torch.nan_to_num(a, 1.5), torch.nan_to_num(b, 1.5))


@pytest.mark.parametrize("heads,fh,ld,off", [(8, 8, 80, 0), (8, 8, 67, 0), (4, 16, 64, 1),
                                              (3, 12, 40, 4)])
def test_gat_logits_strided_and_unaligned(dev, heads, fh, ld, off):
    """Vector (16-B aligned, fh % 4 == 0) and scalar fallbacks agree with the oracle."""
    from graphneuralnetwork_amd.ops import gat_logits
    n = 3000
    rng = np.random.default_rng(ld)
    big = rng.standard_normal((n, ld + off)).astype(np.float32)
    a = (rng.standard_normal(2 * heads * fh + 1) * 0.3).astype(np.float32)
    wh = big[:, off:off + heads * fh]
    whd = torch.from_numpy(big).to(dev)[:, off:off + heads * fh]
    ad = torch.from_numpy(a).to(dev)
    el, er = gat_logits(whd, heads, fh, ad[off % 2:off % 2 + heads * fh],
                        ad[heads * fh:2 * heads * fh])
    el_o, er_o = O.gat_logits(wh, heads, fh, a[off % 2:off % 2 + heads * fh],
                              a[heads * fh:2 * heads * fh])
    close(el.cpu().numpy(), el_o)
    close(er.cpu().numpy(), er_o)


def test_gat_dropout_is_seeded_and_unbiased(dev):
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, gat_aggregate
    n, heads, fh = 400, 2, 8
    rowptr, col = _rand_csr(n, 200 * n, 3)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    wh = torch.ones(n, heads * fh, device=dev)
    el = torch.zeros(n, heads, device=dev)
    er = torch.zeros(n, heads, device=dev)
    a = gat_aggregate(g, wh, el, er, heads, fh, 0.2, GAT_DENSE, dropout_p=0.5, seed=7)
    b = gat_aggregate(g, wh, el, er, heads, fh, 0.2, GAT_DENSE, dropout_p=0.5, seed=7)
    c = gat_aggregate(g, wh, el, er, heads, fh, 0.2, GAT_DENSE, dropout_p=0.5, seed=8)
    assert torch.equal(a, b) and not torch.equal(a, c)
    # uniform attention over ~200 edges, inverted dropout keeps the expectation at 1
    assert abs(float(a.mean()) - 1.0) < 0.02


def _torch_gat(Wh, a_src, a_dst, mask, H, fh, slope, sparse, elu):
    """Dense torch (float64) statement of both GAT layers for gradient checks."""
    n = Wh.shape[0]
    W3 = Wh.view(n, H, fh)
    el = (W3 * a_src.view(H, fh)).sum(-1)
    er = (W3 * a_dst.view(H, fh)).sum(-1)
    s = el[:, None, :] + er[None, :, :]
    x = torch.nn.functional.leaky_relu(s, slope)
    z = -x if sparse else x
    z = z.masked_fill(~mask[..., None], float("-inf"))
    att = torch.softmax(z, dim=1)
    out = torch.einsum("ijh,jhf->ihf", att, W3).reshape(n, H * fh)
    return torch.nn.functional.elu(out) if elu else out


@pytest.mark.parametrize("heads,fh", [(8, 8), (1, 7), (3, 4), (2, 16), (12, 4), (17, 2)])
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("seg_len", [None, 16])
@pytest.mark.parametrize("path", ["two_pass", "two_pass_sym", "three_pass"])
def test_gat_backward_vs_torch(dev, heads, fh, sparse, seg_len, path, monkeypatch):
    """Every head count trains: more than 8 heads run the edge pass in groups of 8 and
    reduce der 8 heads per pass inside the node kernel (>8 heads used to raise).
    two_pass: the row pass + recomputing node pass (every shape but fh = 7, whose 7 lanes per
    head take the three passes), over the transposed CSR or, for a graph marked symmetric, the
    graph itself; three_pass: GAT_BWD_RECOMPUTE off. Row 4 holds 200 extra edges (a long row /
    long column at seg_len 16); rows of <= 8 edges take the packed short-row waves."""
    from graphneuralnetwork_amd.gat import _GatLayerFn
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd import graph as graph_mod
    from graphneuralnetwork_amd import ops
    n = 300
    rng = np.random.default_rng(heads * 10 + fh)
    s = np.concatenate([rng.integers(0, n, 3000), np.arange(n), np.full(200, 4)])
    d = np.concatenate([rng.integers(0, n, 3000), np.arange(n), rng.integers(0, n, 200)])
    if path == "two_pass_sym":
        s, d = np.concatenate([s, d]), np.concatenate([d, s])
    key = np.unique(s * n + d)
    rowptr, col, _ = O.coo_to_csr(key // n, key % n, np.ones(key.size, np.float32), n)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n, symmetric=path == "two_pass_sym")
    monkeypatch.setattr(ops, "GAT_BWD_RECOMPUTE", path != "three_pass")
    ran = []
    inner = ops._gat_backward_recompute
    monkeypatch.setattr(ops, "_gat_backward_recompute",
                        lambda *a: ran.append(inner(*a)) or ran[-1])
    mask = torch.zeros(n, n, dtype=torch.bool)
    mask[key // n, key % n] = True
    feat = heads * fh
    Wh0 = torch.randn(n, feat, dtype=torch.float64) * 0.5
    as0 = torch.randn(feat, dtype=torch.float64) * 0.3
    ad0 = torch.randn(feat, dtype=torch.float64) * 0.3
    R = torch.randn(n, feat, dtype=torch.float64)
    old = graph_mod.seg_len_for
    if seg_len is not None:
        graph_mod.seg_len_for = lambda f, *a: seg_len
        import graphneuralnetwork_amd.ops as ops_mod
        ops_mod.seg_len_for = graph_mod.seg_len_for
    try:
        Wh = Wh0.float().to(dev).requires_grad_()
        a_s = as0.float().to(dev).requires_grad_()
        a_d = ad0.float().to(dev).requires_grad_()
        out = _GatLayerFn.apply(Wh, a_s, a_d, g, heads, fh, 0.2, 1 if sparse else 0, "elu", 0.0, 0)
        (out * R.float().to(dev)).sum().backward()
    finally:
        graph_mod.seg_len_for = old
        import graphneuralnetwork_amd.ops as ops_mod
        ops_mod.seg_len_for = old
    Wt = Wh0.clone().requires_grad_()
    ast = as0.clone().requires_grad_()
    adt = ad0.clone().requires_grad_()
    ref = _torch_gat(Wt, ast, adt, mask, heads, fh, 0.2, sparse, True)
    (ref * R).sum().backward()
    close(out.detach().cpu().numpy(), ref.detach().numpy())
    close(Wh.grad.cpu().numpy(), Wt.grad.numpy(), rtol=2e-4)
    close(a_s.grad.cpu().numpy(), ast.grad.numpy(), rtol=2e-4)
    close(a_d.grad.cpu().numpy(), adt.grad.numpy(), rtol=2e-4)
    if path == "three_pass":
        assert not ran
    else:  # the two-pass kernels ran unless the shape is one they refuse
        assert len(ran) == 1 and (ran[0] is not None) == (fh != 7)


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_gat_model_trains(golden, dev, kind):
    """GAT drop-in under autograd (train mode, dropout 0.6): loss decreases with SGD."""
    from graphneuralnetwork_amd.gat import GAT, SpGAT
    g = golden("gat")
    n = int(g["n"])
    A = torch.from_numpy(_dense(g, "adj", n)).to(dev)
    h = torch.from_numpy(g["h"]).to(dev)
    model = (GAT if kind == "dense" else SpGAT)(64, 8, 7, 0.6, float(g["alpha"]), 8).to(dev)
    _load_heads(model, g, kind)
    model.to(dev).train()
    labels = torch.from_numpy(np.random.default_rng(0).integers(0, 7, n)).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    losses = []
    torch.manual_seed(0)
    for _ in range(30):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(h, A), labels)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert all(np.isfinite(losses)) and np.mean(losses[-5:]) < np.mean(losses[:5])


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("recompute", [True, False])
def test_gat_dropout_backward_exact(dev, sparse, recompute, monkeypatch):
    """With dropout the backward must use the forward's mask: recover the mask by running
    the forward on an identity Wh (out = m * alpha), then check gradients against torch
    (the two-pass backward hashes the CSR edge id read through eid_t, the three-pass one the
    edge it walks)."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gat import _GatLayerFn
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, GAT_SPARSE, gat_aggregate, gat_logits
    monkeypatch.setattr(ops, "GAT_BWD_RECOMPUTE", recompute)
    n, p, seed = 64, 0.4, 1234
    rng = np.random.default_rng(3)
    s = np.concatenate([rng.integers(0, n, 600), np.arange(n)])
    d = np.concatenate([rng.integers(0, n, 600), np.arange(n)])
    key = np.unique(s * n + d)
    rowptr, col, _ = O.coo_to_csr(key // n, key % n, np.ones(key.size, np.float32), n)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    mode = GAT_SPARSE if sparse else GAT_DENSE
    # mask: the logits do not depend on Wh when a_src = a_dst = 0 -> alpha = uniform
    eye = torch.eye(n, device=dev)
    z = torch.zeros(n, 1, device=dev)
    masked = gat_aggregate(g, eye, z, z, 1, n, 0.2, mode, dropout_p=p, seed=seed)
    plain = gat_aggregate(g, eye, z, z, 1, n, 0.2, mode)
    M = torch.where(plain > 0, masked / plain, torch.zeros_like(plain)).double().cpu()
    mask = torch.zeros(n, n, dtype=torch.bool)
    mask[key // n, key % n] = True
    Wh0 = torch.randn(n, n, dtype=torch.float64) * 0.5
    as0 = torch.randn(n, dtype=torch.float64) * 0.2
    ad0 = torch.randn(n, dtype=torch.float64) * 0.2
    R = torch.randn(n, n, dtype=torch.float64)
    Wh = Wh0.float().to(dev).requires_grad_()
    a_s = as0.float().to(dev).requires_grad_()
    a_d = ad0.float().to(dev).requires_grad_()
    out = _GatLayerFn.apply(Wh, a_s, a_d, g, 1, n, 0.2, mode, None, p, seed)
    (out * R.float().to(dev)).sum().backward()
    Wt, ast, adt = (t.clone().requires_grad_() for t in (Wh0, as0, ad0))
    el = Wt @ ast
    er = Wt @ adt
    x = torch.nn.functional.leaky_relu(el[:, None] + er[None, :], 0.2)
    zz = (-x if sparse else x).masked_fill(~mask, float("-inf"))
    ref = (M * torch.softmax(zz, dim=1)) @ Wt
    (ref * R).sum().backward()
    close(out.detach().cpu().numpy(), ref.detach().numpy())
    close(Wh.grad.cpu().numpy(), Wt.grad.numpy(), rtol=2e-4)
    close(a_s.grad.cpu().numpy(), ast.grad.numpy(), rtol=2e-4)
    close(a_d.grad.cpu().numpy(), adt.grad.numpy(), rtol=2e-4)


@pytest.mark.parametrize("n,k,heads,fh", [(1000, 64, 8, 8), (777, 32, 2, 16), (50, 16, 1, 16),
                                          (3001, 128, 4, 8), (129, 256, 2, 8), (64, 64, 4, 16),
                                          (500, 64, 1, 64), (300, 32, 1, 32), (99, 64, 8, 8),
                                          (70, 16, 8, 2), (40, 32, 4, 4)])
def test_gat_project_mfma_vs_oracle(dev, n, k, heads, fh):
    """Fused MFMA transform: Wh = X W within fp32 tolerance of a float64 GEMM; el/er
    within fp32 tolerance of gnn_gat_logits_f32 run on the produced Wh."""
    from graphneuralnetwork_amd.ops import gat_logits, gat_project
    rng = np.random.default_rng(n + k)
    x = rng.standard_normal((n, k)).astype(np.float32)
    w = (rng.standard_normal((k, heads * fh)) / np.sqrt(k)).astype(np.float32)
    a_s = rng.standard_normal(heads * fh).astype(np.float32)
    a_d = rng.standard_normal(heads * fh).astype(np.float32)
    r = gat_project(torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev), heads, fh,
                    torch.from_numpy(a_s).to(dev), torch.from_numpy(a_d).to(dev))
    assert r is not None
    wh, el, er = r
    close(wh.cpu().numpy(), x.astype(np.float64) @ w.astype(np.float64))
    el2, er2 = gat_logits(wh, heads, fh, torch.from_numpy(a_s).to(dev), torch.from_numpy(a_d).to(dev))
    close(el.cpu().numpy(), el2.cpu().numpy())
    close(er.cpu().numpy(), er2.cpu().numpy())
    el_o, er_o = O.gat_logits(wh.cpu().numpy(), heads, fh, a_s, a_d)
    close(el.cpu().numpy(), el_o)


def test_gat_project_packed_layout_bitexact(dev):
    """gat_project(packed=True): Wh / er / el as views of one [n, H*Fh + 2H] buffer; the
    aggregation over them (el / er row stride H*Fh + 2H) gives the same bits."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, GAT_SPARSE, gat_aggregate, gat_project
    n, H, fh, k = 3000, 8, 8, 64
    rowptr, col = _rand_csr(n, 8 * n, 11, hub=2000)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    x = torch.randn(n, k, device=dev)
    w = torch.randn(k, H * fh, device=dev) * 0.2
    a_s, a_d = torch.randn(H * fh, device=dev) * 0.3, torch.randn(H * fh, device=dev) * 0.3
    p0 = gat_project(x, w, H, fh, a_s, a_d)
    p1 = gat_project(x, w, H, fh, a_s, a_d, packed=True)
    assert p1[0].stride(0) == H * fh + 2 * H and p1[1].stride(0) == H * fh + 2 * H
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    for mode in (GAT_DENSE, GAT_SPARSE):
        for hubs in (0, 100):
            r0 = gat_aggregate(g, *p0, H, fh, 0.2, mode, "elu", seg_len=32, hubs=hubs)
            r1 = gat_aggregate(g, *p1, H, fh, 0.2, mode, "elu", seg_len=32, hubs=hubs)
            assert torch.equal(r0, r1), (mode, hubs)


def test_gat_project_unsupported_shapes_fall_back(dev):
    from graphneuralnetwork_amd.ops import gat_project
    x = torch.randn(10, 48, device=dev)
    assert gat_project(x, torch.randn(48, 64, device=dev), 8, 8, torch.randn(64, device=dev),
                       torch.randn(64, device=dev)) is None          # k = 48
    assert gat_project(torch.randn(10, 64, device=dev), torch.randn(64, 7, device=dev), 1, 7,
                       torch.randn(7, device=dev), torch.randn(7, device=dev)) is None  # fout = 7
    assert gat_project(torch.randn(10, 32, device=dev), torch.randn(32, 64, device=dev), 16, 4,
                       torch.randn(64, device=dev), torch.randn(64, device=dev)) is None  # 16 heads
    # strided x (not 16-B aligned rows) is copied, still exact
    big = torch.randn(33, 65, device=dev)
    w = torch.randn(64, 16, device=dev)
    wh, _, _ = gat_project(big[:, 1:], w, 2, 8, torch.randn(16, device=dev), torch.randn(16, device=dev))
    close(wh.cpu().numpy(), big[:, 1:].cpu().double().numpy() @ w.cpu().double().numpy())


def test_gat_project_col_rows_bitexact(dev):
    """gat_project(col_rows=inv): Wh / er of node i land in row inv[i], el stays in row i;
    the values are the in-order projection's bits. An id out of range is not stored."""
    from graphneuralnetwork_amd.ops import gat_project
    n, H, fh, k = 3000, 8, 8, 64
    x = torch.randn(n, k, device=dev)
    w = torch.randn(k, H * fh, device=dev) * 0.2
    a_s, a_d = torch.randn(H * fh, device=dev) * 0.3, torch.randn(H * fh, device=dev) * 0.3
    wh0, el0, er0 = gat_project(x, w, H, fh, a_s, a_d)
    inv = torch.randperm(n, device=dev)
    wh, el, er = gat_project(x, w, H, fh, a_s, a_d, col_rows=inv)
    assert torch.equal(wh[inv], wh0) and torch.equal(er[inv], er0) and torch.equal(el, el0)
    bad = inv.clone()
    bad[5] = n + 7
    wh2, el2, er2 = gat_project(x, w, H, fh, a_s, a_d, col_rows=bad)
    keep = torch.ones(n, dtype=torch.bool, device=dev)
    keep[5] = False
    assert torch.equal(wh2[bad[keep]], wh0[keep]) and torch.equal(el2, el0)
    with pytest.raises(ValueError):
        gat_project(x, w, H, fh, a_s, a_d, packed=True, col_rows=inv)


@pytest.mark.parametrize("kind", ["GAT", "SpGAT"])
def test_gat_model_column_order(dev, kind, monkeypatch):
    """GAT / SpGAT inference on a graph whose Wh is hub-staged: every attention layer runs
    over the column-degree-ordered graph (projection rows scattered, hub rows read in place)
    and equals the natural-order path bit for bit (no edgeless rows) and the oracle."""
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    monkeypatch.setattr(ops, "HUB_MIN_X_BYTES", 0)
    n, nfeat = 2500, 64
    rowptr, col = _rand_csr(n, 8 * n, 21, hub=1800)
    assert (np.diff(rowptr) > 0).all()
    torch.manual_seed(0)
    model = getattr(gat_mod, kind)(nfeat, 8, 16, 0.1, 0.2, 8).to(dev).eval()
    x = torch.randn(n, nfeat, device=dev)

    def graph():
        return CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                        torch.ones(col.size, device=dev), n, n)

    g = graph()
    with torch.no_grad():
        y = model(x, g)
        assert ("_colorder",) in g._plans
        hp = next(p for key, p in g._plans[("_colorder",)].graph._plans.items()
                  if isinstance(key, tuple) and key[0] == "_hub")
        assert hp.prefix
        monkeypatch.setattr(ops, "DEGREE_ORDER", False)
        y_nat = model(x, graph())
    assert torch.equal(y, y_nat)


@pytest.mark.parametrize("er_rec", [False, True])
def test_gat_backward_two_pass_matches_three_pass_cfg3(dev, monkeypatch, er_rec):
    """At BASELINE cfg3 size (R-MAT 1M / 10M, symmetric normalised adjacency, 8 x 8 heads) the
    two-pass backward (row pass + recomputing node pass over the graph itself; er_rec: the row
    pass takes er_j from the gathered rows) and the three-pass one agree on dWh, dout, del and
    der within fp32 summation-order differences."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(1_000_000, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), 1_000_000, device=dev)
    H, Fh = 8, 8
    gen = torch.Generator(device=dev).manual_seed(2)
    wh = torch.randn(g.n_rows, H * Fh, device=dev, generator=gen)
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    el, er = ops.gat_logits(wh, H, Fh, a_s, a_d)
    stats = torch.empty((g.n_rows, H), device=dev)
    y = ops.gat_aggregate(g, wh, el, er, H, Fh, 0.2, ops.GAT_DENSE, "elu", stats=stats)
    dy = torch.randn(g.n_rows, H * Fh, device=dev, generator=gen)
    monkeypatch.setattr(ops, "GAT_ER_RECOMPUTE", er_rec)
    res = {}
    for rc in (True, False):
        monkeypatch.setattr(ops, "GAT_BWD_RECOMPUTE", rc)
        tl = []
        res[rc] = ops.gat_backward(g, wh, el, er, stats, y, dy, a_s, a_d, H, Fh, 0.2,
                                   ops.GAT_DENSE, True, timings=tl)
        assert [t[0] for t in tl] == (["rows", "nodes"] if rc else ["prep", "edges", "nodes"])
    for a, b in zip(res[True], res[False]):
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err < 1e-5, err


@pytest.mark.parametrize("heads,fh", [(8, 8), (1, 16), (4, 4), (2, 32), (3, 8), (1, 7), (16, 4)])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("hubs", [0, 64])
def test_gat_er_recomputed_from_rows(dev, heads, fh, mode, hubs, monkeypatch):
    """gnn_gat_csr_ex_f32 with a_dst (er_j recomputed from the gathered Wh_j rows: one-chunk
    rows, short rows, one-edge rows) against the er-gathering launch: outputs and per-row LSE
    stats within fp32 rounding of er's dot product, dropout masks identical; rows of every class
    (edgeless, one edge, short, mid, a long row split into segments), hub tables on and off.
    Shapes whose head lanes are not a power of two (fh = 7) fall back to gathering er."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import gat_aggregate, gat_logits
    monkeypatch.setattr(ops, "GAT_ER_RECOMPUTE", True)
    n = 700
    rng = np.random.default_rng(heads * 100 + fh)
    deg = rng.choice([0, 1, 2, 5, 12, 40], n)
    deg[3] = 900  # a long row
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(n, d, replace=d > n)) for d in deg]).astype(np.int32)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    feat = heads * fh
    gen = torch.Generator(device=dev).manual_seed(7)
    wh = torch.randn(n, feat, device=dev, generator=gen)
    a_s = torch.randn(feat, device=dev, generator=gen) * 0.3
    a_d = torch.randn(feat, device=dev, generator=gen) * 0.3
    el, er = gat_logits(wh, heads, fh, a_s, a_d)
    for drop in (0.0, 0.3):
        s0 = torch.empty(n, heads, device=dev)
        s1 = torch.empty(n, heads, device=dev)
        y0 = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", dropout_p=drop, seed=5,
                           stats=s0, hubs=hubs)
        y1 = gat_aggregate(g, wh, el, er, heads, fh, 0.2, mode, "elu", dropout_p=drop, seed=5,
                           stats=s1, hubs=hubs, a_dst=a_d)
        fin = torch.isfinite(y0)
        assert torch.equal(fin, torch.isfinite(y1))
        close(y1[fin].cpu().numpy(), y0[fin].cpu().numpy(), rtol=1e-5)
        sf = torch.isfinite(s0)
        assert torch.equal(sf, torch.isfinite(s1))
        close(s1[sf].cpu().numpy(), s0[sf].cpu().numpy(), rtol=1e-5)


@pytest.mark.parametrize("kind", ["GAT", "SpGAT"])
def test_gat_training_in_degree_order_equals_natural(dev, kind, monkeypatch):
    """GATBase.forward in training runs the model over P A P^T (ops.gat_train_order: x permuted
    on entry, the logits on exit): logits and every parameter's gradient equal the
    natural-order training step within fp32 rounding (dropout 0: the relabelled edges would
    draw other masks), and x's gradient comes back in the original row order."""
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    monkeypatch.setattr(ops, "HUB_MIN_X_BYTES", 0)
    n, nfeat = 3000, 64
    rowptr, col = _rand_csr(n, 8 * n, 23, hub=2200)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    key = np.unique(np.concatenate([rows * n + col, col.astype(np.int64) * n + rows,
                                    np.arange(n) * (n + 1)]))  # symmetric, self-loops
    r, c = key // n, (key % n).astype(np.int32)
    rp = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=n))]).astype(np.int64)

    def graph():
        return CsrGraph(torch.from_numpy(rp).to(dev), torch.from_numpy(c).to(dev),
                        torch.ones(c.size, device=dev), n, n, symmetric=True)

    torch.manual_seed(0)
    model = getattr(gat_mod, kind)(nfeat, 8, 5, 0.0, 0.2, 8).to(dev).train()
    x = torch.randn(n, nfeat, device=dev)
    lab = torch.randint(0, 5, (n,), device=dev)
    res = {}
    for use in (True, False):
        monkeypatch.setattr(ops, "GAT_TRAIN_ORDER", use)
        g = graph()
        xx = x.clone().requires_grad_(True)
        model.zero_grad(set_to_none=True)
        y = model(xx, g)
        torch.nn.functional.nll_loss(torch.nn.functional.log_softmax(y, 1), lab).backward()
        assert (("_nodeorder",) in g._plans) == use
        res[use] = [y.detach(), xx.grad] + [p.grad.clone() for p in model.parameters()]
    for a, b in zip(res[True], res[False]):
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err < 1e-5, err


@pytest.mark.parametrize("kind", ["GAT", "SpGAT"])
@pytest.mark.parametrize("nclass", [3, 7])
def test_gat_narrow_out_att_padded_backward(dev, kind, nclass, monkeypatch):
    """A classifier attention layer whose width the two-pass backward cannot lay out (3 or 7
    classes: GAT/run.py's out_att) trains zero-padded to 4 / 8 features: the logits and every
    gradient equal the unpadded three-pass backward's, and its dW / da come from the narrow
    gemm_tn kernel."""
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd.graph import CsrGraph
    n = 2000
    rowptr, col = _rand_csr(n, 12 * n, 31, hub=900)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    key = np.unique(np.concatenate([rows * n + col, np.arange(n) * (n + 1)]))  # self-loops
    r, c = key // n, (key % n).astype(np.int32)
    rp = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=n))]).astype(np.int64)
    g = CsrGraph(torch.from_numpy(rp).to(dev), torch.from_numpy(c).to(dev),
                 torch.ones(c.size, device=dev), n, n)
    torch.manual_seed(0)
    model = getattr(gat_mod, kind)(64, 8, nclass, 0.0, 0.2, 8).to(dev).train()
    x = torch.randn(n, 64, device=dev)
    lab = torch.randint(0, nclass, (n,), device=dev)
    assert gat_mod._padded_fh(1, nclass, torch.empty(1, nclass, device=dev)) in (4, 8)
    res = {}
    for pad in (True, False):
        if not pad:
            monkeypatch.setattr(gat_mod, "_padded_fh", lambda heads, fh, Wh: fh)
        xx = x.clone().requires_grad_(True)
        model.zero_grad(set_to_none=True)
        y = model(xx, g)
        torch.nn.functional.nll_loss(torch.nn.functional.log_softmax(y, 1), lab).backward()
        res[pad] = [y.detach(), xx.grad] + [p.grad.clone() for p in model.parameters()]
    for a, b in zip(res[True], res[False]):
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err < 1e-5, err


def test_gat_replay_restores_the_plan(dev):
    """bench.gat_replay (the GAT aggregation's measured ceiling, gathered ids rewritten in place
    in the hub plan's column array) leaves the plan as it found it: the aggregation after the
    replay equals the one before it bit for bit; every gather from an L2-sized table is faster
    than the step as built."""
    import bench
    from graphneuralnetwork_amd.ops import (GAT_DENSE, gat_aggregate, gat_column_order,
                                            gat_project, hub_rows_for)
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, H, Fh = 1_000_000, 8, 8
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    order = gat_column_order(g, H, Fh)
    assert order is not None
    ga = order.graph
    gen = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn(n, 64, device=dev, generator=gen)
    W = torch.randn(64, H * Fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    wh, el, er = gat_project(X, W, H, Fh, a_s, a_d, col_rows=order.inv)
    out = torch.empty_like(wh)
    fn = lambda: gat_aggregate(ga, wh, el, er, H, Fh, 0.2, GAT_DENSE, "elu", out=out, a_dst=a_d)
    y0 = fn().clone()
    r = bench.gat_replay(ga, hub_rows_for(ga.n_cols, H * Fh + H), fn, reps=2)
    assert r is not None and r["hub_gathers"] > 0 and r["nonhub_gathers"] > 0
    assert r["all_gathers_in_L2_ms"] < r["as_built_ms"]
    assert torch.equal(fn(), y0)
