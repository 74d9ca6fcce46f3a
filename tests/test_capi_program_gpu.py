"""A plain-C caller of the library (examples/capi_gcn_spmm.c, built next to it by build.py):
the GCN aggregation of bench.py's cfg2 step with every schedule built through the C-ABI --
adjacency, column order, hub ranks, XCD items, row plans, packed tasks, both SpMM passes --
and no Python in the process. Its output must equal the package's spmm_forward over the same
column-ordered graph bit for bit (same kernels, same schedules), and the oracle on a row sample
within the north star's 1e-4."""
import json
import subprocess

import numpy as np
import pytest
import torch

from oracle import c_oracle

pytestmark = pytest.mark.gpu


def test_c_program_matches_package(dev, tmp_path):
    from graphneuralnetwork_amd import build as B
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    exe = B.LIB_DIR / "capi_gcn_spmm"
    assert exe.exists(), "examples/capi_gcn_spmm.c is built by graphneuralnetwork_amd.build"
    # above the XCD path's thresholds (X >= 192 MiB, >= 4M entries), like cfg2
    n, m, F = 500_000, 5_000_000, 128
    s, d = rmat_edges(n, m, 3)
    (tmp_path / "edges.bin").write_bytes(
        np.concatenate([s.astype(np.int64), d.astype(np.int64)]).tobytes())
    X = np.random.default_rng(1).standard_normal((n, F)).astype(np.float32)
    (tmp_path / "x.bin").write_bytes(X.tobytes())
    r = subprocess.run([str(exe), str(tmp_path / "edges.bin"), str(tmp_path / "x.bin"),
                        str(tmp_path / "y.bin"), str(n), str(m), str(F)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    Yc = np.fromfile(tmp_path / "y.bin", dtype=np.float32).reshape(n, F)

    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    assert info["nnz"] == g.nnz and info["items"] > 0 and info["tasks"] > 0
    o = column_order(g, F)
    assert o is not None
    Xd = torch.from_numpy(X).to(dev)
    Yp = spmm_forward(o.graph, Xd[o.perm].contiguous())
    assert np.array_equal(Yc, Yp.cpu().numpy())

    h = {k: getattr(g, k).cpu().numpy() for k in ("rowptr", "col", "val")}
    deg = np.diff(h["rowptr"])
    rows = np.unique(np.concatenate([np.argsort(-deg)[:16],
                                     np.random.default_rng(2).choice(n, 500, replace=False)]))
    ref = np.concatenate([c_oracle.spmm_csr(h["rowptr"], h["col"], h["val"], X, None, r0, r0 + 1)
                          for r0 in rows])
    got = Yc[rows].astype(np.float64)
    scale = max(1.0, float(np.abs(ref).max()))
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5 * scale)
