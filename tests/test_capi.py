"""The C-ABI library: loads, exports every symbol include/gnn_mi355x.h declares,
and rejects bad arguments before launching anything (no GPU needed)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "gnn_mi355x.h"


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(gnn_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from graphneuralnetwork_amd import _lib
    return _lib.load(build_if_missing=True)


def test_header_symbols_exported(lib):
    from graphneuralnetwork_amd import _lib
    names = header_functions()
    assert names, "no functions parsed from the header"
    for n in names:
        assert hasattr(lib, n), f"{n} declared in gnn_mi355x.h but not exported"
    assert set(names) == set(_lib.SIGNATURES), "ctypes SIGNATURES out of sync with the header"


def test_exports_are_c_abi():
    import subprocess
    from graphneuralnetwork_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.library_path())],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gnn_\w+)", out))
    assert set(header_functions()) <= exported


def test_error_strings_and_version(lib):
    from graphneuralnetwork_amd import _lib
    assert lib.gnn_version() >= 100
    assert "invalid argument" in _lib.error_string(-1)
    assert "unsupported" in _lib.error_string(-3) or "not supported" in _lib.error_string(-3)


def test_argument_rejection_without_launch(lib):
    # null pointers / negative sizes -> GNN_E_ARG before anything reaches the device
    tail = (8, None, None, 0, None, None, 0, None, None, None, 0, None, 0, None, 0, None)
    rc = lib.gnn_spmm_csr_f32(None, None, None, 10, None, 4, 4, None, None, 4, *tail)
    assert rc == -1
    rc = lib.gnn_spmm_csr_f32(None, None, None, -1, None, 4, 4, None, None, 4, *tail)
    assert rc == -1
    assert lib.gnn_spmm_plan_count(None, 10, 4, None, None, None) == -1
    assert lib.gnn_spmm_plan_scratch_bytes(-5) < 0
    assert lib.gnn_spmm_plan_scratch_bytes(10_000_000) > 0
    # the transforms' arithmetic: the previous mode back, anything but 0 / 1 refused
    prev = lib.gnn_transform_set_precision(0)
    assert prev in (0, 1)
    assert lib.gnn_transform_get_precision() == 0
    from graphneuralnetwork_amd.ops import transform_precision
    assert transform_precision() == "fp32-mfma"  # read back from the library, not mirrored
    assert lib.gnn_transform_set_precision(prev) == 0
    assert lib.gnn_transform_get_precision() == prev
    assert lib.gnn_transform_set_precision(2) == -1
    # the task-list validator: argument checks before any launch
    assert lib.gnn_spmm_tasks_check(None, 1, 10, None, None) == -1
    assert lib.gnn_spmm_tasks_check(None, 0, 10, 16, None) == 0
    # the fused classifier: n_cls outside [1, 4] / missing operands, nothing launched
    for n_cls, wd, lg in ((0, 1, 1), (5, 1, 1), (3, None, 1), (3, 1, None)):
        assert lib.gnn_linear_relu_cls_f32(16, 256, 100, 256, 16, 128, 16, 128, wd, None, n_cls,
                                           lg, 4, None) == -1


def test_ops_refuse_cpu_tensors():
    import torch
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import spmm_forward
    g = CsrGraph(torch.zeros(3, dtype=torch.int64), torch.zeros(0, dtype=torch.int32),
                 torch.zeros(0), 2, 2)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        spmm_forward(g, torch.zeros(2, 4))


def test_halo_exchange_entry_without_gpu(lib):
    """gnn_halo_alltoallv_f32: argument checks before any RCCL call, and the
    RCCL the entry would call is resolved from the process (torch's own librccl)."""
    import ctypes
    import torch  # noqa: F401  (loads the RCCL that torch.distributed's nccl backend uses)
    counts = (ctypes.c_int64 * 2)(1, 1)
    assert lib.gnn_halo_alltoallv_f32(None, counts, None, counts, 4, 2, None, None) == -1
    assert lib.gnn_halo_alltoallv_f32(None, counts, None, counts, 4, 0, 1, None) == -1
    # rows * row_floats (or the running offsets) past 2^62 elements: refused, nothing called
    huge = (ctypes.c_int64 * 2)(1 << 40, 1)
    assert lib.gnn_halo_alltoallv_f32(16, huge, 16, counts, 1 << 30, 2, 1, None) == -3
    big = (ctypes.c_int64 * 2)(1 << 61, 1 << 61)
    assert lib.gnn_halo_alltoallv_f32(16, big, 16, counts, 2, 2, 1, None) == -3
    buf = ctypes.create_string_buffer(4096)
    assert lib.gnn_halo_rccl_path(buf, 4096) == 0, "ncclAllToAllv not resolvable"
    assert "rccl" in buf.value.decode()


def test_c_program_links_and_checks_usage():
    """examples/capi_gcn_spmm.c is built next to the library (build.py) from the header alone and
    loads here (no GPU): the usage check runs before any HIP call."""
    import subprocess
    from graphneuralnetwork_amd import build as B
    exe = B.LIB_DIR / "capi_gcn_spmm"
    if not exe.exists():
        B.build()
    B.build_examples()  # build() only warns when the example fails to build; here it must not
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


def test_build_stamp_ties_library_to_tree(lib, monkeypatch):
    """The library carries the stamp of the sources it was built from (build.lib_source_stamp,
    embedded as gnn_build_stamp()); load() refuses one whose stamp differs from this tree."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd import build as B
    assert _lib.build_stamp(lib) == B.lib_source_stamp()
    assert lib.gnn_build_defines().decode() == ""
    assert B.lib_source_stamp(("-DX=1",)) != B.lib_source_stamp()
    _lib.check_stamp(lib)
    monkeypatch.setattr(B, "lib_source_stamp", lambda defines=(): "0" * 16)
    with pytest.raises(RuntimeError, match="rebuild"):
        _lib.check_stamp(lib)
