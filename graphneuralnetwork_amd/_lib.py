"""ctypes binding of libgnn_mi355x.so (the C-ABI in include/gnn_mi355x.h).

This is the Python-side FFI the reference's modules call into: plain device
pointers (``tensor.data_ptr()``), sizes and the current HIP stream handle go
across; nothing else.  The library is loaded lazily and only after ``torch``
(so that it binds to the HIP runtime torch already loaded).  There is no CPU
fallback: if the library is missing every op raises.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

import torch  # noqa: F401  (must be imported before the HIP library is dlopen'ed)

from . import build as _build

_lock = threading.Lock()
_lib: ctypes.CDLL | None = None

_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/gnn_mi355x.h exactly.
SIGNATURES: dict[str, tuple] = {
    "gnn_version": (ctypes.c_int, []),
    "gnn_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "gnn_build_stamp": (ctypes.c_char_p, []),
    "gnn_build_defines": (ctypes.c_char_p, []),
    "gnn_spmm_csr_f32": (ctypes.c_int, [
        _vp, _vp, _vp, _i64,            # rowptr, col, val, n_rows
        _vp, _i64, _i64,                # x, ldx, feat
        _vp, _vp, _i64,                 # bias, y, ldy
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _vp, _vp, _i64,            # small_row, small_col, small_val, n_small
        _vp, _i64, _vp,                 # mid_row, n_mid, partial
        _u32, _vp]),                    # flags, stream
    "gnn_spmm_csr_hub_f32": (ctypes.c_int, [
        _vp, _vp, _vp, _i64,            # rowptr, col_hub, val, n_rows
        _vp, _i64, _vp, _i64, _i64,     # x, ldx, xh, ldh, feat
        _vp, _vp, _i64,                 # bias, y, ldy
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _vp, _vp, _i64,            # small_row, small_col, small_val, n_small
        _vp, _i64, _vp,                 # mid_row, n_mid, partial
        _u32, _vp]),                    # flags, stream
    "gnn_spmm_csr_tasks_f32": (ctypes.c_int, [
        _vp, _vp, _vp, _i64,            # rowptr, col, val, n_rows
        _vp, _i64, _vp, _i64, _i64,     # x, ldx, xh (nullable), ldh, feat
        _vp, _vp, _i64,                 # bias, y, ldy
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _i64, _vp, _i64,           # mid_row, n_mid, task_row, n_task
        _vp, _u32, _vp]),               # partial, flags, stream
    "gnn_spmm_tasks_check": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp]),
    "gnn_sage_gather_concat_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp, _i64, _i64, _i64,
                                                   _i64, _i32, _vp, _i64, _vp, _i64, _vp, _vp]),
    "gnn_sage_gather_concat_live_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp, _i64, _i64, _vp,
                                                        _i64, _i64, _i32, _vp, _i64, _vp, _i64,
                                                        _vp, _vp]),
    "gnn_halo_alltoallv_f32": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp]),
    "gnn_halo_rccl_path": (ctypes.c_int, [ctypes.c_char_p, _i64]),
    "gnn_spmm_plan_scratch_bytes": (_i64, [_i64]),
    "gnn_hub_plan_workspace_bytes": (_i64, [_i64]),
    "gnn_spmm_tasks_workspace_bytes": (_i64, [_i64]),
    "gnn_spmm_tasks_build": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64,
                                            _vp]),
    "gnn_column_order_workspace_bytes": (_i64, [_i64]),
    "gnn_column_order": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gnn_cover_workspace_bytes": (_i64, [_i64, _i64, _i64, _i32]),
    "gnn_cover_build": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i32, _i32, _vp, _vp, _i64, _vp]),
    "gnn_cover_fill": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _i32, _i32, _vp,
                                      _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _vp, _vp, _vp]),
    "gnn_cover_send_workspace_bytes": (_i64, [_i64]),
    "gnn_cover_send_partials": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, _i64, _i64, _i64, _vp,
                                               _vp, _vp, _vp, _i64, _vp]),
    "gnn_xcd_hub_plan_workspace_bytes": (_i64, [_i64, _i64]),
    "gnn_xcd_slice_group": (_i64, []),
    "gnn_xcd_hub_plan_build": (ctypes.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                              _i64, _vp, _vp, _i64, _vp]),
    "gnn_xcd_hub_plan_fill": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp,
                                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gnn_in_degree_u32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gnn_hub_plan_build": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gnn_spmm_plan_count": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gnn_spmm_plan_fill": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp, _vp]),
    "gnn_gat_logits_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64,
                                          _vp]),
    "gnn_gat_project_supported": (ctypes.c_int, [_i64, _i64, _i64]),
    "gnn_gcn_transform_supported": (ctypes.c_int, [_i64, _i64]),
    "gnn_transform_set_precision": (ctypes.c_int, [ctypes.c_int]),
    "gnn_transform_get_precision": (ctypes.c_int, []),
    "gnn_gcn_transform_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "gnn_gcn_transform_epi_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i32,
                                                 ctypes.c_float, ctypes.c_uint64, _vp, _i64, _vp]),
    "gnn_linear_relu_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "gnn_linear_relu_live_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                                                _vp]),
    "gnn_linear_relu_cls_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64,
                                               _vp, _vp, _i64, _vp, _i64, _vp]),
    "gnn_gcn_transform_rows_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64,
                                                  _vp, _i64, _vp, _vp]),
    "gnn_normalize_features_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp]),
    "gnn_gat_project_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _i64,
                                           _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "gnn_gat_project_rows_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64,
                                                _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp]),
    "gnn_gat_csr_f32": (ctypes.c_int, [
        _vp, _vp, _i64,                 # rowptr, col, n_rows
        _vp, _i64, _i64, _i64,          # wh, ldw, heads, fh
        _vp, _vp, _i64,                 # el, er, lde
        ctypes.c_float, _i32, _vp,      # negative_slope, mode, empty_row_fill
        ctypes.c_float, ctypes.c_uint64,  # dropout_p, dropout_seed
        _vp, _i64,                      # out, ldo
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _vp, _i64,                 # small_row, small_col, n_small
        _vp, _i64, _vp, _i64,           # mid_row, n_mid, short_row, n_short
        _vp, _vp,                       # partial, stats
        _u32, _vp]),                    # flags, stream
    "gnn_gat_csr_hub_f32": (ctypes.c_int, [
        _vp, _vp, _i64,                 # rowptr, col_hub, n_rows
        _vp, _i64, _i64, _i64,          # wh, ldw, heads, fh
        _vp, _vp, _i64,                 # el, er, lde
        ctypes.c_float, _i32, _vp,      # negative_slope, mode, empty_row_fill
        ctypes.c_float, ctypes.c_uint64,  # dropout_p, dropout_seed
        _vp, _i64,                      # out, ldo
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _vp, _i64,                 # small_row, small_col, n_small
        _vp, _i64, _vp, _i64,           # mid_row, n_mid, short_row, n_short
        _vp, _vp,                       # partial, stats
        _u32, _vp,                      # flags, stream
        _vp, _i64, _vp, _i64]),
    "gnn_gat_csr_ex_f32": (ctypes.c_int, [
        _vp, _vp, _i64,                 # rowptr, col_hub, n_rows
        _vp, _i64, _i64, _i64,          # wh, ldw, heads, fh
        _vp, _vp, _i64,                 # el, er, lde
        ctypes.c_float, _i32, _vp,      # negative_slope, mode, empty_row_fill
        ctypes.c_float, ctypes.c_uint64,  # dropout_p, dropout_seed
        _vp, _i64,                      # out, ldo
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _vp, _i64,                 # small_row, small_col, n_small
        _vp, _i64, _vp, _i64,           # mid_row, n_mid, short_row, n_short
        _vp, _vp,                       # partial, stats
        _u32, _vp,                      # flags, stream
        _vp, _i64, _vp, _i64,           # whh, ldwh, erh, ldeh (NULL: no staged tables)
        _vp]),                          # a_dst (NULL: er gathered)
    "gnn_gat_csr_tasks_f32": (ctypes.c_int, [
        _vp, _vp, _i64,                 # rowptr, col (hub ranks -1-k when staged), n_rows
        _vp, _i64, _i64, _i64,          # wh, ldw, heads, fh
        _vp, _vp, _i64,                 # el, er, lde
        ctypes.c_float, _i32, _vp,      # negative_slope, mode, empty_row_fill
        ctypes.c_float, ctypes.c_uint64,  # dropout_p, dropout_seed
        _vp, _i64,                      # out, ldo
        _i64, _vp, _vp, _i64,           # seg_len, seg_row, seg_begin, n_seg
        _vp, _vp, _i64,                 # long_row, long_seg_ptr, n_long
        _vp, _i64, _vp, _i64,           # mid_row, n_mid, task_row, n_task
        _vp, _vp, _u32, _vp,            # partial, stats, flags, stream
        _vp, _i64, _vp, _i64]),         # whh, ldwh, erh, ldeh (NULL: no staged tables)         # whh, ldwh, erh, ldeh
    "gnn_gat_backward_prep_f32": (ctypes.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp,
                                                 _vp]),
    "gnn_gat_backward_edges_f32": (ctypes.c_int, [
        _vp, _vp, _i64, _vp, _i64, _i64, _i64,      # rowptr, col, n_rows, wh, ldw, heads, fh
        _vp, _vp, _vp, _vp, _vp,                    # el, er, lse, dout, D
        ctypes.c_float, _i32, ctypes.c_float, ctypes.c_uint64,  # slope, mode, drop_p, seed
        _vp, _vp, _vp,                              # w_edge, ds_edge, del
        _i64, _vp, _vp, _i64, _vp, _vp, _i64,       # seg_len, seg_row, seg_begin, n_seg, long...
        _vp, _i64, _vp, _vp]),                      # rows, n_rows_list, del_part, stream
    "gnn_gat_backward_nodes_f32": (ctypes.c_int, [
        _vp, _vp, _vp, _i64, _i64, _i64,            # rowptr_t, src_t, eid_t, n, heads, fh
        _vp, _vp, _vp, _vp, _vp, _vp,               # dout, w_edge, ds_edge, del, a_src, a_dst
        _vp, _vp,                                   # dwh, der
        _i64, _vp, _vp, _i64, _vp, _vp, _i64,       # plan of the transposed graph
        _vp, _i64, _vp, _vp]),                      # rows, n_rows_list, part, stream
    "gnn_gat_backward_rows_f32": (ctypes.c_int, [
        _vp, _vp, _i64, _vp, _i64, _i64, _i64,      # rowptr, col, n_rows, wh, ldw, heads, fh
        _vp, _vp, _vp, _vp, _vp, _i64, _i32,        # el, er, lse, dy, y, ldo, elu
        ctypes.c_float, _i32, ctypes.c_float, ctypes.c_uint64,  # slope, mode, drop_p, seed
        _vp, _vp, _vp,                              # dout, nstat, del
        _i64, _vp, _vp, _i64, _vp, _vp, _i64,       # plan
        _vp, _i64, _vp, _i64, _vp, _vp, _vp]),      # rows, n, short_rows, n, del_part, a_dst,
                                                    # stream
    "gnn_gat_backward_rows_ex_f32": (ctypes.c_int, [
        _vp, _vp, _i64, _vp, _i64, _i64, _i64,
        _vp, _vp, _vp, _vp, _vp, _i64, _i32,
        ctypes.c_float, _i32, ctypes.c_float, ctypes.c_uint64,
        _vp, _vp, _vp,
        _i64, _vp, _vp, _i64, _vp, _vp, _i64,
        _vp, _i64, _vp, _i64, _vp, _vp,
        ctypes.c_float, ctypes.c_uint64, _vp]),     # ... a_dst, dy_drop_p, dy_drop_seed, stream
    "gnn_gat_backward_nodes_recompute_f32": (ctypes.c_int, [
        _vp, _vp, _vp, _i64, _i64, _i64,            # rowptr_t, src_t, eid_t, n, heads, fh
        _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,    # dout, nstat, wh, ldw, er, del, a_src, a_dst
        ctypes.c_float, _i32, ctypes.c_float, ctypes.c_uint64,  # slope, mode, drop_p, seed
        _vp, _vp,                                   # dwh, der
        _i64, _vp, _vp, _i64, _vp, _vp, _i64,       # plan of the transposed graph
        _vp, _i64, _vp, _i64, _vp, _vp]),           # rows, n, short_rows, n, part, stream
    "gnn_col_mean_scratch_bytes": (_i64, [_i64, _i64]),
    "gnn_col_mean_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "gnn_sage_aggregate_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i32, _vp, _i64,
                                              _vp]),
    "gnn_sage_gather_aggregate_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _i64,
                                                     _i32, _vp, _i64, _vp, _vp]),
    "gnn_gather_rows_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _vp]),
    "gnn_dropout_rows_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, ctypes.c_int32, _i64, _i64,
                                            ctypes.c_float, ctypes.c_uint64, _vp, _i64, _vp, _vp]),
    "gnn_sage_layer_supported": (ctypes.c_int, [_i64, _i64]),
    "gnn_sage_layer_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _i64,
                                          _i64, _i64, _vp, _i64, _vp, _i64, _vp, _vp]),
    "gnn_dev_spmm_variant_f32": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _i64,
                                                _i64, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp,
                                                _vp, _i64, _vp, _i64, _vp, _i32, _vp]),
    "gnn_gcn_adjacency_workspace_bytes": (_i64, [_i64, _i64]),
    "gnn_gcn_adjacency_build": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp, _i64,
                                               ctypes.POINTER(ctypes.c_int64), _vp]),
    "gnn_gcn_adjacency_fill": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "gnn_sample_neighbors": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, ctypes.c_uint64, _vp,
                                            _vp, _vp]),
    "gnn_frontier_workspace_bytes": (ctypes.c_int64, [_i64]),
    "gnn_frontier_build": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _vp]),
    "gnn_frontier_emit": (ctypes.c_int, [_i64, _vp, _vp, _vp]),
    "gnn_frontier_rank": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gnn_sample_layers_workspace_bytes": (ctypes.c_int64, [_i64]),
    "gnn_linear_small_supported": (ctypes.c_int, [_i64, _i64]),
    "gnn_linear_small_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "gnn_gemm_tn_supported": (ctypes.c_int, [_i64, _i64]),
    "gnn_gemm_tn_workspace_bytes": (_i64, [_i64, _i64, _i64]),
    "gnn_gemm_tn_masked_supported": (ctypes.c_int, [_i64, _i64]),
    "gnn_gemm_tn_masked_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, ctypes.c_float,
                                              _i64, _i64, _i64, _vp, _i64, _i32, _vp, _vp, _i64,
                                              _vp]),
    "gnn_gemm_tn_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _i64, _i32,
                                       _vp, _i64, _vp, _vp, _i64, _vp]),
    "gnn_sample_layers": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _vp, _i32, _vp,
                                         _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    # CPython-exact host sampler (pysample.cpp): host pointers, no stream
    "gnn_pyadj_build": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp, _vp]),
    "gnn_py_layer_sample": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _i32, _i64, _i32, _vp,
                                           ctypes.POINTER(_vp)]),
    "gnn_py_layer_result_shape": (ctypes.c_int, [_vp, _vp]),
    "gnn_py_layer_result_copy": (ctypes.c_int, [_vp, _vp, _vp]),
    "gnn_py_layer_result_free": (None, [_vp]),
    "gnn_pyset_order": (ctypes.c_int, [_vp, _i64, _vp, _vp]),
    "gnn_pyset_union_order": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp]),
}

EPI_RELU = 1
EPI_ELU = 2
EPI_ACCUMULATE = 4
EPI_SKIP_EMPTY = 8
E_ARG = -1
E_ALIGN = -2
E_UNSUPPORTED = -3


def library_path() -> Path:
    return _build.LIB_PATH


def load(build_if_missing: bool = False) -> ctypes.CDLL:
    """dlopen libgnn_mi355x.so and bind every C-ABI symbol (raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not path.exists():
            if not build_if_missing:
                raise RuntimeError(
                    f"{path} is missing: build it with `python -m graphneuralnetwork_amd.build` "
                    "(the MI355X aggregation ops have no CPU fallback)")
            _build.build()
        lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        check_stamp(lib)
        _lib = lib
        return lib


def build_stamp(lib=None) -> str:
    """The source stamp embedded in the loaded library (``gnn_build_stamp()``)."""
    return (lib or load()).gnn_build_stamp().decode()


def check_stamp(lib) -> None:
    """Refuse a library not built from this tree's sources: a stale
    prebuilt .so would otherwise run silently under a newer tree's tests and bench."""
    built, tree = lib.gnn_build_stamp().decode(), _build.lib_source_stamp()
    if built != tree:
        raise RuntimeError(
            f"{library_path()} was built from sources with stamp {built}, but this tree's are "
            f"{tree}: rebuild with `python -m graphneuralnetwork_amd.build`")
    if lib.gnn_build_defines().decode():
        raise RuntimeError(f"{library_path()} is a tuning-variant build "
                           f"({lib.gnn_build_defines().decode()}), not the product library")


def use_variant(path) -> ctypes.CDLL:
    """Kernel-tuning hook (tools/*_ab.py): route every op through another build
    of the same C-ABI (``build.build_variant``); ``use_variant(None)`` restores."""
    global _lib
    if path is None:
        _lib = None
        return load()
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_LOCAL)
    if not hasattr(lib, "gnn_build_stamp"):
        raise RuntimeError(f"{path}: no gnn_build_stamp (built before round 6); rebuild it")
    for name, (res, args) in SIGNATURES.items():
        try:  # an older build may lack entries added since (A/B of a previous tree)
            fn = getattr(lib, name)
        except AttributeError:
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def error_string(code: int) -> str:
    return load().gnn_error_string(int(code)).decode()


def check(code: int, what: str) -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed with code {code}: {error_string(code)}")


def ptr(t) -> int | None:
    """Device address of a tensor (None for an absent optional operand)."""
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
