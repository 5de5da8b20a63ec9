"""ctypes binding of libradargnn.so -- the C ABI declared in include/radar_gnn.h.

The library is built in-tree (``build.py``) and loaded from
``graph_neural_network_for_radar_perception_amd/lib/libradargnn.so``.  There is
no fallback: if the library is missing or fails to load, every entry point
raises ``NativeLibraryError``.

Calls take ``torch.Tensor`` arguments only for convenience at this layer; they
are reduced to raw device pointers (``data_ptr()``) and sizes before crossing
the boundary, and every call is enqueued on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Optional

PKG = os.path.dirname(os.path.abspath(__file__))
# RG_LIBRARY overrides the in-tree library (kernel experiments: build.build_variant)
LIB_PATH = os.environ.get('RG_LIBRARY') or os.path.join(PKG, 'lib', 'libradargnn.so')
HEADER = os.path.join(os.path.dirname(PKG), 'include', 'radar_gnn.h')

RG_F32, RG_BF16, RG_F16, RG_F32X3 = 0, 1, 6, 7
RG_PACK_FAST_IN, RG_PACK_FAST_CHAIN, RG_PACK_FAST_UPD, RG_PACK_F32_FAST = 2, 3, 4, 5
RG_PACK_CENTERED = 0x100
RG_PACK_TRANSPOSE = 0x200
RG_PACK_X3 = 0x400
RG_PACK_F16 = 0x800
RG_LAYER_CENTERED = 1
RG_LAYER_F16 = 2
RG_ERR_UNSUPPORTED = 3
ACT = {'none': 0, 'relu': 1, 'leakyrelu': 2, 'swish': 3}
GRAPH_KNN, GRAPH_RADIUS, GRAPH_KNN_RADIUS = 0, 1, 2
REDUCE = {'add': 0, 'sum': 0, 'mean': 1, 'max': 2}
IN_DENSE, IN_CONCAT2, IN_GATHER3, IN_PAIRADD, IN_PAIRPRE = 0, 1, 2, 3, 4
MAX_LAYERS = 8


class NativeLibraryError(RuntimeError):
    pass


class rg_layer(ctypes.Structure):
    _fields_ = [('w_packed', ctypes.c_void_p), ('norm_mu', ctypes.c_void_p),
                ('norm_std', ctypes.c_void_p), ('in_dim', ctypes.c_int),
                ('out_dim', ctypes.c_int), ('act', ctypes.c_int), ('flags', ctypes.c_int),
                ('save_pre', ctypes.c_void_p), ('save_out', ctypes.c_void_p)]


class rg_pack_job(ctypes.Structure):
    _fields_ = [('weight', ctypes.c_void_p), ('bias', ctypes.c_void_p),
                ('packed', ctypes.c_void_p), ('in_dim', ctypes.c_int),
                ('out_dim', ctypes.c_int), ('fmt', ctypes.c_int), ('transpose', ctypes.c_int),
                ('ld', ctypes.c_int)]


class rg_loss_args(ctypes.Structure):
    _fields_ = [('node_cls', ctypes.c_void_p), ('node_reg', ctypes.c_void_p),
                ('link', ctypes.c_void_p), ('obj', ctypes.c_void_p),
                ('node_class', ctypes.c_void_p), ('node_offsets', ctypes.c_void_p),
                ('edge_class', ctypes.c_void_p), ('obj_class', ctypes.c_void_p),
                ('class_w', ctypes.c_void_p),
                ('n_nodes', ctypes.c_long), ('n_pairs', ctypes.c_long),
                ('n_clusters', ctypes.c_long), ('n_classes', ctypes.c_int),
                ('mu_x', ctypes.c_float), ('mu_y', ctypes.c_float),
                ('sigma_x', ctypes.c_float), ('sigma_y', ctypes.c_float),
                ('w_node_cls', ctypes.c_float), ('w_node_reg', ctypes.c_float),
                ('w_edge_cls', ctypes.c_float), ('w_obj_cls', ctypes.c_float)]


LR_MILESTONES_MAX = 16


class rg_lr_schedule(ctypes.Structure):
    _fields_ = [('n_milestones', ctypes.c_int),
                ('milestones', ctypes.c_int * LR_MILESTONES_MAX),
                ('lr', ctypes.c_double * (LR_MILESTONES_MAX + 1))]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_S = ctypes.c_size_t
_D = ctypes.c_double
_F = ctypes.c_float

_SIGNATURES = {
    'rg_last_error': (ctypes.c_char_p, []),
    'rg_version': (_I, []),
    'rg_build_graph_workspace_size': (_S, [_I, _I, _I, _I, _I]),
    'rg_build_graph': (_I, [_P, _P, _P, _I, _I, _I, _I, _F, _I, _P, _P, _L, _P, _P, _P, _S, _P]),
    'rg_node_features': (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _D, _D, _D, _D, _P, _P]),
    'rg_edge_features': (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _L, _P, _P]),
    'rg_node_features_f64': (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _D, _D, _D, _D, _P, _P]),
    'rg_edge_features_f64': (_I, [_P, _P, _P, _P, _P, _P, _P, _L, _P, _P]),
    'rg_dense_pair_rows_workspace_size': (_S, [_I]),
    'rg_dense_pair_rows': (_I, [_P, _I, _P, _P, _P, _S, _P]),
    'rg_dense_pair_emit': (_I, [_P, _I, _P, _P, _P, _P]),
    'rg_pair_add_rows_f32': (_I, [_P, _I, _I, _P, _P, _L, _P, _I, _P]),
    'rg_pack_kinematics': (_I, [_P, _P, _P, _P, _I, _P, _P]),
    'rg_edge_features_packed': (_I, [_P, _P, _P, _P, _P, _L, _P, _P]),
    'rg_link_pairs_workspace_size': (_S, [_I]),
    'rg_link_pairs': (_I, [_P, _P, _I, _P, _P, _P, _L, _P, _P, _S, _P]),
    'rg_pairs_from_edge_index_workspace_size': (_S, [_L]),
    'rg_pairs_from_edge_index': (_I, [_P, _L, _P, _P, _P, _P, _S, _P]),
    'rg_csr_rows': (_I, [_P, _I, _P, _P]),
    'rg_csr_clamp': (_I, [_P, _I, _P, _L, _P, _P]),
    # real-data front-end (frontend.hip)
    'rg_frontend_sync': (_I, [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _F, _I, _P, _P, _P, _P,
                              _P, _P]),
    'rg_frontend_gate_lists': (_I, [_P, _P, _I, _P, _P, _P]),
    'rg_ransac_consensus_sets': (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    'rg_frontend_ransac': (_I, [_P, _P, _P, _I, _P, _P, _P, _I, _I, _D, _I, _D, _P, _P, _P, _P]),
    'rg_frontend_labels_workspace_size': (_S, [_I]),
    'rg_frontend_labels': (_I, [_P, _I, _P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _P, _S, _P]),
    'rg_frontend_select_workspace_size': (_S, [_I]),
    'rg_frontend_select': (_I, [_P, _P, _P, _I, _F, _F, _F, _F, _F, _P, _I, _P, _P, _P, _P, _S,
                                _P]),
    'rg_proposal_centres': (_I, [_P, _I, _P, _I, _I, _F, _F, _F, _F, _P, _P, _P]),
    'rg_cluster_radius_workspace_size': (_S, [_I, _I, _I]),
    'rg_cluster_radius': (_I, [_P, _P, _P, _I, _I, _I, _F, _P, _P, _S, _P]),
    'rg_cluster_pairs': (_I, [_P, _P, _P, _P, _P, _L, _P, _I, _F, _I, _P, _P]),
    'rg_cluster_lists_workspace_size': (_S, [_I]),
    'rg_cluster_lists': (_I, [_P, _I, _P, _P, _P, _P, _P, _S, _P]),
    'rg_csr_by_dst_workspace_size': (_S, [_I, _L]),
    'rg_csr_by_dst': (_I, [_P, _L, _I, _P, _P, _P, _P, _S, _P]),
    'rg_dense_adjacency': (_I, [_P, _P, _P, _P, _I, _P, _P, _P]),
    'rg_i32_to_i64': (_I, [_P, _L, _P, _P]),
    'rg_gather_rows_f32': (_I, [_P, _P, _L, _I, _P, _P]),
    'rg_packed_linear_bytes': (_S, [_I, _I, _I]),
    'rg_pack_linear': (_I, [_P, _P, _I, _I, _I, _P, _P]),
    'rg_pack_linear_jobs': (_I, [_P, _I, _P]),
    'rg_pack_linear_ld': (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    'rg_mlp_chain': (_I, [_I, ctypes.POINTER(rg_layer), _I, _L, _P, _I, _I, _P, _I, _I, _P, _I,
                          _I, _P, _I, _I, _P, _P, _P, _I, _I, _P, _I, _I, _P]),
    'rg_mlp_chain_fast': (_I, [ctypes.POINTER(rg_layer), _I, _L, _P, _I, _I, _P, _I, _I, _P, _I,
                               _I, _P, _I, _I, _P, _P, _P, _I, _I, _P, _I, _I, _P]),
    'rg_mlp_chain_f32': (_I, [ctypes.POINTER(rg_layer), _I, _L, _P, _I, _P, _I, _I, _P, _P, _P,
                              _I, _P]),
    'rg_mlp_chain_f32_ex': (_I, [ctypes.POINTER(rg_layer), _I, _L, _P, _I, _P, _I, _I, _P, _I, _I,
                                 _P, _I, _I, _P, _P, _P, _I, _P, _I, _P]),
    'rg_mlp_chain_x3': (_I, [ctypes.POINTER(rg_layer), _I, _L, _P, _I, _P, _I, _I, _P, _P, _P,
                             _I, _P]),
    'rg_conv_layer_f32_workspace_size': (_S, [_I]),
    'rg_conv_layer_f32': (_I, [ctypes.POINTER(rg_layer), _I, _P, _I, _P, _I, _P, _P, _P, _I, _P,
                               _I, _P, _S, _P]),
    'rg_conv_layer_x3_workspace_size': (_S, [_I]),
    'rg_conv_layer_x3': (_I, [ctypes.POINTER(rg_layer), ctypes.POINTER(rg_layer), _I, _P, _I, _P,
                              _I, _P, _P, _P, _P, _I, _P, _I, _P, _P, _S, _P]),
    'rg_conv_layer_x3_blocks': (_I, [ctypes.POINTER(rg_layer), ctypes.POINTER(rg_layer), _I, _P,
                                     _I, _P, _I, _P, _P, _P, _P, _I, _P, _I, _P, _P, _P, _S, _P]),
    'rg_conv_x3_blocks_bytes': (_S, [_I]),
    'rg_conv_x3_blocks': (_I, [_P, _I, _P, _P]),
    'rg_conv_proj_x3': (_I, [ctypes.POINTER(rg_layer), _P, _I, _I, _P, _P]),
    'rg_conv_layer_workspace_size': (_S, []),
    'rg_conv_layer_fused': (_I, [ctypes.POINTER(rg_layer), ctypes.POINTER(rg_layer), _I, _P, _I,
                                 _P, _I, _P, _P, _P, _I, _P, _I, _P, _P]),
    'rg_conv_layer_fused_blocks': (_I, [ctypes.POINTER(rg_layer), ctypes.POINTER(rg_layer), _I,
                                        _P, _I, _P, _I, _P, _P, _P, _I, _P, _I, _P, _P, _P, _P]),
    'rg_conv_blocks_workspace_size': (_S, [_I]),
    'rg_conv_blocks': (_I, [_P, _I, _P, _P, _P, _S, _P]),
    'rg_conv_wave_nodes': (_I, [_P, _I, _I, _P, _P]),
    'rg_conv_layer_fused_waves': (_I, [ctypes.POINTER(rg_layer), ctypes.POINTER(rg_layer), _I, _P,
                                       _I, _P, _I, _P, _P, _P, _I, _P, _I, _P, _I, _P, _P]),
    'rg_cluster_majority_label': (_I, [_P, _P, _P, _I, _I, _P, _P, _P]),
    'rg_cross_entropy': (_I, [_P, _I, _P, _I, _I, _P, _P, _P]),
    'rg_cross_entropy_backward': (_I, [_P, _I, _P, _I, _I, _P, _P, _I, _P]),
    'rg_frame_norm_workspace_size': (_S, [_I, _I]),
    'rg_frame_norm': (_I, [_P, _I, _I, _I, _P, _I, _P, _P, _I, _P, _I, _P, _I, _P, _S, _P]),
    'rg_frame_norm_backward_workspace_size': (_S, [_I, _I]),
    'rg_frame_norm_backward': (_I, [_P, _I, _P, _I, _I, _I, _P, _I, _P, _P, _I, _P, _I, _P, _P,
                                    _P, _S, _P]),
    'rg_gather_i32': (_I, [_P, _P, _I, _P, _P]),
    'rg_lower_bound_i32': (_I, [_P, _P, _L, _P, _I, _P, _P]),
    'rg_segment_reduce': (_I, [_P, _I, _I, _P, _P, _I, _I, _I, _P, _I, _I, _P]),
    'rg_segment_order_workspace_size': (_S, []),
    'rg_segment_order': (_I, [_P, _I, _P, _P, _S, _P]),
    'rg_segment_reduce_ordered': (_I, [_P, _I, _I, _P, _P, _I, _I, _I, _P, _I, _I, _P]),
    'rg_segment_reduce_sched': (_I, [_P, _I, _I, _P, _P, _I, _I, _I, _P, _I, _I, _I, _I, _I, _P]),
    'rg_segment_reduce_ranges_workspace_size': (_S, [_L, _I, _I]),
    'rg_segment_reduce_ranges': (_I, [_P, _I, _I, _L, _P, _P, _I, _I, _I, _P, _I, _I, _P, _S,
                                      _P]),
    # classifier GNN graph build (classifier.hip)
    'rg_object_graph_workspace_size': (_S, [_I]),
    'rg_object_complete_graph': (_I, [_P, _I, _I, _L, _P, _P, _P, _P, _S, _P]),
    'rg_object_row_ranges': (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _S, _P]),
    'rg_object_focal_loss': (_I, [_P, _I, _P, _I, _I, _P, _P]),
    'rg_object_focal_loss_backward': (_I, [_P, _I, _P, _I, _I, _P, _P, _I, _P]),
    'rg_range_max_backward': (_I, [_P, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P]),
    'rg_segment_amax_backward': (_I, [_P, _I, _I, _P, _I, _P, _I, _P, _I, _P]),
    # training (train.hip)
    'rg_ffn_backward_workspace_size': (_S, []),
    'rg_ffn_backward': (_I, [_P, _I, _P, _I, _L, _I, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P]),
    'rg_dx_norm_backward_workspace_size': (_S, [_L]),
    'rg_dx_norm_backward': (_I, [_P, _L, _P, _I, _P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _S, _P]),
    'rg_ffn_backward_gather': (_I, [_P, _I, _P, _I, _P, _P, _L, _I, _I, _P, _P, _I, _P, _I, _P, _P,
                                    _P, _P]),
    'rg_linear_grad_workspace_size': (_S, [_L, _I, _I]),
    'rg_linear_grad': (_I, [_P, _I, _L, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _I, _I, _P, _P,
                            _P, _P, _P, _S, _P]),
    'rg_linear_grad_ld': (_I, [_P, _I, _L, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _I, _I, _P, _P,
                               _P, _I, _P, _P, _S, _P]),
    'rg_incidence_workspace_size': (_S, [_I, _L]),
    'rg_incidence': (_I, [_P, _P, _L, _I, _P, _P, _P, _S, _P]),
    'rg_gather_segment_sum': (_I, [_P, _I, _I, _I, _P, _P, _P, _I, _P, _I, _I, _P]),
    'rg_segment_max_backward': (_I, [_P, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P]),
    'rg_loss_workspace_size': (_S, [_L, _L, _L]),
    'rg_loss_graph': (_I, [ctypes.POINTER(rg_loss_args), _P, _P, _P, _S, _P]),
    'rg_loss_graph_backward': (_I, [ctypes.POINTER(rg_loss_args), _P, _P, _P, _P, _P, _P]),
    'rg_sgd_step': (_I, [_P, _P, _P, _L, _F, _F, _F, _I, _F, _P]),
    'rg_clock_probe': (_I, [_I, _I, _P, _P, ctypes.POINTER(_I), _P]),
    'rg_sgd_step_sched': (_I, [_P, _P, _P, _L, ctypes.POINTER(rg_lr_schedule), _F, _F, _F, _P, _I,
                               _P, _I, _P]),
    'rg_adamw_step_sched': (_I, [_P, _P, _P, _P, _L, ctypes.POINTER(rg_lr_schedule), _D, _D, _D,
                                 _D, _F, _P, _I, _P, _I, _P]),
}

_lib = None
_load_error: Optional[str] = None


def header_functions() -> list:
    """Names of every function declared in include/radar_gnn.h."""
    with open(HEADER) as fh:
        text = fh.read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(rg_[a-z0-9_]+)\s*\(', text)))


def lib():
    """The loaded library; raises NativeLibraryError when it is absent."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise NativeLibraryError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f'{LIB_PATH} not built: run `python -m '
                       'graph_neural_network_for_radar_perception_amd.build` (hipcc, gfx950)')
        raise NativeLibraryError(_load_error)
    try:
        handle = ctypes.CDLL(LIB_PATH)
    except OSError as exc:  # pragma: no cover - environment dependent
        _load_error = f'cannot load {LIB_PATH}: {exc}'
        raise NativeLibraryError(_load_error) from exc
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().rg_last_error().decode(errors='replace')
        raise RuntimeError(f'{what} failed (code {rc}): {msg}')


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> Optional[int]:
    """Raw device pointer of a tensor (None stays None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()
