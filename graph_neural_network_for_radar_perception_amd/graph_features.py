"""Graph build on the GPU with the reference's graph_features API.

Drop-in functions (same names, arguments and result keys as
``modules/compute_features/graph_features.py``) that run on the HIP library:

  compute_adjacency_information(data_dict, eps, knn)     graph_features.py:58-84
  compute_adjacency_information_v2(data_dict, eps, knn)  graph_features.py:87-114
  compute_node_features(data_dict, node_degree, ...)     graph_features.py:117-144
  compute_edge_features(data_dict, adj_list)             graph_features.py:147-164

They take and return numpy arrays like the reference (one host round trip per
call) with the reference's dtypes: int64 indices, bool adjacency, float32 distances,
and float64 node / edge features computed on the device exactly as numpy does
(graph_features.py:144,164; the tensorization ``datagen_gnn.py:120-124`` then casts them
to float32, which the batched device path below produces directly).  The batched device-side entry
point for many frames is ``FrameBatch`` + ``build_graph_batch`` below, which
keeps everything in HBM and never materialises an N x N matrix.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import _native as nat
from . import engine

_FIELDS_F32 = ('meas_px', 'meas_py', 'meas_vx', 'meas_vy', 'meas_vr', 'meas_rcs')


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError('graph_features: the HIP graph builder needs a GPU (no CPU fallback)')
    return torch.device('cuda', torch.cuda.current_device())


def _upload(frame: dict, dev, keys=None):
    out = {}
    for k in keys or (_FIELDS_F32 + ('meas_timestamp',)):
        if k not in frame:
            continue
        a = np.asarray(frame[k])
        a = a.astype(np.int64) if k == 'meas_timestamp' else a.astype(np.float32)
        out[k] = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return out


def _adjacency(data_dict, eps, knn, mode):
    dev = _device()
    d = _upload(data_dict, dev, ('meas_px', 'meas_py'))
    n = int(d['meas_px'].shape[0])
    fp = torch.tensor([0, n], dtype=torch.int32, device=dev)
    row_ptr, col, deg, ne, cap = engine.build_graph(d['meas_px'], d['meas_py'], fp, [n], knn,
                                                    eps, mode)
    E = int(ne.item())
    if E > cap:  # radius graphs: capacity is a guess; rebuild at the exact size
        row_ptr, col, deg, ne, cap = engine.build_graph(d['meas_px'], d['meas_py'], fp, [n], knn,
                                                        eps, mode, edge_capacity=E)
    rows = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
    lib = nat.lib()
    st = nat.stream_ptr(dev)
    nat.check(lib.rg_csr_rows(row_ptr.data_ptr(), n, rows.data_ptr(), st), 'rg_csr_rows')
    adj = torch.empty((n, n), dtype=torch.uint8, device=dev)
    dist = torch.empty((n, n), dtype=torch.float32, device=dev)
    if n > 0:
        nat.check(lib.rg_dense_adjacency(d['meas_px'].data_ptr(), d['meas_py'].data_ptr(),
                                         row_ptr.data_ptr(), col.data_ptr(), n, adj.data_ptr(),
                                         dist.data_ptr(), st), 'rg_dense_adjacency')
    adj_list = torch.stack((rows[:E], col[:E]), 0).to(torch.int64)
    return {'adj_matrix': adj.bool().cpu().numpy(),
            'distance_mat': dist.cpu().numpy(),
            'adj_list': adj_list.cpu().numpy(),
            'degree': deg[:n].to(torch.int64).cpu().numpy()}


def compute_adjacency_information(data_dict: dict, eps: float, knn: int) -> dict:
    """graph_features.py:58-84 on the GPU (kNN adjacency; ties -> lower index)."""
    return _adjacency(data_dict, eps, knn, nat.GRAPH_KNN)


def compute_adjacency_information_v2(data_dict: dict, eps: float, knn: int) -> dict:
    """graph_features.py:87-114 on the GPU (kNN union ball-query adjacency)."""
    return _adjacency(data_dict, eps, knn, nat.GRAPH_KNN_RADIUS)


def compute_radius_graph(data_dict: dict, eps: float) -> dict:
    """np.where(compute_ball_query(D, eps)) -- the pure radius graph of BASELINE config 5."""
    return _adjacency(data_dict, eps, 0, nat.GRAPH_RADIUS)


def compute_node_features(data_dict, node_degree, include_region_confidence=False,
                          min_range=None, max_range=None, min_azimuth=None, max_azimuth=None):
    """graph_features.py:117-144 on the GPU: float64 [N, 6] (or [N, 4] without the region
    confidences), like the reference's np.stack."""
    dev = _device()
    d = _upload(data_dict, dev)
    n = int(d['meas_px'].shape[0])
    deg = torch.from_numpy(np.asarray(node_degree).astype(np.int32)).to(dev)
    fp = torch.tensor([0, n], dtype=torch.int32, device=dev)

    class _C:  # range / azimuth limits as the kernel takes them
        grid_min_r = 0.0 if min_range is None else float(min_range)
        grid_max_r = 1.0 if max_range is None else float(max_range)
        grid_min_th = 0.0 if min_azimuth is None else float(min_azimuth)
        grid_max_th = 1.0 if max_azimuth is None else float(max_azimuth)

    out = torch.empty((n, 6), dtype=torch.float64, device=dev)
    nat.check(nat.lib().rg_node_features_f64(
        d['meas_px'].data_ptr(), d['meas_py'].data_ptr(), d['meas_vr'].data_ptr(),
        d['meas_rcs'].data_ptr(), d['meas_timestamp'].data_ptr(), deg.data_ptr(), fp.data_ptr(),
        n, 1, _C.grid_min_r, _C.grid_max_r, _C.grid_min_th, _C.grid_max_th, out.data_ptr(),
        nat.stream_ptr(dev)), 'rg_node_features_f64')
    out = out if include_region_confidence else out[:, :4]
    return out.cpu().numpy()


def compute_edge_features(data_dict, adj_list):
    """graph_features.py:147-164 on the GPU: float64 [E, 7] in the edge order of adj_list,
    like the reference's np.stack (dt is a float64 product there)."""
    dev = _device()
    d = _upload(data_dict, dev)
    al = torch.from_numpy(np.asarray(adj_list).astype(np.int32)).to(dev)
    E = int(al.shape[1])
    src = al[0].contiguous()
    dst = al[1].contiguous()
    out = torch.empty((E, 7), dtype=torch.float64, device=dev)
    nat.check(nat.lib().rg_edge_features_f64(
        d['meas_px'].data_ptr(), d['meas_py'].data_ptr(), d['meas_vx'].data_ptr(),
        d['meas_vy'].data_ptr(), d['meas_timestamp'].data_ptr(), src.data_ptr(), dst.data_ptr(),
        E, out.data_ptr(), nat.stream_ptr(dev)), 'rg_edge_features_f64')
    return out.cpu().numpy()


# --------------------------------------------------------------------------- batched device API
@dataclass
class FrameBatch:
    """A batch of radar frames resident in HBM (disjoint union, frame_ptr offsets)."""
    arrays: dict                  # meas_* -> device tensors [N]
    frame_ptr: torch.Tensor       # int32 [B+1] on device
    frame_sizes: List[int]        # host copy of the frame sizes
    cluster_ptr: torch.Tensor     # int32 [Ncl+1] object-head clusters (global node ids)
    cluster_idx: torch.Tensor     # int32 [sum |c|]
    n_clusters: int
    # recorded on the producing stream once every array above is written (uploads, or device
    # ops of the caller): consumers on other streams wait on it (pipeline.PipelinedSteps)
    ready: Optional['torch.cuda.Event'] = None

    def tensors(self) -> List[torch.Tensor]:
        return list(self.arrays.values()) + [self.frame_ptr, self.cluster_ptr, self.cluster_idx]

    def mark_ready(self, stream=None) -> 'FrameBatch':
        """Record ``ready`` on ``stream`` (default: the current stream) after the caller's
        last write to the batch's arrays."""
        if self.frame_ptr.is_cuda:
            self.ready = torch.cuda.Event()
            self.ready.record(stream if stream is not None else torch.cuda.current_stream())
        return self

    @property
    def n_nodes(self) -> int:
        return int(sum(self.frame_sizes))

    @property
    def n_frames(self) -> int:
        return len(self.frame_sizes)

    @staticmethod
    def from_frames(frames: List[dict], clusters: Optional[List[List[np.ndarray]]] = None,
                    device=None, pinned: bool = False) -> 'FrameBatch':
        """Upload frames (and the object-head clusters) as one batch.  ``pinned``: stage the
        host arrays in page-locked memory and copy them asynchronously on the current stream
        (the ``ready`` event, recorded after the copies, orders every consumer)."""
        dev = torch.device(device) if device is not None else _device()
        async_up = pinned and dev.type == 'cuda'

        def up(a: np.ndarray) -> torch.Tensor:
            t = torch.from_numpy(np.ascontiguousarray(a))
            if async_up:
                return t.pin_memory().to(dev, non_blocking=True)
            return t.to(dev)

        sizes = [int(np.asarray(f['meas_px']).shape[0]) for f in frames]
        cat = {}
        for k in _FIELDS_F32 + ('meas_timestamp',):
            dt = np.int64 if k == 'meas_timestamp' else np.float32
            cat[k] = up(np.concatenate([np.asarray(f[k]).astype(dt) for f in frames]))
        base = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        fp = up(base.astype(np.int32))
        lens, idx = [], []
        if clusters is not None:
            for b, cl in zip(base[:-1], clusters):
                for c in cl:
                    lens.append(len(c))
                    idx.append(np.asarray(c, dtype=np.int64) + b)
        cptr = up(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32))
        cidx = up((np.concatenate(idx) if idx else np.zeros(1)).astype(np.int32))
        return FrameBatch(cat, fp, sizes, cptr, cidx, len(lens)).mark_ready()


@dataclass
class GraphBatch:
    row_ptr: torch.Tensor        # int32 [N+1] CSR of the symmetric adjacency
    col: torch.Tensor            # int32 [cap]
    ball_degree: torch.Tensor    # int32 [N]
    n_edges_dev: torch.Tensor    # int32 [1]
    capacity: int
    graph: engine.DeviceGraph    # destination-major view + link pairs
    node_features: torch.Tensor  # float32 [N, 6]
    edge_features: torch.Tensor  # float32 [cap, 7], destination-major order
    # radius graphs built into an unchecked capacity: (pinned host int32[1] = the true edge
    # count, written by rg_csr_clamp itself; the event after it); None when the capacity was
    # checked on the host (or is exact, kNN)
    need: Optional[tuple] = None
    # the completion event of the step that built this graph and ran its forward on a stream
    # of its own (PipelinedSteps(concurrent=True)); readers wait on it (wait_ready)
    done: Optional[object] = None

    def wait_ready(self):
        """Make the caller's current stream wait for this graph's step (concurrent pipelines
        write the graph and the outputs on a private stream)."""
        if self.done is not None:
            torch.cuda.current_stream(self.row_ptr.device).wait_event(self.done)

    def check_capacity(self):
        """Raise if this graph was cut to its capacity (a radius graph built without a host
        sync whose edges outgrew the capacity that sufficed before): every output computed
        from it is invalid.  Host sync."""
        self.wait_ready()
        if self.need is not None:
            host, ev = self.need
            ev.synchronize()
            need = int(host[0])
            if need > self.capacity:
                raise RuntimeError(f'radius graph needed {need} edges but was built into a '
                                   f'capacity of {self.capacity}; this step\'s outputs are '
                                   f'invalid (the next build uses a larger capacity)')

    def edge_index(self) -> torch.Tensor:
        """int64 [2, E] in the reference's np.where order (host sync for E)."""
        self.check_capacity()
        E = int(self.n_edges_dev.item())
        return torch.stack((self.graph.dst[:E], self.col[:E]), 0).to(torch.int64)


def build_graph_batch(batch: FrameBatch, cfg, k: Optional[int] = None, eps2: Optional[float] = None,
                      mode: int = nat.GRAPH_KNN, ws_cache: Optional[dict] = None) -> GraphBatch:
    """datagen_gnn.py:104-124 for a whole batch, on the device and without host syncs:
    adjacency (rg_build_graph), node features, destination-major edge features,
    link pairs."""
    k = cfg.k_number_nearest_points if k is None else k
    eps2 = cfg.ball_query_eps_square if eps2 is None else eps2
    # radius graphs have no a-priori edge bound.  First build (nothing cached): built,
    # checked with one host sync and rebuilt if short.  Later builds use the cached
    # capacity WITHOUT a host sync: rg_csr_clamp keeps an overflowing graph in bounds and
    # writes the true edge count straight into pinned host memory (no copy launch; an event
    # marks it landed), checked at the next build -- a short capacity grows there -- and by
    # GraphBatch.check_capacity() (called by edge_index() / RadarGNNPipeline.trim()).
    cap_key = ('radius_cap', mode, float(eps2))
    pend_key = ('radius_need', mode, float(eps2))
    cap0 = ws_cache.get(cap_key) if (ws_cache is not None and mode != nat.GRAPH_KNN) else None
    if cap0 is not None:
        # every earlier build's count that has landed grows the capacity (the largest
        # one); counts still in flight stay queued, so a host running ahead of the GPU
        # loses none of them
        pend = ws_cache.get(pend_key, [])
        landed = [h for h, ev in pend if ev.query()]
        if landed:
            need = max(int(h[0]) for h in landed)
            if need > cap0:
                cap0 = need + need // 4
                ws_cache[cap_key] = cap0
            ws_cache[pend_key] = [(h, ev) for h, ev in pend if not any(h is x for x in landed)]
    row_ptr, col, deg, ne, cap = engine.build_graph(batch.arrays['meas_px'],
                                                    batch.arrays['meas_py'], batch.frame_ptr,
                                                    batch.frame_sizes, k, eps2, mode,
                                                    edge_capacity=cap0, ws_cache=ws_cache)
    need = None
    if mode != nat.GRAPH_KNN and cap0 is None:
        E = int(ne.item())
        if E > cap:
            row_ptr, col, deg, ne, cap = engine.build_graph(
                batch.arrays['meas_px'], batch.arrays['meas_py'], batch.frame_ptr,
                batch.frame_sizes, k, eps2, mode, edge_capacity=E, ws_cache=ws_cache)
        if ws_cache is not None:
            ws_cache[cap_key] = cap
    elif mode != nat.GRAPH_KNN:
        # pinned host memory is mapped into the device's address space: the clamp kernel
        # stores the count there directly
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        nat.check(nat.lib().rg_csr_clamp(row_ptr.data_ptr(), batch.n_nodes, ne.data_ptr(), cap,
                                         host.data_ptr(), nat.stream_ptr(row_ptr.device)),
                  'rg_csr_clamp')
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(row_ptr.device))
        ws_cache.setdefault(pend_key, []).append((host, ev))
        need = (host, ev)
    g = engine.graph_from_csr(row_ptr, col, batch.n_nodes, ne, cap)
    g.set_frames(batch.frame_ptr, batch.n_frames)
    nf = engine.node_features(batch.arrays, deg, batch.frame_ptr, batch.n_frames, cfg)
    # destination-major edge (src = g.src[p] -> dst = g.dst[p])
    ef = engine.edge_features(batch.arrays, g.src, g.dst, ne, cap)
    return GraphBatch(row_ptr, col, deg, ne, cap, g, nf, ef, need)
