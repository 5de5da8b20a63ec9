"""End-to-end batched hot path: raw radar measurements in HBM -> graph build ->
input features -> GNN forward -> four task heads, on one GPU.

One ``step`` = ``datagen_gnn.py:104-124`` (graph + features) for every frame of
the batch followed by ``Model_Inference.forward`` (gnn_detector.py:141-201) over
the batch, with no host synchronisation inside: capacities are exact upper
bounds for kNN graphs, and a radius graph syncs once, on its first build, then
reuses that capacity behind a device-side guard (rg_csr_clamp; checked lazily,
GraphBatch.check_capacity).  A step can be timed with HIP events.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native as nat
from . import engine
from .graph_features import FrameBatch, GraphBatch, build_graph_batch


class RadarGNNPipeline:
    def __init__(self, model, cfg, dtype: str = 'fp32', mode: int = nat.GRAPH_KNN,
                 eps2: Optional[float] = None):
        """mode: nat.GRAPH_KNN (datagen_gnn.py:104-106, the default), nat.GRAPH_RADIUS (a pure
        ball-query graph, BASELINE config 5) or nat.GRAPH_KNN_RADIUS
        (compute_adjacency_information_v2); eps2: squared radius (default
        cfg.ball_query_eps_square)."""
        self.model = model
        self.cfg = cfg
        self.dtype = dtype
        self.mode = mode
        self.eps2 = eps2
        self.plans = model.plans(dtype)
        self.ws_cache: dict = {}
        self.buffers: dict = {}

    def build(self, batch: FrameBatch) -> GraphBatch:
        return build_graph_batch(batch, self.cfg, eps2=self.eps2, mode=self.mode,
                                 ws_cache=self.ws_cache)

    def forward(self, batch: FrameBatch, gb: GraphBatch, events=None) -> engine.ForwardOutputs:
        return engine.forward_batched(self.plans, gb.node_features, gb.edge_features, gb.graph,
                                      batch.cluster_ptr, batch.cluster_idx, batch.n_clusters,
                                      n_pairs_cap=gb.capacity // 2 + 1, buffers=self.buffers,
                                      events=events)

    def step(self, batch: FrameBatch, events=None):
        gb = self.build(batch)
        return gb, self.forward(batch, gb, events)

    @staticmethod
    def trim(gb: GraphBatch, out: engine.ForwardOutputs):
        """Host-synchronising view of the outputs at their true sizes (raises if a radius
        graph built without a host sync outgrew its capacity: GraphBatch.check_capacity)."""
        gb.check_capacity()
        U = int(gb.graph.n_pairs_dev.item())
        return out.node_cls, out.node_reg, out.link_cls[:U], out.obj_cls
