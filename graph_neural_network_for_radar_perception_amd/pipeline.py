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


# the 16-bit conv's static schedule (small graphs) while forwards overlap: fewer waves per
# launch, so the launches of the in-flight forwards share the chip (C5, three in flight:
# 2048 -> 1536 waves, +8 %, profiles/r05_conv_waves_ab.log)
CONCURRENT_CONV_WAVES = 1536


class RadarGNNPipeline:
    def __init__(self, model, cfg, dtype: str = 'fp32', mode: int = nat.GRAPH_KNN,
                 eps2: Optional[float] = None, conv_waves: Optional[int] = None):
        """mode: nat.GRAPH_KNN (datagen_gnn.py:104-106, the default), nat.GRAPH_RADIUS (a pure
        ball-query graph, BASELINE config 5) or nat.GRAPH_KNN_RADIUS
        (compute_adjacency_information_v2); eps2: squared radius (default
        cfg.ball_query_eps_square); conv_waves: the built graphs' 16-bit conv wave count
        (DeviceGraph.conv_waves; None: DeviceGraph.CONV_WAVES)."""
        self.model = model
        self.conv_waves = conv_waves
        self.cfg = cfg
        self.dtype = dtype
        self.mode = mode
        self.eps2 = eps2
        self.plans = model.plans(dtype)
        self.ws_cache: dict = {}
        self.buffers: dict = {}

    def build(self, batch: FrameBatch) -> GraphBatch:
        gb = build_graph_batch(batch, self.cfg, eps2=self.eps2, mode=self.mode,
                               ws_cache=self.ws_cache)
        if self.conv_waves:
            gb.graph.conv_wave_count = self.conv_waves
        return gb

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
        graph built without a host sync outgrew its capacity: GraphBatch.check_capacity).  A
        concurrent pipeline's step is waited for first (GraphBatch.done)."""
        gb.check_capacity()
        U = int(gb.graph.n_pairs_dev.item())
        return out.node_cls, out.node_reg, out.link_cls[:U], out.obj_cls


class PipelinedSteps:
    """Two batches in flight: the graph build + features of step i run on a side stream while
    the GNN forward of step i - 1 runs on the caller's stream (the build's grid / selection
    kernels are latency-bound and need little LDS, so they fill the CUs the persistent forward
    kernels leave idle).  Every step still builds its own graph and runs the whole forward;
    results are those of ``RadarGNNPipeline.step`` bit for bit.

    ``depth`` pipelines (own workspaces and buffers: a build never overwrites arrays a forward
    in flight reads) are used round robin; pipeline p's build waits for its previous forward
    (an event), and its GraphBatch is kept alive until that point, so the caching allocator
    cannot hand the build stream memory the forward stream still reads.  The build also waits
    for the batch itself: ``FrameBatch.ready``, recorded on the stream that wrote its arrays
    (``from_frames`` records it after its uploads, asynchronous ones included; a batch without
    one makes the build wait for everything enqueued on the caller's stream so far), and the
    batch's arrays are marked as in use on the side stream (``record_stream``), so freeing the
    batch early cannot hand its memory to the caller's stream while the build reads it."""

    def __init__(self, model, cfg, dtype: str = 'fp32', mode: int = nat.GRAPH_KNN,
                 eps2: Optional[float] = None, depth: int = 2, concurrent: bool = False,
                 conv_waves: Optional[int] = None):
        """concurrent: each pipeline runs its build AND its forward on a stream of its own,
        so the forwards of consecutive steps overlap too (latency-bound single-frame steps:
        one 20 000-node frame leaves the persistent kernels a few tiles per wave); the
        caller's stream then waits for nothing -- the step's GraphBatch carries its completion
        event (``gb.done``; trim / check_capacity / edge_index wait on it, and
        ``gb.wait_ready()`` makes the current stream wait before reading an output).
        conv_waves: as RadarGNNPipeline's (default with concurrent: CONCURRENT_CONV_WAVES)."""
        if conv_waves is None and concurrent:
            conv_waves = CONCURRENT_CONV_WAVES
        self.pipes = [RadarGNNPipeline(model, cfg, dtype, mode=mode, eps2=eps2,
                                       conv_waves=conv_waves) for _ in range(depth)]
        self.depth = depth
        self.concurrent = concurrent
        self.streams = None
        self.done = [None] * depth
        self.last_done = None   # concurrent: the latest step's completion (wait on it to read)
        self.side = None
        self.ev_fwd = [None] * depth
        self.keep = [None] * depth
        self.i = 0

    def _step_concurrent(self, batch: FrameBatch, events=None):
        main = torch.cuda.current_stream()
        if self.streams is None:
            self.streams = [torch.cuda.Stream(device=main.device) for _ in range(self.depth)]
        p = self.i % self.depth
        self.i += 1
        st = self.streams[p]
        with torch.cuda.stream(st):
            # the pipeline's previous step ran on this same stream: its arrays are free
            if batch.ready is not None:
                st.wait_event(batch.ready)
            else:
                st.wait_stream(main)
            for t in batch.tensors():
                t.record_stream(st)
            gb = self.pipes[p].build(batch)
            out = self.pipes[p].forward(batch, gb, events)
            ev = torch.cuda.Event()
            ev.record(st)
        gb.done = ev          # trim / check_capacity / edge_index wait on it before reading
        self.done[p] = ev
        self.last_done = ev
        self.keep[p] = (gb, out)
        return gb, out

    def step(self, batch: FrameBatch, events=None):
        if self.concurrent:
            return self._step_concurrent(batch, events)
        main = torch.cuda.current_stream()
        if self.side is None:
            self.side = torch.cuda.Stream(device=main.device)
        p = self.i % self.depth
        self.i += 1
        with torch.cuda.stream(self.side):
            if self.ev_fwd[p] is not None:
                self.side.wait_event(self.ev_fwd[p])
            if batch.ready is not None:
                self.side.wait_event(batch.ready)
            else:
                self.side.wait_stream(main)
            for t in batch.tensors():
                t.record_stream(self.side)
            gb = self.pipes[p].build(batch)
            ev_b = torch.cuda.Event()
            ev_b.record(self.side)
        main.wait_event(ev_b)
        out = self.pipes[p].forward(batch, gb, events)
        ev_f = torch.cuda.Event()
        ev_f.record(main)
        self.ev_fwd[p] = ev_f
        self.keep[p] = (gb, out)
        return gb, out
