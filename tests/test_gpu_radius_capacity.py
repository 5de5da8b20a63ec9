"""The sync-free radius graph build (graph_features.build_graph_batch after the first
build): the capacity that sufficed is reused without a host sync behind rg_csr_clamp.
Checked: repeated steps are bit-identical to the first (synchronised) one; an artificially
short capacity leaves a memory-safe, truncated CSR, is reported by check_capacity() /
trim(), and the next build grows the capacity and is exact again."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pipe(dev, n=4000, eps2=2.5):
    from graph_neural_network_for_radar_perception_amd import _native as nat, synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    cfg = default_config()
    torch.manual_seed(7)
    pred = Model_Training(cfg, 'cpu').to(dev).pred.eval().requires_grad_(False)
    frames = [synthetic.make_frame(n, synthetic.SEED0 + i) for i in range(2)]
    clusters = [synthetic.cluster_lists(n) for _ in range(2)]
    batch = FrameBatch.from_frames(frames, clusters, device=dev)
    return RadarGNNPipeline(pred, cfg, 'fp16', mode=nat.GRAPH_RADIUS, eps2=eps2), batch


def _host(gb, out):
    E = int(gb.n_edges_dev.item())
    return (gb.row_ptr.cpu().numpy(), gb.col[:E].cpu().numpy(),
            [t.float().cpu().numpy() for t in (out.node_cls, out.node_reg, out.obj_cls)])


def test_radius_steps_without_sync_match_first(cuda_device):
    pipe, batch = _pipe(cuda_device)
    with torch.no_grad():
        gb0, out0 = pipe.step(batch)            # first build: host-checked capacity
        assert gb0.need is None
        ref = _host(gb0, out0)
        for _ in range(3):
            gb, out = pipe.step(batch)          # cached capacity, device guard
            assert gb.need is not None
            gb.check_capacity()
            got = _host(gb, out)
            np.testing.assert_array_equal(got[0], ref[0])
            np.testing.assert_array_equal(got[1], ref[1])
            for a, b in zip(got[2], ref[2]):
                np.testing.assert_array_equal(a, b)


def test_radius_short_capacity_is_guarded_then_grows(cuda_device):
    pipe, batch = _pipe(cuda_device)
    with torch.no_grad():
        gb0, out0 = pipe.step(batch)
        E = int(gb0.n_edges_dev.item())
        ref = _host(gb0, out0)
        key = [k for k in pipe.ws_cache if isinstance(k, tuple) and k[0] == 'radius_cap'][0]
        short = E // 2
        pipe.ws_cache[key] = short
        gb, out = pipe.step(batch)              # overflows: cut, not out of bounds
        torch.cuda.synchronize()
        assert int(gb.need[0][0]) == E  # written by the clamp kernel into pinned memory
        rp = gb.row_ptr.cpu().numpy()
        ne = int(gb.n_edges_dev.item())
        assert ne <= short // 2 and rp[-1] == ne and np.all(np.diff(rp) >= 0)
        assert int(gb.graph.n_pairs_dev.item()) <= gb.capacity // 2 + 1
        with pytest.raises(RuntimeError, match='capacity'):
            gb.check_capacity()
        with pytest.raises(RuntimeError, match='capacity'):
            pipe.trim(gb, out)
        gb2, out2 = pipe.step(batch)            # the landed count grows the capacity
        assert gb2.capacity >= E
        gb2.check_capacity()
        got = _host(gb2, out2)
        np.testing.assert_array_equal(got[1], ref[1])
        for a, b in zip(got[2], ref[2]):
            np.testing.assert_array_equal(a, b)
