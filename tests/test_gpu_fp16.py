"""GPU parity of the IEEE fp16 path (BASELINE config 5: "fp16 + MFMA edge-MLP").

The 16-bit kernels (register-resident fast chains, fused conv layer, segment reductions)
are compiled for fp16 operands as well as bf16 (v_mfma_f32_32x32x16_f16, f32
accumulation; weights packed with RG_PACK_F16).  fp16 keeps 11 significant bits (u = 2^-11)
against bf16's 8, so its error bound is fp16_bound = 8 u S_k -- the bf16_bound construction
of test_gpu_parity.py with fp16's unit roundoff: every output is a final Linear of
channel-normalised activations, perturbed by a few roundoffs of their own scale S_k.
"""
import numpy as np
import pytest
import torch

from conftest import cluster_lists, golden
from oracle import gnn_forward_ref, graph_features_ref as gref
from test_gpu_parity import GRID_MAX_R, HEAD_LAST, _model

pytestmark = pytest.mark.gpu

FP16_U = 2.0 ** -11   # fp16 unit roundoff (11 significant bits, round to nearest)


def fp16_bound(key, ref, pred):
    mod = dict(pred.named_parameters())
    w = mod[HEAD_LAST[key]].detach().float().cpu().numpy()
    rms = np.sqrt(np.mean(np.asarray(ref, np.float64) ** 2, axis=0))
    return 8.0 * FP16_U * np.maximum(rms, np.abs(w).sum(1))


def assert_fp16_close(pred, key, got, ref):
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    assert np.isfinite(got).all(), key
    err = np.abs(got - ref)
    worst = float((err / fp16_bound(key, ref, pred)).max()) if err.size else 0.0
    assert worst <= 1.0, (key, worst, float(err.max()))
    if key != 'node_reg' and len(ref):
        agree = float((got.argmax(-1) == ref.argmax(-1)).mean())
        assert agree >= 0.995, (key, agree)


@pytest.mark.parametrize('name', ['model_trained_N500', 'model_random_L6_N300_k32'])
def test_forward_fp16_close_to_reference(cuda_device, name):
    """fp16 forward vs the reference's fp32 golden outputs, within fp16_bound; the fp16
    fast chains and the fused fp16 conv are the kernels used."""
    d = golden(name)
    pred, cfg = _model(name, cuda_device, 'fp16')
    dev = cuda_device
    ei = torch.from_numpy(d['edge_index'].astype(np.int64)).to(dev)
    with torch.no_grad():
        out = pred(torch.from_numpy(d['node_features']).to(dev),
                   torch.from_numpy(d['edge_features']).to(dev), ei, None,
                   [c.to(dev) for c in cluster_lists(d)])
    plans = pred.plans('fp16')
    assert all(cv.fused_ok for cv in plans.convs), 'fused fp16 conv not used'
    assert any(plans.edge_enc.fast_ok.values()), 'fp16 fast chain not used'
    for got, key in zip(out, ('node_cls', 'node_reg', 'link_cls', 'obj_cls')):
        assert_fp16_close(pred, key, got.cpu().numpy(), d[key])


def test_fp16_tighter_than_bf16(cuda_device):
    """The fp16 path is measurably closer to the fp32 reference than bf16 (3 more mantissa
    bits): on the trained checkpoint its worst node-logit error is below half of bf16's."""
    d = golden('model_trained_N500')
    errs = {}
    for dt in ('bf16', 'fp16'):
        pred, _ = _model('model_trained_N500', cuda_device, dt)
        ei = torch.from_numpy(d['edge_index'].astype(np.int64)).to(cuda_device)
        with torch.no_grad():
            out = pred(torch.from_numpy(d['node_features']).to(cuda_device),
                       torch.from_numpy(d['edge_features']).to(cuda_device), ei, None,
                       [c.to(cuda_device) for c in cluster_lists(d)])
        errs[dt] = float(np.abs(out[0].cpu().numpy() - d['node_cls']).max())
    assert errs['fp16'] < 0.5 * errs['bf16'], errs


def test_c5_full_size_fp16_within_bound(cuda_device):
    """BASELINE config 5 at its full size -- one 20,000-node frame, pure radius graph
    (eps^2 = 2.5, ~400k edges), L = 7, the bench's seeded random-init weights, the bench's
    own pipeline in fp16 -- against the fp32 oracle within fp16_bound."""
    from graph_neural_network_for_radar_perception_amd import _native as nat, synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    dev = cuda_device
    N, L, EPS2 = 20000, 7, 2.5
    cfg = default_config(graph_convolution_stem_channels=[64] * L, k_number_nearest_points=10)
    torch.manual_seed(1234)
    m = Model_Training(cfg, 'cpu')
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    pred = m.to(dev).pred.eval().requires_grad_(False)
    frame = synthetic.make_frame(N, synthetic.SEED0)
    clusters = synthetic.cluster_lists(N)
    batch = FrameBatch.from_frames([frame], [clusters], device=dev)
    pipe = RadarGNNPipeline(pred, cfg, 'fp16', mode=nat.GRAPH_RADIUS, eps2=EPS2)
    with torch.no_grad():
        gb, out = pipe.step(batch)
    torch.cuda.synchronize()
    assert all(cv.fused_ok for cv in pipe.plans.convs), 'fused fp16 conv not used'
    g = gref.build_frame_graph_radius(frame, EPS2, GRID_MAX_R)
    E = int(gb.n_edges_dev.item())
    assert E == g['edge_index'].shape[1] and E > 300000
    with torch.no_grad():
        ref = gnn_forward_ref.forward(sd, cfg, torch.from_numpy(g['node_features']),
                                      torch.from_numpy(g['edge_features']),
                                      torch.from_numpy(g['edge_index']), None,
                                      [torch.from_numpy(c) for c in clusters])
    U = int(gb.graph.n_pairs_dev.item())
    got = (out.node_cls.cpu().numpy(), out.node_reg.cpu().numpy(),
           out.link_cls[:U].cpu().numpy(), out.obj_cls.cpu().numpy())
    for key, gt, rf in zip(('node_cls', 'node_reg', 'link_cls', 'obj_cls'), got, ref):
        assert gt.shape == tuple(rf.shape), key
        assert_fp16_close(pred, key, gt, rf.numpy())


@pytest.mark.parametrize('over', [dict(node_feat_enc_stem_channels=[256, 128, 96],
                                       graph_convolution_stem_channels=[96, 96]),
                                  dict(graph_convolution_stem_channels=[64, 64],
                                       msg_mlp_hidden_dim=96)])
@pytest.mark.parametrize('dtype', ['fp16', 'bf16'])
def test_half_non_yml_widths_match_oracle(cuda_device, over, dtype):
    """16-bit models whose conv blocks are NOT the compiled fused shape (96-wide blocks, a
    96-wide message hidden layer): the unfused path runs -- the generic chain kernel
    (v_mfma_f32_16x16x32_f16 / _bf16 with fp16 / bf16 activations between launches) and
    the fp16 / bf16 segment reduce -- and every output is within its 16-bit bound of the
    fp32 oracle (fp16: 8 u S_k with u = 2^-11; bf16: u = 2^-8)."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    dev = cuda_device
    cfg = default_config(**over)
    torch.manual_seed(31)
    m = Model_Training(cfg, 'cpu')
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    m.pred.compute_dtype = dtype
    pred = m.pred.eval().requires_grad_(False)
    fr = synthetic.make_frame(400, 4242)
    g = gref.build_frame_graph(fr, 25.0, 10, GRID_MAX_R)
    cl = [torch.from_numpy(c) for c in synthetic.cluster_lists(400)]
    args = (torch.from_numpy(g['node_features']), torch.from_numpy(g['edge_features']),
            torch.from_numpy(g['edge_index']))
    with torch.no_grad():
        out = pred(*(a.to(dev) for a in args), None, [c.to(dev) for c in cl])
        ref = gnn_forward_ref.forward(sd, cfg, *args, None, cl)
    plans = pred.plans(dtype)
    assert any(not cv.fused_ok for cv in plans.convs), 'expected an unfused conv layer'
    u = FP16_U if dtype == 'fp16' else 2.0 ** -8
    for key, o, r in zip(('node_cls', 'node_reg', 'link_cls', 'obj_cls'), out, ref):
        got, rf = o.float().cpu().numpy(), r.numpy()
        assert got.shape == rf.shape, key
        assert np.isfinite(got).all(), key
        bound = fp16_bound(key, rf, pred) * (u / FP16_U)
        worst = float((np.abs(got - rf) / bound).max()) if got.size else 0.0
        assert worst <= 1.0, (key, worst)
