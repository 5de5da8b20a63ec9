"""GPU parity: the HIP path against the reference's golden outputs and the oracle.

Tolerances (north_star: fp32 outputs within 1e-4 of the reference CPU path,
edge_index bit-exact):
  * edge_index, ball degree, CSR, link pairs          : bit-exact
  * edge features                                      : bit-exact (same fp32 ops, no FMA)
  * node features                                      : bit-exact except azimuth_conf, which
                                                         depends on numpy's float32 arctan2
                                                         (SIMD/libm-specific): <= 4e-7 abs
  * fp32 forward outputs                               : |d| <= 1e-4 + 1e-4 |ref|
  * bf16 forward outputs (BASELINE config 2 dtype)     : |d_k| <= 8 u max(rms(ref_k), ||w_k||_1), u = 2^-8
                                                         per output k (bf16_bound), >= 99.5 %
                                                         argmax agreement of class logits
"""
import itertools
import os

import numpy as np
import pytest
import torch

from conftest import cluster_lists, golden, golden_names, model_cfg, model_state_dict
from oracle import gnn_forward_ref, graph_features_ref as gref

pytestmark = pytest.mark.gpu

FP32_TOL = dict(rtol=1e-4, atol=1e-4)
FRAME_KEYS = ('meas_px', 'meas_py', 'meas_vx', 'meas_vy', 'meas_vr', 'meas_rcs', 'meas_timestamp')
GRID_MAX_R = float(np.sqrt(np.float64(100 ** 2 + 50 ** 2)))


def _frame(d):
    return {k: d[k] for k in FRAME_KEYS}


def _node_features_close(got, want):
    """Columns 0-4 (vr, rcs, t_norm, degree/10, range_conf) bit-exact.  Column 5
    (azimuth_conf) goes through numpy's float32 arctan2, which is libm/SIMD
    dependent (SVML on AVX-512 hosts: up to 3 ulp off the correctly rounded value
    the kernel produces), so it is checked to 4 ulp of the angle: 4e-7 absolute."""
    got = np.asarray(got, np.float32)
    want = np.asarray(want, np.float32)
    bad = np.argwhere(got[:, :5] != want[:, :5])
    assert len(bad) == 0, [(int(i), int(c), float(got[i, c]), float(want[i, c])) for i, c in bad[:5]]
    np.testing.assert_allclose(got[:, 5], want[:, 5], rtol=0, atol=4e-7)
    return True


def _ulp_close(a, b, ulps=2):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7fffffff), ai)
    bi = np.where(bi < 0, -(bi & 0x7fffffff), bi)
    return np.all(np.abs(ai - bi) <= ulps)


# ------------------------------------------------------------------------- graph build
@pytest.mark.parametrize('name', golden_names('graph_N'))
def test_graph_build_bit_exact(cuda_device, name):
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    d = golden(name)
    fr = _frame(d)
    adj = gf.compute_adjacency_information(fr, float(d['eps']), int(d['k']))
    np.testing.assert_array_equal(adj['adj_list'], d['adj_list'].astype(np.int64))
    np.testing.assert_array_equal(adj['degree'], d['degree'])
    oracle = gref.compute_adjacency_information(fr, float(d['eps']), int(d['k']))
    np.testing.assert_array_equal(adj['adj_matrix'], oracle['adj_matrix'])
    np.testing.assert_array_equal(adj['distance_mat'], oracle['distance_mat'])
    # float64 results like the reference's np.stack (graph_features.py:144,164)
    ef = gf.compute_edge_features(fr, adj['adj_list'])
    assert ef.dtype == np.float64
    np.testing.assert_array_equal(ef, gref.compute_edge_features(fr, d['adj_list']))
    np.testing.assert_array_equal(ef.astype(np.float32), d['edge_features'])
    nf = gf.compute_node_features(fr, adj['degree'], True, 0, GRID_MAX_R, 0, np.pi * 0.5)
    assert nf.dtype == np.float64 and nf.shape[1] == 6
    np.testing.assert_array_equal(nf[:, :5], d['node_features_f64'][:, :5])
    np.testing.assert_allclose(nf[:, 5], d['node_features_f64'][:, 5], rtol=0, atol=4e-7)
    assert _node_features_close(nf, d['node_features'])
    nf4 = gf.compute_node_features(fr, adj['degree'])
    assert nf4.shape[1] == 4 and nf4.dtype == np.float64
    np.testing.assert_array_equal(nf4, d['node_features_f64'][:, :4])


def test_radius_graph_bit_exact(cuda_device):
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    d = golden('graph_radius_N2000')
    adj = gf.compute_radius_graph(_frame(d), float(d['eps']))
    np.testing.assert_array_equal(adj['adj_list'], d['adj_list'].astype(np.int64))


def test_radius_graph_long_rows_and_windows(cuda_device):
    """The pure radius graph (cooperative count + emit, no bitset) against the oracle's dense
    np.where(ball query): a 5 000-point frame (two 4 096-index windows) holding a 300-point
    clump of near-duplicates spread over the index range (rows with > 128 columns take the
    window path) and exact duplicates (d = 0: in the ball, j != i); degree and adj_list
    bit-exact."""
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from graph_neural_network_for_radar_perception_amd import synthetic
    fr = synthetic.make_frame(5000, 77)
    rng = np.random.default_rng(5)
    clump = rng.choice(5000, 300, replace=False)
    fr['meas_px'][clump] = (fr['meas_px'][0] + rng.normal(0, 0.3, 300)).astype(np.float32)
    fr['meas_py'][clump] = (fr['meas_py'][0] + rng.normal(0, 0.3, 300)).astype(np.float32)
    fr['meas_px'][4100:4140] = fr['meas_px'][7]
    fr['meas_py'][4100:4140] = fr['meas_py'][7]
    for eps in (2.5, 0.04):
        got = gf.compute_radius_graph(fr, eps)
        dm = gref.pairwise_sq_distance(fr['meas_px'], fr['meas_py'])
        ball = gref.compute_ball_query(dm, eps)
        want = np.stack(np.where(ball), 0)
        assert int(ball.sum(1).max()) > 128 or eps < 1
        np.testing.assert_array_equal(got['adj_list'], want)
        np.testing.assert_array_equal(got['degree'], ball.sum(1))


def test_knn_union_radius_matches_oracle(cuda_device):
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from graph_neural_network_for_radar_perception_amd import synthetic
    fr = synthetic.make_frame(700, 31)
    got = gf.compute_adjacency_information_v2(fr, 4.0, 6)
    dm = gref.pairwise_sq_distance(fr['meas_px'], fr['meas_py'])
    want = np.stack(np.where(gref.compute_ball_query(dm, 4.0) | gref.compute_knn(dm, 6)), 0)
    np.testing.assert_array_equal(got['adj_list'], want)


def test_lattice_ties_lower_index_first(cuda_device):
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    d = golden('graph_lattice_N400_k10')
    got = gf.compute_adjacency_information(_frame(d), float(d['eps']), int(d['k']))
    want = gref.compute_adjacency_information(_frame(d), float(d['eps']), int(d['k']))
    np.testing.assert_array_equal(got['adj_list'], want['adj_list'])


@pytest.mark.parametrize('n,k', [(1, 10), (2, 10), (5, 10), (11, 10), (12, 10), (40, 33),
                                 (300, 63), (64, 0)])
def test_graph_edge_sizes(cuda_device, n, k):
    """N <= k+1 -> complete graph (graph_features.py:35); k=0 -> self only -> empty graph."""
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from graph_neural_network_for_radar_perception_amd import synthetic
    fr = synthetic.make_frame(n, 1000 + n)
    got = gf.compute_adjacency_information(fr, 25.0, k)
    want = gref.compute_adjacency_information(fr, 25.0, k)
    np.testing.assert_array_equal(got['adj_list'], want['adj_list'])
    np.testing.assert_array_equal(got['degree'], want['degree'])


def test_duplicate_points(cuda_device):
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from graph_neural_network_for_radar_perception_amd import synthetic
    fr = synthetic.make_frame(200, 5)
    fr['meas_px'][50:90] = fr['meas_px'][10]
    fr['meas_py'][50:90] = fr['meas_py'][10]
    got = gf.compute_adjacency_information(fr, 25.0, 10)
    want = gref.compute_adjacency_information(fr, 25.0, 10)
    np.testing.assert_array_equal(got['adj_list'], want['adj_list'])
    np.testing.assert_array_equal(got['degree'], want['degree'])


def _layout(kind, n, seed):
    rng = np.random.default_rng(seed)
    from graph_neural_network_for_radar_perception_amd import synthetic
    fr = synthetic.make_frame(n, seed)
    if kind == 'blobs':      # dense clusters in an empty field (cell occupancy far from uniform)
        c = rng.uniform([0, -50], [100, 50], size=(5, 2))
        pts = c[rng.integers(0, 5, n)] + rng.normal(0, 0.3, size=(n, 2))
    elif kind == 'same':     # every point identical: all distances tie at 0
        pts = np.tile([[12.5, -3.25]], (n, 1))
    elif kind == 'line':     # zero-height bounding box
        pts = np.stack([rng.uniform(0, 100, n), np.full(n, 7.0)], 1)
    elif kind == 'outlier':  # one far point stretches the grid
        pts = rng.uniform([0, -5], [10, 5], size=(n, 2))
        pts[n // 2] = [9000.0, -7000.0]
    elif kind == 'lattice':  # integer lattice: exact distance ties everywhere
        side = int(np.ceil(np.sqrt(n)))
        g = np.stack(np.meshgrid(np.arange(side), np.arange(side)), -1).reshape(-1, 2)[:n]
        pts = g.astype(np.float64) * 0.5
    elif kind == 'offset':   # large coordinates, small spread (f32 cell rounding)
        pts = np.array([1.0e4, -2.0e4]) + rng.uniform(0, 3, size=(n, 2))
    else:
        raise ValueError(kind)
    fr['meas_px'] = pts[:, 0].astype(np.float32)
    fr['meas_py'] = pts[:, 1].astype(np.float32)
    return fr


@pytest.mark.parametrize('kind', ['blobs', 'same', 'line', 'outlier', 'lattice', 'offset'])
@pytest.mark.parametrize('k', [10, 32])
def test_knn_adversarial_layouts(cuda_device, kind, k):
    """Grid ring search == dense argsort oracle on layouts that stress the cell grid
    (kNN set, ties by lower index, ball-query degree, knn | radius union)."""
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    fr = _layout(kind, 700, 4242 + k)
    got = gf.compute_adjacency_information(fr, 25.0, k)
    want = gref.compute_adjacency_information(fr, 25.0, k)
    np.testing.assert_array_equal(got['adj_list'], want['adj_list'])
    np.testing.assert_array_equal(got['degree'], want['degree'])
    got2 = gf.compute_adjacency_information_v2(fr, 4.0, k)
    dm = gref.pairwise_sq_distance(fr['meas_px'], fr['meas_py'])
    want2 = np.stack(np.where(gref.compute_ball_query(dm, 4.0) | gref.compute_knn(dm, k)), 0)
    np.testing.assert_array_equal(got2['adj_list'], want2)


def test_batched_graph_build_equals_per_frame(cuda_device):
    """Disjoint-union batch (frames of different sizes) == frame-by-frame oracle."""
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    cfg = default_config()
    sizes = [37, 500, 2, 1200, 999]
    frames = [synthetic.make_frame(s, 77 + i) for i, s in enumerate(sizes)]
    batch = gf.FrameBatch.from_frames(frames, device=cuda_device)
    gb = gf.build_graph_batch(batch, cfg)
    ei = gb.edge_index().cpu().numpy()
    nf = gb.node_features.cpu().numpy()
    base = 0
    E0 = 0
    for fr, s in zip(frames, sizes):
        want = gref.build_frame_graph(fr, 25.0, 10, GRID_MAX_R)
        m = (ei[0] >= base) & (ei[0] < base + s)
        np.testing.assert_array_equal(ei[:, m] - base, want['edge_index'])
        assert _node_features_close(nf[base:base + s], want['node_features'])
        # destination-major edge features: position p of row i = edge (col -> i)
        E = want['edge_index'].shape[1]
        ef = gb.edge_features[E0:E0 + E].cpu().numpy()
        rev = gref.compute_edge_features(fr, want['edge_index'][::-1].copy()).astype(np.float32)
        np.testing.assert_array_equal(ef, rev)
        base += s
        E0 += E


def test_edge_feature_arithmetic_bit_exact(cuda_device):
    """compute_edge_features' x / 10 and sqrt (graph_features.py:147-164) on adversarial
    float32 operands -- random bit patterns over every exponent, denormals, radar-range
    values -- bit-equal to numpy (the kernel's x / 10 is an f64 product, its sqrt the
    correctly rounded f32 sequence)."""
    from graph_neural_network_for_radar_perception_amd import engine
    rng = np.random.default_rng(77)
    n = 1 << 18

    def operands():
        bits = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
        bits = np.where(np.isfinite(bits) & (np.abs(bits) < 1e18), bits, np.float32(1.5))
        den = (rng.integers(-2 ** 23, 2 ** 23, n).astype(np.float32) * np.float32(2.0 ** -149))
        rad = rng.uniform(-100, 100, n).astype(np.float32)
        pick = rng.integers(0, 3, n)
        return np.where(pick == 0, bits, np.where(pick == 1, den, rad)).astype(np.float32)

    fr = {k: operands() for k in ('meas_px', 'meas_py', 'meas_vx', 'meas_vy')}
    fr['meas_timestamp'] = (10 ** 12 + rng.integers(0, 155000, n)).astype(np.int64)
    src = rng.integers(0, n, n).astype(np.int32)
    dst = rng.integers(0, n, n).astype(np.int32)
    dev_fr = {k: torch.from_numpy(v).to(cuda_device) for k, v in fr.items()}
    got = engine.edge_features(dev_fr, torch.from_numpy(src).to(cuda_device),
                               torch.from_numpy(dst).to(cuda_device), None, n).cpu().numpy()
    with np.errstate(over='ignore', invalid='ignore'):
        want = gref.compute_edge_features(fr, np.stack([src, dst])).astype(np.float32)
    np.testing.assert_array_equal(got, want)


# ------------------------------------------------------------------------- model forward
def _model(name, device, dtype='fp32'):
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    cfg = model_cfg(name)
    m = Model_Training(cfg, device)
    m.load_state_dict(model_state_dict(name))
    m = m.to(device)
    m.pred.compute_dtype = dtype
    return m.pred.eval().requires_grad_(False), cfg


@pytest.mark.parametrize('name', golden_names('model_'))
def test_forward_fp32_matches_reference(cuda_device, name):
    d = golden(name)
    pred, cfg = _model(name, cuda_device)
    dev = cuda_device
    ei = torch.from_numpy(d['edge_index'].astype(np.int64)).to(dev)
    n = int(d['n'])
    adj = torch.zeros((n, n), dtype=torch.bool, device=dev)
    adj[ei[0], ei[1]] = True
    with torch.no_grad():
        out = pred(torch.from_numpy(d['node_features']).to(dev),
                   torch.from_numpy(d['edge_features']).to(dev), ei, adj,
                   [c.to(dev) for c in cluster_lists(d)])
    for got, key in zip(out, ('node_cls', 'node_reg', 'link_cls', 'obj_cls')):
        np.testing.assert_allclose(got.cpu().numpy(), d[key], err_msg=key, **FP32_TOL)
    # the fused f32 conv layer ran wherever the block shape allows it (add / mean, no
    # residual projection), and the register-resident f32 chains for the encoders
    plans = pred.plans('fp32')
    for cv in plans.convs:
        assert bool(cv.fused) == (cv.aggr != 'max' and cv.res is None), name
        if cv.fused:
            assert cv.fused_ok, name
    if name != 'model_random_widths_N120':   # yml widths: an f32 instantiation exists
        assert any(plans.edge_enc.fast_ok.values()) or any(plans.edge_enc.x3_ok.values()), name


BF16_U = 2.0 ** -8   # bf16 unit roundoff (8 significant bits, round to nearest)
HEAD_LAST = {'node_cls': 'predict_node.pred_cls.head.1.weight',
             'node_reg': 'predict_offset.pred_offsets.head.1.weight',
             'link_cls': 'predict_link.pred_cls.head.1.weight',
             'obj_cls': 'predict_class.pred_cls.head.1.weight'}


def bf16_bound(key, ref, pred):
    """Per-output error bound of the bf16 path against the fp32 reference.

    Every output is a final Linear w_k . h + b_k of channel-normalised activations h,
    and the bf16 path perturbs h (and the packed weights) by a few units of bf16
    roundoff relative to their own scale.  So the error of output k is bounded by
    c * u * S_k, u = 2^-8 and S_k = max(rms(ref_k), ||w_k||_1): ||w_k||_1 is the largest
    output an activation of magnitude <= 1 can produce (it floors the scale of outputs
    that are small by cancellation, e.g. the 0.01-scale offsets of node_reg), rms(ref_k)
    the scale of outputs that are large (logits ~5).  c = 8 (|d| <= 3.1 % of S_k): the
    worst measured is 1.1 % (trained checkpoint, N = 500: the trained gains amplify the
    rounding of the 7 bf16 node-state round trips), 0.06 % with the seeded random weights
    at BASELINE config 2's full size (scripts/bf16_error.py)."""
    mod = dict(pred.named_parameters())
    w = mod[HEAD_LAST[key]].detach().float().cpu().numpy()
    l1 = np.abs(w).sum(1)                         # [n_out]
    rms = np.sqrt(np.mean(np.asarray(ref, np.float64) ** 2, axis=0))
    return 8.0 * BF16_U * np.maximum(rms, l1)


def argmax_flips(got, ref):
    """Per row: (the class argmax differs from the reference's, the row is a near-tie: its
    reference top-2 margin is below twice the row's largest error -- the only rows an error
    within the bound can flip)."""
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    if not len(ref):
        return np.zeros(0, bool), np.zeros(0, bool)
    flipped = got.argmax(-1) != ref.argmax(-1)
    top2 = np.sort(ref, axis=-1)[:, -2:]
    tie = (top2[:, 1] - top2[:, 0]) < 2 * np.abs(got - ref).max(-1)
    return flipped, tie


def assert_bf16_close(pred, key, got, ref, min_agree=0.995):
    """Every output within bf16_bound; class argmax agreement >= min_agree (None: reported by
    the caller only -- the seeded random-init model's class logits are near-uniform, so argmax
    flips among near-ties say nothing beyond the bound)."""
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    bound = bf16_bound(key, ref, pred)
    err = np.abs(got - ref)
    worst = float((err / bound).max()) if err.size else 0.0
    assert worst <= 1.0, (key, worst, float(err.max()))
    if key != 'node_reg' and len(ref) and min_agree is not None:
        agree = float((got.argmax(-1) == ref.argmax(-1)).mean())
        assert agree >= min_agree, (key, agree)
    return worst, float(err.max()) if err.size else 0.0


@pytest.mark.parametrize('name', ['model_trained_N500', 'model_random_L6_N300_k32'])
def test_forward_bf16_close_to_reference(cuda_device, name):
    """bf16 forward vs the reference's fp32 golden outputs, within bf16_bound."""
    d = golden(name)
    pred, cfg = _model(name, cuda_device, 'bf16')
    dev = cuda_device
    ei = torch.from_numpy(d['edge_index'].astype(np.int64)).to(dev)
    with torch.no_grad():
        out = pred(torch.from_numpy(d['node_features']).to(dev),
                   torch.from_numpy(d['edge_features']).to(dev), ei, None,
                   [c.to(dev) for c in cluster_lists(d)])
    for got, key in zip(out, ('node_cls', 'node_reg', 'link_cls', 'obj_cls')):
        assert_bf16_close(pred, key, got.cpu().numpy(), d[key])


@pytest.mark.timeout(900)
def test_c2_full_size_bf16_within_bound(cuda_device):
    """BASELINE config 2 at its full size -- 64 frames x 3000 nodes, k = 32, L = 6, the
    bench's seeded random-init weights, the bench's own pipeline -- every frame's four
    outputs against the fp32 oracle within bf16_bound (the fused bf16 conv, the
    register-resident bf16 chains and the graph build all in the loop); the worst error over
    all 64 frames is reported as a fraction of the bound, with the class-argmax flips (all at
    near-ties of the near-uniform random-init logits) ($RG_PARITY_REPORT_C2)."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    dev = cuda_device
    B, N, K, L = 64, 3000, 32, 6
    cfg = default_config(graph_convolution_stem_channels=[64] * L, k_number_nearest_points=K)
    torch.manual_seed(1234)
    m = Model_Training(cfg, 'cpu')
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    pred = m.to(dev).pred.eval().requires_grad_(False)
    frames = [synthetic.make_frame(N, synthetic.SEED0 + f) for f in range(B)]
    clusters = [synthetic.cluster_lists(N) for _ in range(B)]
    batch = FrameBatch.from_frames(frames, clusters, device=dev)
    pipe = RadarGNNPipeline(pred, cfg, 'bf16')
    with torch.no_grad():
        gb, out = pipe.step(batch)
    torch.cuda.synchronize()
    assert all(cv.fused_ok for cv in pipe.plans.convs), 'fused bf16 conv not used'
    U = int(gb.graph.n_pairs_dev.item())
    ps = gb.graph.pair_src[:U].cpu().numpy()
    link = out.link_cls[:U].cpu().numpy()
    keys = ('node_cls', 'node_reg', 'link_cls', 'obj_cls')
    worst = {k: 0.0 for k in keys}
    maxabs = {k: 0.0 for k in keys}
    flips = {k: [0, 0, 0] for k in keys if k != 'node_reg'}  # rows, argmax flips, near-tie rows
    for f in range(B):
        g = gref.build_frame_graph(frames[f], 25.0, K, GRID_MAX_R)
        with torch.no_grad():
            ref = gnn_forward_ref.forward(sd, cfg, torch.from_numpy(g['node_features']),
                                          torch.from_numpy(g['edge_features']),
                                          torch.from_numpy(g['edge_index']), None,
                                          [torch.from_numpy(c) for c in clusters[f]])
        sl = slice(f * N, (f + 1) * N)
        sel = (ps >= f * N) & (ps < (f + 1) * N)
        ncl = len(clusters[f])
        got = (out.node_cls[sl].cpu().numpy(), out.node_reg[sl].cpu().numpy(), link[sel],
               out.obj_cls[f * ncl:(f + 1) * ncl].cpu().numpy())
        for key, gt, rf in zip(keys, got, ref):
            assert gt.shape == tuple(rf.shape), key
            w, a = assert_bf16_close(pred, key, gt, rf.numpy(), min_agree=None)
            worst[key] = max(worst[key], w)
            maxabs[key] = max(maxabs[key], a)
            if key in flips and len(gt):
                fl, tie = argmax_flips(gt, rf.numpy())
                # every argmax flip is a near-tie, row by row: a flip needs err_i + err_j >=
                # the reference margin; a flip on a wide-margin row is a regression
                wide = np.flatnonzero(fl & ~tie)
                assert len(wide) == 0, (key, f, wide[:8].tolist())
                flips[key][0] += len(gt)
                flips[key][1] += int(fl.sum())
                flips[key][2] += int(tie.sum())
    report = {'frames': B, 'nodes': N, 'k': K, 'layers': L, 'dtype': 'bf16',
              'worst_over_bound': worst, 'max_abs_err': maxabs,
              'argmax_rows_flips_near_ties': flips}
    print('C2 bf16 headroom (1.0 = bf16_bound):', report)
    path = os.environ.get('RG_PARITY_REPORT_C2')
    if path:
        import json
        with open(path, 'w') as fh:
            json.dump(report, fh, indent=1)


def test_conv_block_dropin(cuda_device):
    """residual_graph_conv_block.forward on its own (block-level drop-in)."""
    name = 'model_random_widths_N120'
    d = golden(name)
    pred, cfg = _model(name, cuda_device)
    sd = model_state_dict(name)
    dev = cuda_device
    ei = torch.from_numpy(d['edge_index'].astype(np.int64))
    x0 = torch.from_numpy(d['inter/x_enc'])
    e0 = torch.from_numpy(d['inter/e_enc'])
    with torch.no_grad():
        got = pred.pass_messages.conv_blk[0](x0.to(dev), e0.to(dev), ei.to(dev))
    np.testing.assert_allclose(got.cpu().numpy(), d['inter/x_l0'], **FP32_TOL)
    enc = pred.encode_node_feat(torch.from_numpy(d['node_features']).to(dev))
    np.testing.assert_allclose(enc.cpu().numpy(), d['inter/x_enc'], **FP32_TOL)
    del sd


def test_model_training_batched_equals_oracle(cuda_device):
    """Model_Training.forward over several frames (one batched launch sequence)
    == the oracle frame by frame, including the loss values."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.config import default_config
    cfg = default_config(graph_convolution_stem_channels=[64, 64, 64])
    torch.manual_seed(3)
    m = Model_Training(cfg, cuda_device)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(cuda_device).eval().requires_grad_(False)
    dev = cuda_device
    lists = {k: [] for k in ('nf', 'ef', 'ei', 'cl', 'ncls', 'noff', 'ecls', 'clab')}
    outs_ref = []
    rng = np.random.default_rng(0)
    for f, n in enumerate([60, 333, 128]):
        fr = synthetic.make_frame(n, 900 + f)
        g = gref.build_frame_graph(fr, 25.0, 10, GRID_MAX_R)
        cl = [torch.from_numpy(c) for c in synthetic.cluster_lists(n)]
        E = g['edge_index'].shape[1]
        lists['nf'].append(torch.from_numpy(g['node_features']).to(dev))
        lists['ef'].append(torch.from_numpy(g['edge_features']).to(dev))
        lists['ei'].append(torch.from_numpy(g['edge_index']).to(dev))
        lists['cl'].append([c.to(dev) for c in cl])
        lists['ncls'].append(torch.from_numpy(rng.integers(0, 7, n)).to(dev))
        lists['noff'].append(torch.from_numpy(rng.normal(0, 2, (n, 2)).astype(np.float32)).to(dev))
        lists['ecls'].append(torch.from_numpy(rng.integers(0, 2, E // 2)).to(dev))
        lists['clab'].append(torch.from_numpy(rng.integers(0, 7, len(cl))).to(dev))
        with torch.no_grad():
            adj = torch.from_numpy(g['adj_matrix'])
            outs_ref.append(gnn_forward_ref.forward(sd, cfg, torch.from_numpy(g['node_features']),
                                                    torch.from_numpy(g['edge_features']),
                                                    torch.from_numpy(g['edge_index']), adj, cl))
    labels = {'node_class': lists['ncls'], 'node_offsets': lists['noff'],
              'edge_class': lists['ecls'], 'cluster_node_idx': lists['cl'],
              'cluster_labels': lists['clab']}
    with torch.no_grad():
        pred = m.predict(lists['nf'], lists['ef'], lists['ei'], lists['cl'])
        loss, acc = m(lists['nf'], lists['ef'], lists['ei'], [None] * 3, labels)
    for i, key in enumerate(('node_cls', 'node_reg', 'link_cls', 'obj_cls')):
        ref = torch.cat([o[i] for o in outs_ref], 0).numpy()
        np.testing.assert_allclose(pred[i].cpu().numpy(), ref, err_msg=key, **FP32_TOL)
    for k, v in loss.items():
        assert torch.isfinite(v), k


# ------------------------------------------------------------------------- kernels
def test_segment_reduce_ops(cuda_device):
    from graph_neural_network_for_radar_perception_amd import engine
    dev = cuda_device
    torch.manual_seed(0)
    counts = torch.tensor([0, 3, 1, 0, 7, 64, 5, 0, 130], dtype=torch.int64)
    ptr = torch.cat([torch.zeros(1, dtype=torch.int64), counts.cumsum(0)]).to(torch.int32).to(dev)
    E = int(counts.sum())
    for C in (64, 128, 32):
        src = torch.randn(E, C, device=dev)
        seg = torch.repeat_interleave(torch.arange(len(counts)), counts).to(dev)
        for op in ('add', 'mean', 'max'):
            out = torch.empty(len(counts), C, device=dev)
            engine.segment_reduce(src, ptr, len(counts), op, out)
            ref = torch.zeros(len(counts), C, device=dev)
            if op == 'max':
                ref = ref.scatter_reduce(0, seg.view(-1, 1).expand(-1, C), src, 'amax',
                                         include_self=False)
            else:
                ref = ref.index_add(0, seg, src)
                if op == 'mean':
                    ref = ref / counts.clamp(min=1).to(dev).view(-1, 1)
            torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
        # gathered rows (cluster max-pool form) in bf16
        idx = torch.randperm(E, device=dev).to(torch.int32)
        out = torch.empty(len(counts), C, device=dev, dtype=torch.bfloat16)
        engine.segment_reduce(src.bfloat16(), ptr, len(counts), 'max', out, idx=idx)
        ref = torch.zeros(len(counts), C, device=dev).scatter_reduce(
            0, seg.view(-1, 1).expand(-1, C), src.bfloat16().float()[idx.long()], 'amax',
            include_self=False)
        torch.testing.assert_close(out.float(), ref, rtol=0, atol=0)
    # bf16 messages, f32 / bf16 aggregates: 16-B loads (C % 8 == 0) and the 8-B fallback
    for C in (64, 36):
        src = torch.randn(E, C, device=dev).bfloat16()
        seg = torch.repeat_interleave(torch.arange(len(counts)), counts).to(dev)
        ref = torch.zeros(len(counts), C, device=dev).index_add(0, seg, src.float())
        for odt in (torch.float32, torch.bfloat16):
            out = torch.empty(len(counts), C, device=dev, dtype=odt)
            engine.segment_reduce(src, ptr, len(counts), 'add', out)
            torch.testing.assert_close(out.float(), ref.to(odt).float(), rtol=1e-2, atol=1e-2)


def _sequential_segment_sum(src32: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """float32 sums of each segment's rows in row order (one rounding per addition: the
    reference scatter_add_ order on a destination-major CSR), evaluated on the CPU."""
    ptr = torch.cat([torch.zeros(1, dtype=torch.int64), counts.cumsum(0)])
    acc = torch.zeros(len(counts), src32.shape[1], dtype=torch.float32)
    for j in range(int(counts.max())):
        m = counts > j
        acc[m] = acc[m] + src32[ptr[:-1][m] + j]
    return acc


def test_segment_stream_bit_exact(cuda_device):
    """rg_segment_reduce sum / mean / max over a plain CSR (the streaming kernel: one or two
    segments per lane group as one row stream, restarting the sum at each boundary, 8 / 16 / 32
    rows in flight -- every compiled schedule, rg_segment_reduce_sched) equals the in-order
    float32 sum bit for bit: empty segments at every position of a group, an odd segment
    count, short (kNN-like) and long row runs, f32 and bf16 messages, C = 64 and 128; max:
    empty segments 0, as PyG / scatter_reduce(include_self=False)."""
    from graph_neural_network_for_radar_perception_amd import engine
    dev = cuda_device
    g = torch.Generator().manual_seed(7)
    counts = torch.randint(0, 30, (4099,), generator=g)
    counts[::5] = 0
    counts[1::7] = 0
    counts[100] = 700
    counts[-1] = 0
    ptr = torch.cat([torch.zeros(1, dtype=torch.int64), counts.cumsum(0)]).to(torch.int32).to(dev)
    E, S = int(counts.sum()), len(counts)
    # (segments per lane group (0: one-segment-per-group kernel), rows in flight per lane,
    # 8-B bf16 lanes); None: the library's default schedule (rg_segment_reduce)
    variants = [None, (0, 0, False), (2, 8, False), (1, 4, False), (2, 4, False), (4, 8, False),
                (1, 16, False), (1, 12, False), (1, 8, True), (2, 8, True)]

    def run(v, s_dev, op, out):
        if v is None:
            return engine.segment_reduce(s_dev, ptr, S, op, out)
        return engine.segment_reduce_sched(s_dev, ptr, S, op, out, *v)

    for C, sdt, v in itertools.product((64, 128), (torch.float32, torch.bfloat16), variants):
        src = torch.randn(E, C, generator=g)
        s_dev = src.to(sdt).to(dev)
        ref = _sequential_segment_sum(src.to(sdt).float(), counts)
        out = torch.empty(S, C, device=dev)
        run(v, s_dev, 'add', out)
        assert torch.equal(out.cpu(), ref), (C, sdt, v)
        run(v, s_dev, 'mean', out)
        mean = ref / counts.clamp(min=1).to(torch.float32).view(-1, 1)
        assert torch.equal(out.cpu(), mean), (C, sdt, v)
        run(v, s_dev, 'max', out)
        seg = torch.repeat_interleave(torch.arange(S), counts)
        mx = torch.zeros(S, C).scatter_reduce(0, seg.view(-1, 1).expand(-1, C),
                                              src.to(sdt).float(), 'amax', include_self=False)
        assert torch.equal(out.cpu(), mx), (C, sdt, v)


def test_segment_order_and_ordered_reduce_bit_exact(cuda_device):
    """rg_segment_order is a permutation of the segments with non-increasing lengths (capped at
    255); rg_segment_reduce_ordered over it equals the in-order float32 sum / mean / max bit for
    bit (f32 / bf16 rows, C = 64 / 128, 8 / 12 / 16 rows in flight, 8-B and 16-B bf16 lanes),
    on a graph with empty segments and segments longer than the 255 cap."""
    from graph_neural_network_for_radar_perception_amd import engine
    dev = cuda_device
    g = torch.Generator().manual_seed(11)
    counts = torch.randint(0, 64, (5003,), generator=g)
    counts[::9] = 0
    counts[17] = 400
    counts[4000] = 300
    ptr = torch.cat([torch.zeros(1, dtype=torch.int64), counts.cumsum(0)]).to(torch.int32).to(dev)
    E, S = int(counts.sum()), len(counts)
    order = engine.segment_order(ptr, S).cpu()
    assert torch.equal(order.sort().values, torch.arange(S, dtype=torch.int32))
    lens = counts.clamp(max=255)[order.long()]
    assert bool((lens[1:] <= lens[:-1]).all())
    seg = torch.repeat_interleave(torch.arange(S), counts)
    order_d = order.to(dev)
    # None: the library's default (rg_segment_reduce_ordered); else (rows in flight, 8-B lanes)
    variants = [None, (8, True), (16, True), (12, False), (8, False)]

    def run(v, s_dev, op, out):
        if v is None:
            return engine.segment_reduce_ordered(s_dev, ptr, order_d, S, op, out)
        return engine.segment_reduce_sched(s_dev, ptr, S, op, out, 1, v[0], v[1], order=order_d)

    for C, sdt, v in itertools.product((64, 128), (torch.float32, torch.bfloat16), variants):
        src = torch.randn(E, C, generator=g)
        s_dev = src.to(sdt).to(dev)
        ref = _sequential_segment_sum(src.to(sdt).float(), counts)
        out = torch.empty(S, C, device=dev)
        run(v, s_dev, 'add', out)
        assert torch.equal(out.cpu(), ref), (C, sdt, v)
        run(v, s_dev, 'mean', out)
        assert torch.equal(out.cpu(), ref / counts.clamp(min=1).to(torch.float32).view(-1, 1))
        run(v, s_dev, 'max', out)
        mx = torch.zeros(S, C).scatter_reduce(0, seg.view(-1, 1).expand(-1, C),
                                              src.to(sdt).float(), 'amax', include_self=False)
        assert torch.equal(out.cpu(), mx), (C, sdt, v)
        if sdt == torch.bfloat16:  # bf16 output rows
            ob = torch.empty(S, C, dtype=torch.bfloat16, device=dev)
            run(v, s_dev, 'add', ob)
            assert torch.equal(ob.cpu(), ref.to(torch.bfloat16))
    with pytest.raises(RuntimeError):   # not a compiled schedule
        engine.segment_reduce_sched(src.to(dev), ptr, S, 'add', torch.empty(S, 128, device=dev), 3, 8)


@pytest.mark.parametrize('dtype', ['fp32', 'bf16', 'fp16'])
def test_chain_kernel_vs_torch(cuda_device, dtype):
    """rg_mlp_chain against a plain torch fp32 evaluation (widths not multiples of 16,
    norm on/off, every activation, residual); fp16 = the generic chain's IEEE fp16 operands."""
    from graph_neural_network_for_radar_perception_amd import engine
    from graph_neural_network_for_radar_perception_amd.common import ffn_block
    dev = cuda_device
    torch.manual_seed(1)
    blocks = [ffn_block(13, 200, 'leakyrelu'), ffn_block(200, 72, 'relu', 'channel_normalization'),
              ffn_block(72, 256, 'swish', 'channel_normalization'),
              ffn_block(256, 40, 'leakyrelu', 'channel_normalization'), torch.nn.Linear(40, 3)]
    for b in blocks:
        for p in b.parameters():
            if p.numel() == 1:
                p.data.uniform_(0.5, 1.5)
    blocks = [b.to(dev) for b in blocks]
    x = torch.randn(1001, 13, device=dev) * 3
    sd = {}
    with torch.no_grad():
        h = x
        for b in blocks:
            if isinstance(b, torch.nn.Linear):
                h = torch.nn.functional.linear(h, b.weight, b.bias)
                continue
            lin, norm, act = b.block[0], (b.block[1] if len(b.block) == 3 else None), b.block[-1].kind
            h = torch.nn.functional.linear(h, lin.weight, lin.bias)
            if norm is not None:
                h = (h - h.mean(1, keepdim=True)) / (h.std(1, keepdim=True) + 1e-5) * norm.std + norm.mu
            h = {'leakyrelu': lambda t: torch.nn.functional.leaky_relu(t, 0.01),
                 'relu': torch.relu, 'swish': torch.nn.functional.silu}[act](h)
        ref = h
        plan = engine.ChainPlan(engine.specs_from_modules(blocks), dtype, dev)
        out = torch.empty(1001, 3, device=dev)
        res = torch.randn(1001, 3, device=dev)
        plan(1001, out, x, 13, residual=res)
    tol = (FP32_TOL if dtype == 'fp32' else dict(rtol=0.01, atol=0.01) if dtype == 'fp16'
           else dict(rtol=0.05, atol=0.05))
    torch.testing.assert_close(out, ref + res, **tol)
    del sd


# ------------------------------------------------------------------------- pipeline
def test_pipeline_end_to_end_matches_oracle(cuda_device):
    """Raw measurements in HBM -> graph -> features -> forward, batched, vs the
    oracle's per-frame reference path."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    cfg = default_config()
    d = golden('model_trained_N50')
    sd = {k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith('w/')}
    m = Model_Training(cfg, cuda_device)
    m.load_state_dict(sd)
    m = m.to(cuda_device).eval().requires_grad_(False)
    sizes = [300, 41, 777]
    frames = [synthetic.make_frame(s, 4000 + i) for i, s in enumerate(sizes)]
    clusters = [synthetic.cluster_lists(s) for s in sizes]
    batch = FrameBatch.from_frames(frames, clusters, device=cuda_device)
    pipe = RadarGNNPipeline(m.pred, cfg, 'fp32')
    with torch.no_grad():
        gb, out = pipe.step(batch)
        got = RadarGNNPipeline.trim(gb, out)
    refs = []
    for fr, cl in zip(frames, clusters):
        g = gref.build_frame_graph(fr, 25.0, 10, GRID_MAX_R)
        with torch.no_grad():
            refs.append(gnn_forward_ref.forward(sd, cfg, torch.from_numpy(g['node_features']),
                                                torch.from_numpy(g['edge_features']),
                                                torch.from_numpy(g['edge_index']),
                                                torch.from_numpy(g['adj_matrix']),
                                                [torch.from_numpy(c) for c in cl]))
    for i, key in enumerate(('node_cls', 'node_reg', 'link_cls', 'obj_cls')):
        ref = torch.cat([r[i] for r in refs], 0).numpy()
        np.testing.assert_allclose(got[i].cpu().numpy(), ref, err_msg=key, **FP32_TOL)


C5_NODES, C5_EPS2 = 20000, 2.5   # N = 20,000, eps^2 ~2.5 -> E ~ 400k


def test_c5_radius_graph_and_forward_match_oracle(cuda_device):
    """BASELINE config 5 shape (one 20,000-node frame, pure radius graph
    compute_ball_query semantics, L = 7): edge_index / degree / features bit-exact
    against the oracle (evaluated by row blocks), and the fp32 forward through the
    batched pipeline within 1e-4 of the oracle forward."""
    from graph_neural_network_for_radar_perception_amd import _native as nat
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    cfg = default_config(graph_convolution_stem_channels=[64] * 7)
    torch.manual_seed(1234)
    m = Model_Training(cfg, 'cpu')
    sd = {k: v.detach().clone() for k, v in m.pred.state_dict().items()}
    m = m.to(cuda_device).eval().requires_grad_(False)
    fr = synthetic.make_frame(C5_NODES, 777)
    cl = synthetic.cluster_lists(C5_NODES)
    batch = FrameBatch.from_frames([fr], [cl], device=cuda_device)
    pipe = RadarGNNPipeline(m.pred, cfg, 'fp32', mode=nat.GRAPH_RADIUS, eps2=C5_EPS2)
    with torch.no_grad():
        gb, out = pipe.step(batch)
        got = RadarGNNPipeline.trim(gb, out)
    want = gref.build_frame_graph_radius(fr, C5_EPS2, GRID_MAX_R)
    E = int(gb.n_edges_dev.item())
    assert 300_000 < E < 500_000, E
    rp = gb.row_ptr.cpu().numpy().astype(np.int64)
    rows = np.repeat(np.arange(C5_NODES), np.diff(rp))
    np.testing.assert_array_equal(np.stack((rows, gb.col[:E].cpu().numpy())), want['edge_index'])
    np.testing.assert_array_equal(gb.ball_degree.cpu().numpy(), want['degree'])
    assert _node_features_close(gb.node_features.cpu().numpy(), want['node_features'])
    with torch.no_grad():
        ref = gnn_forward_ref.forward(sd, cfg, torch.from_numpy(want['node_features']),
                                      torch.from_numpy(want['edge_features']),
                                      torch.from_numpy(want['edge_index']), None,
                                      [torch.from_numpy(c) for c in cl])
    for i, key in enumerate(('node_cls', 'node_reg', 'link_cls', 'obj_cls')):
        np.testing.assert_allclose(got[i].cpu().numpy(), ref[i].numpy(), err_msg=key, **FP32_TOL)


def test_large_batch_graph_properties(cuda_device):
    """BASELINE config 2 scale (64 frames x 3000 nodes, k=32): size-independent
    properties -- symmetric, sorted rows, no self loops, degree >= k, ball degree
    and link pair count consistent -- plus bit-exact spot frames vs the oracle."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    cfg = default_config(k_number_nearest_points=32)
    frames = synthetic.make_batch(64, 3000)
    batch = gf.FrameBatch.from_frames(frames, device=cuda_device)
    gb = gf.build_graph_batch(batch, cfg)
    E = int(gb.n_edges_dev.item())
    rp = gb.row_ptr.cpu().numpy().astype(np.int64)
    col = gb.col[:E].cpu().numpy().astype(np.int64)
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    assert rp[-1] == E
    assert np.all(np.diff(rp) >= 32)
    assert not np.any(rows == col)
    same_row = rows[1:] == rows[:-1]
    assert np.all(col[1:][same_row] > col[:-1][same_row])
    key = rows * 10**6 + col
    rkey = col * 10**6 + rows
    assert np.array_equal(np.sort(key), np.sort(rkey))
    assert int(gb.graph.n_pairs_dev.item()) * 2 == E
    for f in (0, 37, 63):
        want = gref.compute_adjacency_information(frames[f], 25.0, 32)
        m = (rows >= 3000 * f) & (rows < 3000 * (f + 1))
        np.testing.assert_array_equal(np.stack((rows[m], col[m])) - 3000 * f, want['adj_list'])
        np.testing.assert_array_equal(gb.ball_degree[3000 * f:3000 * (f + 1)].cpu().numpy(),
                                      want['degree'])


def test_fast_chains_match_generic_and_fp32(cuda_device):
    """rg_mlp_chain_fast (register-resident, 32x32x16 MFMA) is used for every chain of
    the yml architecture in bf16 and agrees with the generic bf16 kernel and with a
    torch fp32 evaluation of the same weights."""
    from graph_neural_network_for_radar_perception_amd import _native as nat
    from graph_neural_network_for_radar_perception_amd import engine
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    dev = cuda_device
    torch.manual_seed(5)
    cfg = default_config()
    m = Model_Training(cfg, dev).to(dev).eval().requires_grad_(False)
    plans = m.pred.plans('bf16')
    g = torch.Generator(device='cpu').manual_seed(0)
    R = 2000

    def rnd(*shape, dtype=torch.bfloat16):
        return (torch.randn(*shape, generator=g) * 2).to(dtype).to(dev)

    def torch_chain(plan, x):
        h = x.float()
        for s in plan.specs:
            h = torch.nn.functional.linear(h, s.weight.float(), s.bias.float())
            if s.mu is not None:
                h = (h - h.mean(1, keepdim=True)) / (h.std(1, keepdim=True) + 1e-5) * s.std + s.mu
            if s.act == 'leakyrelu':
                h = torch.nn.functional.leaky_relu(h, 0.01)
        return h

    idx0 = torch.randint(0, R, (R,), generator=g).to(torch.int32).to(dev)
    idx1 = torch.randint(0, R, (R,), generator=g).to(torch.int32).to(dev)
    x64 = rnd(R, 64)
    cases = [
        (plans.node_enc, dict(in0=rnd(R, 6, dtype=torch.float32), w0=6),
         lambda: rnd(R, 6, dtype=torch.float32)),
        (plans.edge_enc, dict(in0=rnd(R, 7, dtype=torch.float32), w0=7), None),
        (plans.convs[0].msg, dict(in0=x64, w0=64, mode=nat.IN_GATHER3, in2=rnd(R, 64), w2=64,
                                  idx0=idx0, idx1=idx1), None),
        (plans.convs[0].upd, dict(in0=x64, w0=64, mode=nat.IN_CONCAT2, in1=rnd(R, 64), w1=64,
                                  residual=x64), None),
        (plans.node_head, dict(in0=x64, w0=64), None),
        (plans.offset_head, dict(in0=x64, w0=64), None),
        (plans.link_pair, dict(in0=x64, w0=64, mode=nat.IN_PAIRADD, idx0=idx0, idx1=idx1), None),
        (plans.cls_stem, dict(in0=x64, w0=64), None),
        (plans.cls_head, dict(in0=x64, w0=64), None),
    ]
    for plan, kw, _ in cases:
        outs = []
        for use_fast in (True, False):
            plan.use_fast = use_fast
            plan.fast_ok = {}
            out = torch.empty(R, plan.out_dim, device=dev)
            plan(R, out, **kw)
            outs.append(out)
            if use_fast:
                assert plan.fast_ok.get(kw.get('mode', nat.IN_DENSE)), 'fast kernel not used'
        plan.use_fast = True
        mode = kw.get('mode', nat.IN_DENSE)
        if mode == nat.IN_GATHER3:
            xin = torch.cat([kw['in0'][idx0.long()], kw['in0'][idx1.long()], kw['in2']], 1)
        elif mode == nat.IN_CONCAT2:
            xin = torch.cat([kw['in0'], kw['in1']], 1)
        elif mode == nat.IN_PAIRADD:
            xin = kw['in0'][idx0.long()].float() + kw['in0'][idx1.long()].float()
        else:
            xin = kw['in0']
        ref = torch_chain(plan, xin)
        if kw.get('residual') is not None:
            ref = ref + kw['residual'].float()
        torch.testing.assert_close(outs[0], outs[1], rtol=0.05, atol=0.05)
        err = (outs[0] - ref).abs()
        assert float((err <= 0.05 + 0.05 * ref.abs()).float().mean()) >= 0.995


@pytest.mark.parametrize('aggr', ['add', 'mean'])
def test_fused_conv_layer_matches_unfused(cuda_device, aggr):
    """rg_conv_layer_fused (message MLP + MFMA segment sum + update in one launch)
    against the unfused bf16 path (chain + rg_segment_reduce + chain) and the fp32
    oracle of residual_graph_conv_block on a batched kNN graph."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    dev = cuda_device
    cfg = default_config(graph_convolution_stem_channels=[64], aggregation=aggr,
                         k_number_nearest_points=32)
    torch.manual_seed(11)
    m = Model_Training(cfg, dev).to(dev).eval().requires_grad_(False)
    plans = m.pred.plans('bf16')
    cv = plans.convs[0]
    assert cv.fused
    frames = [synthetic.make_frame(n, 70 + i) for i, n in enumerate([700, 33, 1500])]
    batch = gf.FrameBatch.from_frames(frames, device=dev)
    gb = gf.build_graph_batch(batch, cfg)
    g = gb.graph
    N = batch.n_nodes
    E = int(gb.n_edges_dev.item())
    gen = torch.Generator(device='cpu').manual_seed(1)
    x = (torch.randn(N, 64, generator=gen) * 1.5).bfloat16().to(dev)
    e = (torch.randn(gb.capacity, 64, generator=gen) * 1.5).bfloat16().to(dev)
    out_f = torch.empty(N, 64, dtype=torch.bfloat16, device=dev)
    assert cv.run_fused(x, e, g, out_f)
    # unfused bf16 path
    msg = torch.empty(gb.capacity, 64, dtype=torch.bfloat16, device=dev)
    cv.msg(gb.capacity, msg, x, 64, mode=2, in2=e, w2=64, idx0=g.dst, idx1=g.src,
           rows_dev=gb.n_edges_dev)
    agg = torch.empty(N, 64, dtype=torch.bfloat16, device=dev)
    from graph_neural_network_for_radar_perception_amd import engine
    engine.segment_reduce(msg, g.seg_ptr, N, aggr, agg)
    out_u = torch.empty(N, 64, dtype=torch.bfloat16, device=dev)
    cv.upd(N, out_u, x, 64, mode=1, in1=agg, w1=64, residual=x)
    # fp32 oracle of the block on the same (bf16-valued) inputs
    sd = {k: v.float().cpu() for k, v in m.state_dict().items()}
    ei = torch.stack((g.src[:E], g.dst[:E])).long().cpu()
    with torch.no_grad():
        ctx = gnn_forward_ref._Ctx(sd, cfg)
        ref = gnn_forward_ref.conv_block(ctx, 'pass_messages.conv_blk.0', x.float().cpu(),
                                         e[:E].float().cpu(), ei)
    of, ou = out_f.float().cpu(), out_u.float().cpu()
    torch.testing.assert_close(of, ou, rtol=0.03, atol=0.06)
    err = (of - ref).abs()
    assert float((err <= 0.05 + 0.03 * ref.abs()).float().mean()) >= 0.995, float(err.max())


def test_fused_conv_block_table_bit_identical(cuda_device):
    """Edge-balanced work blocks (rg_conv_blocks + rg_conv_layer_fused_blocks) on a
    skewed-degree radius graph: the (first, end) node pairs cover every node once, in runs
    of <= 8 nodes split only where the edge cap is passed, each XCD's share of the dequeue
    order sorted by tile count (largest first), and the layer output is bit-identical to
    the plain 8-node schedule (each destination still sums its edges in CSR order inside
    one block)."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    dev = cuda_device
    cfg = default_config(graph_convolution_stem_channels=[64])
    torch.manual_seed(3)
    m = Model_Training(cfg, dev).to(dev).eval().requires_grad_(False)
    cv = m.pred.plans('bf16').convs[0]
    fr = synthetic.make_frame(6000, 555)
    fr['meas_px'][:400] = np.float32(50.0) + fr['meas_px'][:400] * np.float32(0.01)  # a hub
    fr['meas_py'][:400] = np.float32(0.0) + fr['meas_py'][:400] * np.float32(0.01)
    batch = gf.FrameBatch.from_frames([fr], device=dev)
    from graph_neural_network_for_radar_perception_amd import _native as nat
    gb = gf.build_graph_batch(batch, cfg, mode=nat.GRAPH_RADIUS, eps2=4.0)
    g = gb.graph
    N = batch.n_nodes
    tbl, nb = g.conv_blocks()
    assert tbl is not None
    nbk = int(nb.item())
    pairs = tbl[:2 * nbk].cpu().numpy().reshape(nbk, 2)
    seg = g.seg_ptr.cpu().numpy()
    tiles = (seg[pairs[:, 1]] - seg[pairs[:, 0]] + 31) // 32
    for x in range(8):                                      # per-XCD share: largest first
        lo, hi = nbk * x // 8, nbk * (x + 1) // 8
        assert np.all(np.diff(tiles[lo:hi]) <= 0)
    order = np.argsort(pairs[:, 0], kind='stable')
    t = np.concatenate([pairs[order, 0], pairs[order[-1:], 1]])
    assert np.all(pairs[order[:-1], 1] == pairs[order[1:], 0])  # contiguous cover
    assert t[0] == 0 and t[-1] == N and np.all(np.diff(t) >= 1) and np.all(np.diff(t) <= 8)
    assert set(range(0, N, 8)) <= set(t.tolist())          # only splits of the 8-node runs
    cap = max(128, int(seg[N]) // 4096)
    sizes = seg[t[1:]] - seg[t[:-1]]
    single = np.diff(t) == 1
    assert np.all((sizes <= cap) | single), 'a multi-node block over the edge cap'
    assert nbk > (N + 7) // 8                               # the hub was split
    gen = torch.Generator(device='cpu').manual_seed(2)
    x = (torch.randn(N, 64, generator=gen) * 1.5).bfloat16().to(dev)
    e = (torch.randn(gb.capacity, 64, generator=gen) * 1.5).bfloat16().to(dev)
    out_t = torch.empty(N, 64, dtype=torch.bfloat16, device=dev)
    assert cv.run_fused(x, e, g, out_t)
    g.CONV_BLOCK_TABLE_MAX_RUNS = 0                         # plain 8-node runs
    out_p = torch.empty(N, 64, dtype=torch.bfloat16, device=dev)
    assert cv.run_fused(x, e, g, out_p)
    assert torch.equal(out_t, out_p)


@pytest.mark.parametrize('dtype', ['bf16', 'fp16'])
def test_fused_conv_wave_schedule(cuda_device, dtype):
    """The static schedule of the 16-bit fused conv (rg_conv_wave_nodes +
    rg_conv_layer_fused_waves): wave ranges cover the nodes in order, XCD-major, each share of
    degree + 4 per node within one node of the mean, and the layer output matches the
    block-table and plain 8-node schedules (test_fused_conv_layer_matches_unfused's bound,
    < 1 % of outputs differing at all): one wave sums each destination's edges in CSR order
    in all three, but where a destination's edges start inside the block's 32-edge tiles --
    the 16-edge groups the aggregation MFMA adds before its f32 accumulator -- follows the
    block boundaries, and a last-bit change of the 16-bit aggregate passes through the
    update MLP.  A skewed radius frame, and a tiny one with more waves than nodes."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from graph_neural_network_for_radar_perception_amd import _native as nat
    dev = cuda_device
    cfg = default_config(graph_convolution_stem_channels=[64])
    torch.manual_seed(4)
    m = Model_Training(cfg, dev).to(dev).eval().requires_grad_(False)
    cv = m.pred.plans(dtype).convs[0]
    td = torch.bfloat16 if dtype == 'bf16' else torch.float16
    for n_nodes, seed in ((6000, 556), (37, 557)):
        fr = synthetic.make_frame(n_nodes, seed)
        fr['meas_px'][:n_nodes // 15] = np.float32(50.0) + fr['meas_px'][:n_nodes // 15] * np.float32(0.01)
        fr['meas_py'][:n_nodes // 15] = fr['meas_py'][:n_nodes // 15] * np.float32(0.01)
        batch = gf.FrameBatch.from_frames([fr], device=dev)
        gb = gf.build_graph_batch(batch, cfg, mode=nat.GRAPH_RADIUS, eps2=4.0)
        g = gb.graph
        N = batch.n_nodes
        wn = g.conv_waves()
        assert wn is not None and wn.numel() == g.CONV_WAVES + 1
        w = wn.cpu().numpy().astype(np.int64)
        seg = g.seg_ptr.cpu().numpy().astype(np.int64)
        # w[-1]: the end of the static ranges -- N, or the start of the dynamic tail the
        # waves take in NB-node blocks once their ranges are done (RG_CONV_TAIL % of the cost)
        assert w[0] == 0 and w[-1] <= N and np.all(np.diff(w) >= 0)
        cost = seg[w] + 4 * w
        total = seg[N] + 4 * N
        assert cost[-1] >= 0.7 * total - 1
        share = cost[-1] / g.CONV_WAVES
        node_max = int(np.max(np.diff(seg))) + 4
        assert np.all(np.diff(cost) <= share + node_max + 1)
        gen = torch.Generator(device='cpu').manual_seed(3)
        x = (torch.randn(N, 64, generator=gen) * 1.5).to(td).to(dev)
        e = (torch.randn(gb.capacity, 64, generator=gen) * 1.5).to(td).to(dev)
        outs = []
        for waves, runs in ((g.CONV_WAVES, g.CONV_BLOCK_TABLE_MAX_RUNS), (0, g.CONV_BLOCK_TABLE_MAX_RUNS),
                            (0, 0)):
            g.CONV_WAVES, g.CONV_BLOCK_TABLE_MAX_RUNS = waves, runs
            o = torch.full((N, 64), float('nan'), dtype=td, device=dev)
            assert cv.run_fused(x, e, g, o)
            outs.append(o)
        del g.CONV_WAVES, g.CONV_BLOCK_TABLE_MAX_RUNS   # back to the class defaults
        assert torch.isfinite(outs[0].float()).all()
        for o in outs[1:]:
            a, b = outs[0].float(), o.float()
            torch.testing.assert_close(a, b, rtol=0.03, atol=0.06)
            assert float(((a - b).abs() > 0).float().mean()) < 0.01


# ------------------------------------------------------------------------ proposal branch
def _lists_from_ids(ids):
    ids = np.asarray(ids)
    return [np.nonzero(ids == i)[0] for i in range(int(ids.max()) + 1)]


def _assert_same_lists(got_ptr, got_idx, want_lists, base=0):
    got_ptr = np.asarray(got_ptr)
    got_idx = np.asarray(got_idx)
    assert len(got_ptr) - 1 == len(want_lists), (len(got_ptr) - 1, len(want_lists))
    for i, w in enumerate(want_lists):
        np.testing.assert_array_equal(got_idx[got_ptr[i]:got_ptr[i + 1]] - base, w)


@pytest.mark.parametrize('name', golden_names('proposals_dbscan'))
def test_proposal_clusters_match_reference_dbscan(cuda_device, name):
    """rg_proposal_centres + rg_cluster_radius / rg_cluster_pairs + rg_cluster_lists ==
    the reference's Simple_DBSCAN (clustering.py:43-93), both adjacency modes, and the
    centres bit-exact (compute_offsets.py:13-17)."""
    from graph_neural_network_for_radar_perception_amd import engine
    import graph_neural_network_for_radar_perception_amd._native as nat
    d = golden(name)
    n = d['centres'].shape[0]
    dev = cuda_device
    off = torch.from_numpy(d['offsets']).to(dev)
    xy = torch.from_numpy(d['other_xy']).to(dev)
    cx = torch.empty(n, device=dev)
    cy = torch.empty(n, device=dev)
    nat.check(nat.lib().rg_proposal_centres(off.data_ptr(), 2, xy.data_ptr(), 2, n,
                                            float(d['mu'][0]), float(d['mu'][1]),
                                            float(d['sigma'][0]), float(d['sigma'][1]),
                                            cx.data_ptr(), cy.data_ptr(), 0), 'centres')
    np.testing.assert_array_equal(torch.stack([cx, cy], 1).cpu().numpy(), d['centres'])
    fptr = torch.tensor([0, n], dtype=torch.int32, device=dev)
    ptr, idx, ncl = engine.propose_clusters(off, xy, fptr, [n], d['mu'], d['sigma'],
                                            float(d['eps']))
    _assert_same_lists(ptr.cpu(), idx.cpu(), _lists_from_ids(d['ids_offsets']))
    # predicted-link mode: logits whose argmax is the fixture's pred_edges
    ei = torch.from_numpy(d['adj_list'].astype(np.int64)).to(dev)
    g = engine.DeviceGraph.from_edge_index(ei, n)
    pe = torch.from_numpy(d['pred_edges']).to(dev).float()
    logits = torch.stack([1.0 - pe, pe], 1).contiguous()
    assert logits.shape[0] == g.n_pairs
    ptr, idx, ncl = engine.propose_clusters(off, xy, fptr, [n], d['mu'], d['sigma'],
                                            float(d['eps']), from_links=True, g=g,
                                            link_cls=logits)
    _assert_same_lists(ptr.cpu(), idx.cpu(), _lists_from_ids(d['ids_links']))


def test_proposal_clusters_batched_frames(cuda_device):
    """Several frames in one call: per-frame components, frames concatenated in order."""
    from graph_neural_network_for_radar_perception_amd import engine
    ds = [golden(nm) for nm in golden_names('proposals_dbscan')]
    dev = cuda_device
    off = torch.from_numpy(np.concatenate([d['offsets'] for d in ds])).to(dev)
    xy = torch.from_numpy(np.concatenate([d['other_xy'] for d in ds])).to(dev)
    sizes = [d['offsets'].shape[0] for d in ds]
    fptr = torch.tensor(np.cumsum([0] + sizes), dtype=torch.int32, device=dev)
    ptr, idx, ncl = engine.propose_clusters(off, xy, fptr, sizes, ds[0]['mu'], ds[0]['sigma'],
                                            float(ds[0]['eps']))
    want, base = [], 0
    for d, s in zip(ds, sizes):
        want += [w + base for w in _lists_from_ids(d['ids_offsets'])]
        base += s
    _assert_same_lists(ptr.cpu(), idx.cpu(), want)


@pytest.mark.parametrize('tag', ['off', 'links'])
def test_model_inference_proposals_match_reference(cuda_device, tag):
    """Model_Inference(extract_proposals=True).forward without cluster_node_idx
    (gnn_detector.py:164-195) against the reference run: the clusters (exact, unless a
    centre pair sits within 1e-4 of the eps threshold) and all five outputs."""
    from oracle import proposals_ref as pref
    d = golden('proposals_model_trained_N300')
    m, _ = _model('proposals_model_trained_N300', cuda_device)
    m.set_param_for_proposal_extraction(float(d['eps']), tag == 'links')
    dev = cuda_device
    args = (torch.from_numpy(d['node_features']).to(dev), torch.from_numpy(d['edge_features']).to(dev),
            torch.from_numpy(d['edge_index'].astype(np.int64)).to(dev), None)
    with torch.no_grad():
        out = m(*args, None, other_features=torch.from_numpy(d['other_features']).to(dev))
    assert len(out) == 5
    for got, key in zip(out[:3], ('node_cls', 'node_reg', 'link_cls')):
        np.testing.assert_allclose(got.cpu().numpy(), d[f'{tag}/{key}'], rtol=1e-4, atol=1e-4)
    ptr, idx = d[f'{tag}/cluster_ptr'], d[f'{tag}/cluster_idx']
    want = [idx[ptr[i]:ptr[i + 1]] for i in range(len(ptr) - 1)]
    centres = pref.cluster_centres(d['other_features'][:, :2], d[f'{tag}/node_reg'], [0, 0], [8, 4])
    dd = ((centres[:, None, :] - centres[None]) ** 2).sum(-1)
    near = np.abs(dd - float(d['eps'])) < 1e-4
    if not near.any():
        got = [c.cpu().numpy() for c in out[4]]
        assert len(got) == len(want)
        for gw, ww in zip(got, want):
            np.testing.assert_array_equal(gw, ww)
        np.testing.assert_allclose(out[3].cpu().numpy(), d[f'{tag}/obj_cls'], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('mode_name,concurrent,dtype', [
    ('knn', False, 'fp32'), ('radius', False, 'fp32'), ('knn', True, 'fp32'),
    ('radius', True, 'fp32'), ('radius', True, 'fp16')])
def test_pipelined_steps_bit_identical(cuda_device, mode_name, concurrent, dtype):
    """pipeline.PipelinedSteps (graph build of step i on a side stream while step i-1's forward
    runs, two pipelines round robin) gives every step exactly the outputs RadarGNNPipeline.step
    gives the same batch: two different batches alternated over six steps, fp32, kNN and
    radius graphs.  The six steps are enqueued back to back with NO host synchronisation
    (outputs cloned on the device at the reference's sizes, one synchronize at the end), so
    builds and forwards of different steps really overlap; every step's batch is uploaded
    asynchronously from pinned memory on the caller's stream right before the step, so the
    build has to wait for that upload (FrameBatch.ready), not for the previous forward.
    concurrent: each in-flight batch's build and forward on a stream of its own, three
    pipelines (the C5 preset's depth), the caller's stream never waiting on a step, so up to
    three builds + forwards run at once (each step's outputs are copied on its own stream);
    also the fp16 path of BASELINE config 5 (the preset that runs concurrent)."""
    from graph_neural_network_for_radar_perception_amd import _native as nat
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import (PipelinedSteps,
                                                                         RadarGNNPipeline)
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    dev = cuda_device
    cfg = model_cfg('model_trained_N500')
    mt = Model_Training(cfg, dev)
    mt.load_state_dict(model_state_dict('model_trained_N500'))
    m = mt.to(dev).pred.eval()
    mode = nat.GRAPH_KNN if mode_name == 'knn' else nat.GRAPH_RADIUS
    host = []
    for b in range(2):
        frs = [synthetic.make_frame(700 + 50 * f, 4000 + 10 * b + f) for f in range(3)]
        cls = [synthetic.cluster_lists(len(fr['meas_px'])) for fr in frs]
        host.append((frs, cls))
    ref = []
    with torch.no_grad():
        # (the 16-bit conv's wave count is part of its schedule -- a different count moves
        # some sums across its 16-edge aggregation groups -- so the sequential reference
        # uses the one the overlapping pipeline sets)
        from graph_neural_network_for_radar_perception_amd.pipeline import CONCURRENT_CONV_WAVES
        seq = RadarGNNPipeline(m, cfg, dtype, mode=mode, eps2=4.0,
                               conv_waves=CONCURRENT_CONV_WAVES if concurrent else None)
        for frs, cls in host:
            b = FrameBatch.from_frames(frs, cls, device=dev)
            for _ in range(2):
                gb, out = seq.step(b)
            torch.cuda.synchronize()
            ref.append([t.clone() for t in RadarGNNPipeline.trim(gb, out)])
        # concurrent: three pipelines (the C5 preset's depth), so three forwards overlap
        run = PipelinedSteps(m, cfg, dtype, mode=mode, eps2=4.0, concurrent=concurrent,
                             depth=3 if concurrent else 2)
        if mode == nat.GRAPH_RADIUS:
            # each pipeline's first radius build checks its capacity on the host (one sync);
            # warm every pipeline so the six steps below run without any
            for i in range(run.depth):
                run.step(FrameBatch.from_frames(*host[i % 2], device=dev))
            torch.cuda.synchronize()
        got, keep = [], []
        for i in range(6):
            batch = FrameBatch.from_frames(*host[i % 2], device=dev, pinned=True)
            gb, out = run.step(batch)
            U = ref[i % 2][2].shape[0]
            # concurrent: the copies are enqueued on the step's own stream right behind it
            # (in order before that pipeline's next step overwrites its buffers); the caller's
            # stream never waits, so the next upload and step start while this one runs
            ctx = (torch.cuda.stream(run.streams[(run.i - 1) % run.depth]) if concurrent
                   else torch.cuda.stream(torch.cuda.current_stream()))
            with ctx:
                got.append([out.node_cls.clone(), out.node_reg.clone(), out.link_cls[:U].clone(),
                            out.obj_cls.clone(), gb.graph.n_pairs_dev.clone()])
            keep.append(gb)
            del batch                      # freed before its build ran: record_stream keeps it
        torch.cuda.synchronize()
    for i, g in enumerate(got):
        keep[i].check_capacity()
        assert int(g[4].item()) == ref[i % 2][2].shape[0], (mode_name, i)
        for a, b in zip(g[:4], ref[i % 2]):
            assert torch.equal(a, b), (mode_name, i)
