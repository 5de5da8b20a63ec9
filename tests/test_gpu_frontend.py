"""Real-data front-end on the GPU against the reference's own
outputs (tests/golden/frontend_*.npz, tests/golden/make_frontend_golden.py).

Tolerances: stationary flags, class labels and the dynamic selection exact (no fixture
measurement lies within 1e-4 of the gate, checked); ego-compensated positions exact in
float32 (the float64 transform differs from numpy's LU inverse / BLAS only in the last f64
bits); vx, vy within 2 float32 ulps (device cosf / sinf vs numpy's float32 cos / sin);
offsets within 2e-5 (float64 track means vs numpy's float32 pairwise means)."""
import numpy as np
import pytest
import torch

from conftest import golden, golden_names
from oracle import frontend_ref

pytestmark = pytest.mark.gpu
NAMES = golden_names('frontend_')


def _window(d):
    w = {k[3:]: d[k] for k in d.files if k.startswith('in/')}
    w['n_scans'] = int(w['n_scans'])
    return w


def _ulps(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


@pytest.mark.parametrize('name', NAMES)
def test_frontend_matches_reference(cuda_device, name):
    from graph_neural_network_for_radar_perception_amd import frontend
    d = golden(name)
    w = _window(d)
    win = frontend.ScanWindow.from_numpy(w, cuda_device)
    full = frontend.extract_and_sync_radar_data(win)
    # no measurement near the gate threshold (else a 1-ulp cos difference could flip it)
    ptr, odo, mount = w['scan_ptr'], w['odometry'], w['mount']
    for s in range(w['n_scans']):
        a, b = int(ptr[s]), int(ptr[s + 1])
        tx, ty, th = (float(v) for v in mount[s])
        vxs = np.float64(odo[s][3]) - np.float64(odo[s][4]) * ty
        vys = 0.0 + np.float64(odo[s][4]) * tx
        vxs, vys = vxs * np.cos(-th) - vys * np.sin(-th), vxs * np.sin(-th) + vys * np.cos(-th)
        err = -(vxs * np.cos(w['azimuth_sc'][a:b].astype(np.float64)) +
                vys * np.sin(w['azimuth_sc'][a:b].astype(np.float64))) - w['vr'][a:b]
        assert np.all(np.abs(np.abs(err) - 1.5) > 1e-4)
    np.testing.assert_array_equal(full['stationary_meas_flag'].cpu().numpy(),
                                  d['full/stationary_meas_flag'])
    for k in ('meas_px', 'meas_py'):
        np.testing.assert_array_equal(full[k].cpu().numpy(), d['full/' + k], err_msg=k)
    for k in ('meas_vx', 'meas_vy'):
        assert _ulps(full[k].cpu().numpy(), d['full/' + k]).max() <= 2, k
    gt = frontend.compute_ground_truth(full)
    np.testing.assert_array_equal(gt['class_labels'].cpu().numpy(), d['full_gt/class_labels'])
    for k in ('offsetx', 'offsety'):
        np.testing.assert_allclose(gt[k].cpu().numpy(), d['full_gt/' + k], rtol=0, atol=2e-5)
    dd, gd = frontend.select_dynamic(full, gt)
    for k in ('meas_px', 'meas_py', 'meas_timestamp'):
        np.testing.assert_array_equal(dd[k].cpu().numpy(), d['dyn/' + k], err_msg=k)
    np.testing.assert_array_equal(gd['class_labels'].cpu().numpy(), d['dyn_gt/class_labels'])


def test_frontend_feeds_graph_build(cuda_device):
    """The dynamic frame goes straight into the graph build: same adjacency as the
    reference graph build on the reference's dynamic frame."""
    from graph_neural_network_for_radar_perception_amd import frontend
    from graph_neural_network_for_radar_perception_amd import graph_features as gf
    from oracle import graph_features_ref as gref
    d = golden('frontend_w10')
    win = frontend.ScanWindow.from_numpy(_window(d), cuda_device)
    dd, _ = frontend.dynamic_frame(win)
    fr = {k: v.cpu().numpy() for k, v in dd.items()}
    got = gf.compute_adjacency_information(fr, 25.0, 10)
    want = gref.compute_adjacency_information({'meas_px': d['dyn/meas_px'],
                                               'meas_py': d['dyn/meas_py']}, 25.0, 10)
    np.testing.assert_array_equal(got['adj_list'], want['adj_list'])


RANSAC = golden_names('ransac_')


@pytest.mark.parametrize('name', RANSAC)
def test_frontend_ransac_matches_reference(cuda_device, name):
    """RANSAC stationary rejection (meas_selection.py:96-166) with numpy's global generator
    seeded as the fixture's was (tests/golden/make_ransac_golden.py): the device flags, each
    scan's inlier ratio and validity equal the reference's, and the host's draws leave the
    generator exactly where the reference's left it.  Exact: the ratios are inlier counts,
    and no fixture measurement's error lies within 1e-5 of the margin under the chosen fit
    (tests/test_frontend_ransac_oracle.py), where a last-place cos / sin difference could
    move a decision."""
    from graph_neural_network_for_radar_perception_amd import frontend
    d = golden(name)
    w = _window(d)
    win = frontend.ScanWindow.from_numpy(w, cuda_device)
    np.random.seed(int(d['rng_seed']))
    full = frontend.extract_and_sync_radar_data(win, reject_outlier_by_ransac=True)
    after = np.random.get_state()[1].copy()
    np.random.seed(int(d['rng_seed']))
    ref = frontend_ref.sync_window(w, reject_outlier_by_ransac=True)
    np.testing.assert_array_equal(np.random.get_state()[1], after)
    np.testing.assert_array_equal(ref['stationary_meas_flag'], d['stationary'])
    np.testing.assert_array_equal(full['stationary_meas_flag'].cpu().numpy(), d['stationary'])
    ratio, valid = full['_ransac']
    np.testing.assert_array_equal(ratio.cpu().numpy(), d['in_ratio'])
    np.testing.assert_array_equal(valid.cpu().numpy(), d['is_valid'])


def test_frontend_ransac_batch_of_windows(cuda_device):
    """Every RANSAC fixture's window in ONE batch, the generator seeded once: the draws run
    window after window, scan after scan, as the reference's loop over windows would; the
    flags equal the oracle's over the same seeded sequence (the oracle is pinned to the
    fixtures above), and the whole dynamic frame follows."""
    from graph_neural_network_for_radar_perception_amd import frontend
    ws = [_window(golden(n)) for n in RANSAC]
    win = frontend.scan_window_batch(ws, cuda_device)
    np.random.seed(2024)
    full = frontend.extract_and_sync_radar_data(win, reject_outlier_by_ransac=True)
    np.random.seed(2024)
    want = np.concatenate([frontend_ref.sync_window(w, reject_outlier_by_ransac=True)
                           ['stationary_meas_flag'] for w in ws])
    np.testing.assert_array_equal(full['stationary_meas_flag'].cpu().numpy(), want)
    np.random.seed(2024)
    dd, gd = frontend.dynamic_frame(win, reject_outlier_by_ransac=True)
    assert int(dd['frame_ptr'][-1]) == len(dd['meas_px'])


def test_frontend_batch_of_windows(cuda_device):
    """All fixtures' windows as ONE batch (per-window current scan and track ids): each
    window's dynamic frame (frame_ptr range) equals its reference frame."""
    from graph_neural_network_for_radar_perception_amd import frontend
    ds = [golden(n) for n in NAMES]
    win = frontend.scan_window_batch([_window(d) for d in ds], cuda_device)
    dd, gd = frontend.dynamic_frame(win)
    fp = dd['frame_ptr'].cpu().numpy()
    assert len(fp) == len(ds) + 1 and fp[0] == 0 and fp[-1] == len(dd['meas_px'])
    for w, d in enumerate(ds):
        a, b = fp[w], fp[w + 1]
        for k in ('meas_px', 'meas_py', 'meas_timestamp'):
            np.testing.assert_array_equal(dd[k][a:b].cpu().numpy(), d['dyn/' + k], err_msg=k)
        np.testing.assert_array_equal(gd['class_labels'][a:b].cpu().numpy(),
                                      d['dyn_gt/class_labels'])
        np.testing.assert_allclose(gd['offsetx'][a:b].cpu().numpy(), d['dyn_gt/offsetx'],
                                   rtol=0, atol=2e-5)


def test_frontend_ransac_edge_scans(cuda_device):
    """RANSAC over a window with an empty scan, a scan of exactly RANSAC_MIN_MEAS + 1 gated
    measurements (the smallest that draws) and ordinary scans, against the oracle (pinned to
    the reference's fixtures) over the same seeded generator: flags, ratios and the
    generator's final state equal."""
    from graph_neural_network_for_radar_perception_amd import frontend, synthetic
    w = synthetic.make_scan_window(seed=31, n_scans=5, mean_meas=40)
    ptr = np.asarray(w['scan_ptr']).copy()
    # scan 1 emptied: its measurements move to scan 2 (both keep scan 2's pose)
    ptr[2] = ptr[1]
    w['scan_ptr'] = ptr
    # scan 3 cut to its first gated measurements: keep min_meas + 1 of them
    a, b = int(ptr[3]), int(ptr[4])
    m, od = w['mount'][3], w['odometry'][3]
    gate = frontend_ref.stationary_flag(w['azimuth_sc'][a:b], w['vr'][a:b], *(float(v) for v in m),
                                        np.float64(od[3]), np.float64(od[4]))
    idx = np.flatnonzero(gate)
    assert len(idx) > frontend_ref.RANSAC_MIN_MEAS + 1
    cut = a + int(idx[frontend_ref.RANSAC_MIN_MEAS]) + 1   # exactly min_meas + 1 gated
    drop = np.arange(cut, b)
    for k in list(w):
        v = w[k]
        if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == int(ptr[-1]):
            w[k] = np.delete(v, drop, axis=0)
    ptr[4:] -= len(drop)
    w['scan_ptr'] = ptr
    win = frontend.ScanWindow.from_numpy(w, cuda_device)
    np.random.seed(77)
    full = frontend.extract_and_sync_radar_data(win, reject_outlier_by_ransac=True)
    after = np.random.get_state()[1].copy()
    np.random.seed(77)
    ref = frontend_ref.sync_window(w, reject_outlier_by_ransac=True)
    np.testing.assert_array_equal(np.random.get_state()[1], after)
    np.testing.assert_array_equal(full['stationary_meas_flag'].cpu().numpy(),
                                  ref['stationary_meas_flag'])
    ratio = full['_ransac'][0].cpu().numpy()
    assert ratio[1] == 0.0 and ratio[3] > 0.0
