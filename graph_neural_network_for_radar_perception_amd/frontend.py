"""Real-data front-end on the GPU: a window of radar scans in HBM
-> the dynamic radar frame the graph build consumes.

Mirrors, for arrays already read from the RadarScenes .h5 files (that I/O stays on the
host), the reference sequence

  read_data.extract_and_sync_radar_data + extract_frame   (read_data.py:227-303, 442-486)
  compute_node_labels.compute_ground_truth                (compute_node_labels.py:89-105)
  grid_properties.select_meas_within_the_grid             (grid_features.py:162-174)
  graph_features.select_moving_data                       (graph_features.py:167-182)

as three native launches (``rg_frontend_sync``, ``rg_frontend_labels``,
``rg_frontend_select``, csrc/frontend.hip) plus one gather of the selected rows.  With
``reject_outlier_by_ransac=True`` (off in configuration_radarscenes_gnn.yml:11) the gate is
followed by the RANSAC rejection of meas_selection.py:96-166: the host draws the consensus
sets exactly as the reference does -- ``np.random.shuffle`` on numpy's global generator,
scans in window order -- and ``rg_frontend_gate_lists`` / ``rg_frontend_ransac`` evaluate
every set on the device, so a seeded generator reproduces the reference's flags.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch

from . import _native as nat
from .engine import _require_device

GAMMA_STATIONARY = 1.5            # data_utils/constants.py:15
LABEL_STATIC = 7                  # labels.py:60-70
GRID_LIMITS = (0.0, 100.0, -50.0, 50.0)   # configuration_radarscenes_gnn.yml:34-38
RANSAC_MIN_SAMPLES, RANSAC_MARGIN, RANSAC_ITERS = 2, 0.25, 30   # data_utils/constants.py:8-10
RANSAC_RATIO, RANSAC_MIN_MEAS = 0.6, 10                         # constants.py:11-12
# labels.py:90-100: old label ids 0..11 -> new ids
OLD_TO_NEW = np.array([0, 4, 4, 4, 4, 3, 3, 1, 2, 5, 5, 7], dtype=np.int32)


class ScanWindow:
    """A window of scans on the device: per measurement x_cc, y_cc, azimuth_sc, vr,
    vr_compensated, rcs (f32), timestamp (int64), sensor_id, label_id (int64), track key
    (int32: 0 = the empty track id b''); per scan mount (x, y, yaw) and odometry
    (x_seq, y_seq, yaw_seq, vx, yaw_rate), float64."""

    FIELDS = ('x_cc', 'y_cc', 'azimuth_sc', 'vr', 'vr_compensated', 'rcs')

    def __init__(self, arrays: Dict[str, torch.Tensor], scan_ptr: torch.Tensor,
                 mount: torch.Tensor, odometry: torch.Tensor, track_key: torch.Tensor,
                 n_tracks: int, scan_ref: torch.Tensor = None, win_ptr: torch.Tensor = None):
        """A batch of windows (from_numpy_batch) adds scan_ref (int32 [n_scans]: the
        current scan of each scan's window) and win_ptr (int32 [n_windows + 1]: each
        window's measurement range)."""
        self.arrays, self.scan_ptr, self.mount, self.odometry = arrays, scan_ptr, mount, odometry
        self.track_key, self.n_tracks = track_key, n_tracks
        self.scan_ref, self.win_ptr = scan_ref, win_ptr
        self.n_scans = int(mount.shape[0])
        self.n_meas = int(arrays['x_cc'].shape[0])
        self.n_windows = 1 if win_ptr is None else int(win_ptr.shape[0]) - 1

    @staticmethod
    def from_numpy(win: dict, device) -> 'ScanWindow':
        """From host arrays (synthetic.make_scan_window layout; ``track_id_bytes`` holds
        the RadarScenes byte-string track ids, or ``track_key`` integer keys)."""
        keys = _host_track_keys(win)
        arr = {k: torch.from_numpy(np.ascontiguousarray(win[k], dtype=np.float32)).to(device)
               for k in ScanWindow.FIELDS}
        arr['timestamp'] = torch.from_numpy(np.asarray(win['timestamp'], np.int64)).to(device)
        arr['sensor_id'] = torch.from_numpy(np.asarray(win['sensor_id'], np.int64)).to(device)
        arr['label_id'] = torch.from_numpy(np.asarray(win['label_id'], np.int64)).to(device)
        i32 = dict(dtype=torch.int32)
        return ScanWindow(
            arr, torch.tensor(np.asarray(win['scan_ptr']), **i32).to(device),
            torch.from_numpy(np.ascontiguousarray(win['mount'], np.float64)).to(device),
            torch.from_numpy(np.ascontiguousarray(win['odometry'], np.float64)).to(device),
            torch.from_numpy(keys.astype(np.int32)).to(device), int(keys.max(initial=0)))


def _host_track_keys(win: dict) -> np.ndarray:
    if 'track_id_bytes' not in win:
        return np.asarray(win['track_key'], dtype=np.int64)
    ids = np.asarray(win['track_id_bytes'])
    uniq, inv = np.unique(ids, return_inverse=True)
    keys = inv.astype(np.int64) + 1                  # 1..n_unique
    if uniq.size and uniq[0] == b'':
        keys -= 1                                    # b'' sorts first: key 0 = no track
    return keys


def scan_window_batch(wins, device) -> ScanWindow:
    """Several windows as ONE device batch (each window keeps its own current scan and
    its own track ids); select_dynamic then returns the graph build's frame_ptr."""
    cat = np.concatenate
    keys, off = [], 0
    for w in wins:
        k = _host_track_keys(w)
        keys.append(np.where(k > 0, k + off, 0))
        off += int(k.max(initial=0))
    scan_ptr, scan_ref, win_ptr, base_m, base_s = [0], [], [0], 0, 0
    for w in wins:
        n_s = int(w['n_scans'])
        scan_ptr += [base_m + int(v) for v in np.asarray(w['scan_ptr'])[1:]]
        scan_ref += [base_s + n_s - 1] * n_s
        base_m += int(np.asarray(w['scan_ptr'])[-1])
        base_s += n_s
        win_ptr.append(base_m)
    merged = {k: cat([np.asarray(w[k]) for w in wins]) for k in ScanWindow.FIELDS +
              ('timestamp', 'sensor_id', 'label_id')}
    merged.update(n_scans=base_s, scan_ptr=np.asarray(scan_ptr), track_key=cat(keys),
                  mount=cat([w['mount'] for w in wins]), odometry=cat([w['odometry'] for w in wins]))
    one = ScanWindow.from_numpy(merged, device)
    i32 = dict(dtype=torch.int32)
    one.scan_ref = torch.tensor(scan_ref, **i32).to(device)
    one.win_ptr = torch.tensor(win_ptr, **i32).to(device)
    one.n_windows = len(wins)
    return one


def extract_and_sync_radar_data(w: ScanWindow, reject_outlier_by_ransac: bool = False) -> dict:
    """extract_frame's data_dict for the window (device tensors): meas_px / py (ego
    compensated into the last scan's frame), meas_vx / vy (vr_cartesian_vf), meas_vr
    (vr_compensated), meas_rcs, meas_timestamp, meas_sensorid, meas_label_id,
    stationary_meas_flag (bool)."""
    a = w.arrays
    _require_device(a['x_cc'], 'x_cc')
    dev = a['x_cc'].device
    n = w.n_meas
    f32 = dict(dtype=torch.float32, device=dev)
    px, py, vx, vy = (torch.empty(n, **f32) for _ in range(4))
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    nat.check(nat.lib().rg_frontend_sync(
        a['x_cc'].data_ptr(), a['y_cc'].data_ptr(), a['azimuth_sc'].data_ptr(),
        a['vr'].data_ptr(), a['vr_compensated'].data_ptr(), w.scan_ptr.data_ptr(), w.n_scans,
        nat.ptr(w.scan_ref), w.mount.data_ptr(), w.odometry.data_ptr(), GAMMA_STATIONARY, n,
        px.data_ptr(),
        py.data_ptr(), vx.data_ptr(), vy.data_ptr(), st.data_ptr(), nat.stream_ptr(dev)),
        'rg_frontend_sync')
    ransac = _ransac(w, st) if reject_outlier_by_ransac and n > 0 else None
    return {'meas_px': px, 'meas_py': py, 'meas_vx': vx, 'meas_vy': vy,
            'meas_vr': a['vr_compensated'], 'meas_rcs': a['rcs'],
            'meas_timestamp': a['timestamp'], 'meas_sensorid': a['sensor_id'],
            'meas_label_id': a['label_id'], 'stationary_meas_flag': st.bool(),
            '_track_key': w.track_key, '_n_tracks': w.n_tracks, '_stationary_u8': st,
            '_win_ptr': w.win_ptr, '_n_windows': w.n_windows, '_ransac': ransac}


def _ransac(w: ScanWindow, st: torch.Tensor):
    """meas_selection.py:96-166 on every scan's gated measurements (st updated in place):
    the device lists each scan's gated measurements, the host draws the consensus sets from
    numpy's global generator in the reference's order (per scan with more than
    RANSAC_MIN_MEAS gated, RANSAC_ITERS np.random.shuffle passes over arange(gated), the
    first RANSAC_MIN_SAMPLES of each -- natively, rg_ransac_consensus_sets, from and back into
    numpy's generator state), the device fits and counts.  Returns the per-scan
    (in_ratio f64, is_valid bool) device tensors.  Synchronises once (the draws need the
    gated counts)."""
    lib = nat.lib()
    a = w.arrays
    dev = a['x_cc'].device
    S = w.n_scans
    stream = nat.stream_ptr(dev)
    i32 = dict(dtype=torch.int32, device=dev)
    gidx = torch.empty(max(w.n_meas, 1), **i32)
    gcnt = torch.empty(S, **i32)
    nat.check(lib.rg_frontend_gate_lists(st.data_ptr(), w.scan_ptr.data_ptr(), S,
                                         gidx.data_ptr(), gcnt.data_ptr(), stream),
              'rg_frontend_gate_lists')
    counts = np.ascontiguousarray(gcnt.cpu().numpy(), dtype=np.int32)
    sets = np.zeros((S, RANSAC_ITERS, RANSAC_MIN_SAMPLES), np.int32)
    # the draws np.random.shuffle would make, from numpy's own generator state, in one native
    # loop (rg_ransac_consensus_sets); the advanced state goes back into numpy
    kind, key, pos, has_gauss, gauss = np.random.get_state()
    key = np.array(key, dtype=np.uint32)
    posa = np.array([pos], dtype=np.int32)
    nat.check(lib.rg_ransac_consensus_sets(key.ctypes.data, posa.ctypes.data, counts.ctypes.data,
                                           S, RANSAC_ITERS, RANSAC_MIN_SAMPLES, RANSAC_MIN_MEAS,
                                           sets.ctypes.data), 'rg_ransac_consensus_sets')
    np.random.set_state((kind, key, int(posa[0]), has_gauss, gauss))
    sets_d = torch.from_numpy(sets).to(dev)
    ratio = torch.empty(S, dtype=torch.float64, device=dev)
    valid = torch.empty(S, dtype=torch.uint8, device=dev)
    nat.check(lib.rg_frontend_ransac(
        a['azimuth_sc'].data_ptr(), a['vr'].data_ptr(), w.scan_ptr.data_ptr(), S, gidx.data_ptr(),
        gcnt.data_ptr(), sets_d.data_ptr(), RANSAC_ITERS, RANSAC_MIN_SAMPLES, RANSAC_MARGIN,
        RANSAC_MIN_MEAS, RANSAC_RATIO, st.data_ptr(), ratio.data_ptr(), valid.data_ptr(), stream),
        'rg_frontend_ransac')
    return ratio, valid.bool()


def compute_ground_truth(d: dict) -> dict:
    """compute_node_labels.compute_ground_truth: class_labels, offsetx, offsety (f32)."""
    lib = nat.lib()
    px = d['meas_px']
    dev = px.device
    n = int(px.shape[0])
    nt = int(d['_n_tracks'])
    f32 = dict(dtype=torch.float32, device=dev)
    cls, ox, oy = (torch.empty(n, **f32) for _ in range(3))
    o2n = torch.from_numpy(OLD_TO_NEW).to(dev)
    ws = torch.empty(lib.rg_frontend_labels_workspace_size(nt), dtype=torch.uint8, device=dev)
    nat.check(lib.rg_frontend_labels(
        d['_track_key'].data_ptr(), nt, d['meas_label_id'].data_ptr(),
        d['_stationary_u8'].data_ptr(), o2n.data_ptr(), int(o2n.numel()), px.data_ptr(),
        d['meas_py'].data_ptr(), n, cls.data_ptr(), ox.data_ptr(), oy.data_ptr(),
        ws.data_ptr(), ws.numel(), nat.stream_ptr(dev)), 'rg_frontend_labels')
    return {'offsetx': ox, 'offsety': oy, 'class_labels': cls}


def select_dynamic(d: dict, gt: dict, grid_limits=GRID_LIMITS) -> Tuple[dict, dict]:
    """select_meas_within_the_grid then select_moving_data, one order-preserving
    compaction (rg_frontend_select) and a gather of every field.  Synchronises once (the
    selected count sizes the outputs, as the reference's boolean indexing does).  For a
    batch of windows the returned data dict also holds 'frame_ptr' (int32, device): the
    dynamic frame of each window, ready for the batched graph build."""
    lib = nat.lib()
    px = d['meas_px']
    dev = px.device
    n = int(px.shape[0])
    idx = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    ws = torch.empty(lib.rg_frontend_select_workspace_size(n), dtype=torch.uint8, device=dev)
    x0, x1, y0, y1 = (float(v) for v in grid_limits)
    wp = d.get('_win_ptr')
    nw = int(d.get('_n_windows', 1))
    fptr = torch.empty(nw + 1, dtype=torch.int32, device=dev) if wp is not None else None
    nat.check(lib.rg_frontend_select(px.data_ptr(), d['meas_py'].data_ptr(),
                                     gt['class_labels'].data_ptr(), n, x0, x1, y0, y1,
                                     float(LABEL_STATIC), nat.ptr(wp), nw, nat.ptr(fptr),
                                     idx.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(),
                                     nat.stream_ptr(dev)), 'rg_frontend_select')
    k = int(cnt.item())
    sel = idx[:k].long()
    dd = {key: v.index_select(0, sel) for key, v in d.items()
          if isinstance(v, torch.Tensor) and not key.startswith('_')}
    gd = {key: v.index_select(0, sel) for key, v in gt.items()}
    if fptr is not None:
        dd['frame_ptr'] = fptr
    return dd, gd


def dynamic_frame(w: ScanWindow, reject_outlier_by_ransac: bool = False) -> Tuple[dict, dict]:
    """The whole front-end for one window: (data_dict_dyn, node_labels_dict_dyn) of
    datagen_gnn.RadarScenesDataset.__getitem__ (datagen_gnn.py:96-102)."""
    d = extract_and_sync_radar_data(w, reject_outlier_by_ransac)
    gt = compute_ground_truth(d)
    return select_dynamic(d, gt)
