"""Golden fixtures of the real-data front-end made by the REFERENCE.

Runs only in the build container, where /root/reference exists (never on the GPU box;
nothing in tests/ imports this file).  ``modules/data_utils/read_data.py`` imports h5py
(absent) and reads the RadarScenes .h5 files (absent), so the window of radar scans is
synthetic (``synthetic.make_scan_window``: RadarScenes field names and dtypes); every
function applied to it is the reference's own, in the order of
``read_data.extract_and_sync_radar_data`` (read_data.py:227-303), ``extract_frame``
(:442-486) and ``datagen_gnn.RadarScenesDataset.__getitem__`` (datagen_gnn.py:96-102):

  identify_stationary_measurements (meas_selection.py:169-200, gating; ransac off as in
  configuration_radarscenes_gnn.yml:11), vr_cartesian_vf (meas_sync.py:15-20),
  ego_compensate_radar_frames_list (meas_sync.py:74-103), the concatenation and float32
  casts of convert_list_ndarry_to_ndarray / extract_frame, compute_ground_truth
  (compute_node_labels.py:89-105), grid_properties.select_meas_within_the_grid
  (grid_features.py:162-174, GRID_LIMITS of the yml) and select_moving_data
  (graph_features.py:167-182).

Usage:  python tests/golden/make_frontend_golden.py   (writes tests/golden/frontend_*.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from graph_neural_network_for_radar_perception_amd import synthetic  # noqa: E402
from modules.compute_features.graph_features import select_moving_data  # noqa: E402
from modules.compute_features.grid_features import grid_properties  # noqa: E402
from modules.compute_groundtruth.compute_node_labels import compute_ground_truth  # noqa: E402
from modules.data_utils.labels import (compute_new_labels_to_id_dict,  # noqa: E402
                                       compute_old_to_new_label_id_map)
from modules.data_utils.meas_selection import identify_stationary_measurements  # noqa: E402
from modules.data_utils.meas_sync import (ego_compensate_radar_frames_list,  # noqa: E402
                                          vr_cartesian_vf)


def reference_frame(win):
    """The reference's front-end on one window (dict from synthetic.make_scan_window)."""
    px_l, py_l, vx_l, vy_l, vr_l, rcs_l, ts_l, tid_l, sid_l, st_l, lab_l = ([] for _ in range(11))
    ex, ey, eyaw = [], [], []
    for s in range(win['n_scans']):
        a, b = win['scan_ptr'][s], win['scan_ptr'][s + 1]
        m = win['mount'][s]
        od = win['odometry'][s]
        st = identify_stationary_measurements(win['azimuth_sc'][a:b], win['vr'][a:b],
                                              float(m[0]), float(m[1]), float(m[2]),
                                              np.float64(od[3]), np.float64(od[4]), False)
        st_l.append(st)
        ex.append(np.float64(od[0]))
        ey.append(np.float64(od[1]))
        eyaw.append(np.float64(od[2]))
        px_l.append(win['x_cc'][a:b])
        py_l.append(win['y_cc'][a:b])
        vx, vy = vr_cartesian_vf(win['vr_compensated'][a:b], win['azimuth_sc'][a:b], float(m[2]))
        vx_l.append(vx)
        vy_l.append(vy)
        vr_l.append(win['vr_compensated'][a:b])
        rcs_l.append(win['rcs'][a:b])
        ts_l.append(win['timestamp'][a:b])
        tid_l.append(win['track_id_bytes'][a:b])
        sid_l.append(win['sensor_id'][a:b])
        lab_l.append(win['label_id'][a:b])
    px_l, py_l, vx_l, vy_l = ego_compensate_radar_frames_list(px_l, py_l, vx_l, vy_l, ex, ey, eyaw)
    cat = np.concatenate
    d = {'meas_px': cat(px_l).astype(np.float32), 'meas_py': cat(py_l).astype(np.float32),
         'meas_vx': cat(vx_l).astype(np.float32), 'meas_vy': cat(vy_l).astype(np.float32),
         'meas_vr': cat(vr_l).astype(np.float32), 'meas_rcs': cat(rcs_l).astype(np.float32),
         'meas_timestamp': cat(ts_l), 'meas_trackid': cat(tid_l), 'meas_sensorid': cat(sid_l),
         'stationary_meas_flag': cat(st_l), 'meas_label_id': cat(lab_l)}
    full = {k: v.copy() for k, v in d.items()}
    labels_to_id = compute_new_labels_to_id_dict()
    gt = compute_ground_truth(d, labels_to_id, compute_old_to_new_label_id_map())
    full_gt = {k: v.copy() for k, v in gt.items()}
    grid = grid_properties(0, 100, -50, 50, 0.5, 2, 0.5, 2, 0.5, 0.5)  # yml:34-44
    d, gt = grid.select_meas_within_the_grid(d, gt)
    dd, gd = select_moving_data(d, gt, labels_to_id)
    return full, full_gt, dd, gd


def main():
    cases = {'frontend_w10': dict(seed=7, n_scans=10), 'frontend_w4': dict(seed=11, n_scans=4),
             'frontend_w1': dict(seed=13, n_scans=1)}
    for name, kw in cases.items():
        win = synthetic.make_scan_window(**kw)
        full, full_gt, dd, gd = reference_frame(win)
        out = {f'in/{k}': v for k, v in win.items() if k != 'track_id_bytes'}
        out.update({f'full/{k}': v for k, v in full.items() if k != 'meas_trackid'})
        out.update({f'full_gt/{k}': v for k, v in full_gt.items()})
        out.update({f'dyn/{k}': v for k, v in dd.items() if k != 'meas_trackid'})
        out.update({f'dyn_gt/{k}': v for k, v in gd.items()})
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **out)
        print(name, 'scans', win['n_scans'], 'meas', len(full['meas_px']), 'dynamic',
              len(dd['meas_px']), 'stationary', int(full['stationary_meas_flag'].sum()))


if __name__ == '__main__':
    main()
