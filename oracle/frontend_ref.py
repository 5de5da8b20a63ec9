"""CPU oracle of the real-data front-end -- TEST INFRASTRUCTURE.

Only tests/ may import this module; the product path is csrc/frontend.hip.

A numpy restatement, on a window of scans already in memory (the .h5 reading of
read_data.py stays out of scope: h5py and the data are absent), of
  read_data.extract_and_sync_radar_data + extract_frame (read_data.py:227-303, 442-486):
    identify_stationary_measurements (meas_selection.py:22-70, 169-200): the gate, and
    with ransac=True the RANSAC rejection (:72-166) -- its consensus sets are
    np.random.shuffle draws from numpy's global generator, so a seeded generator makes it
    reproducible (pinned by tests/golden/make_ransac_golden.py -> ransac_*.npz),
    vr_cartesian_vf (meas_sync.py:15-20),
    ego_compensate_radar_frames_list (meas_sync.py:23-103),
    the concatenation and float32 casts;
  compute_ground_truth (compute_node_labels.py:50-105);
  select_meas_within_the_grid (grid_features.py:162-174) + select_moving_data
  (graph_features.py:167-182).
Every expression keeps the reference's numpy dtypes (float32 arrays, np.float64 odometry
scalars, python-float mount parameters).  Pinned to fixtures produced by the reference's
own functions (tests/golden/make_frontend_golden.py -> tests/golden/frontend_*.npz).
"""
from __future__ import annotations

import numpy as np

GAMMA_STATIONARY = 1.5            # data_utils/constants.py:15
LABEL_FALSE, LABEL_STATIC = 6, 7  # labels.py:60-70
GRID = (0, 100, -50, 50)          # configuration_radarscenes_gnn.yml:34-38 (min_x, max_x, min_y, max_y)


def old_to_new_label_map() -> np.ndarray:
    """labels.py:90-100 (old ids 0..11 -> new ids)."""
    # CAR, LARGE_VEHICLE, TRUCK, BUS, TRAIN, BICYCLE, MOTORIZED_TWO_WHEELER, PEDESTRIAN,
    # PEDESTRIAN_GROUP, ANIMAL, OTHER, STATIC
    return np.array([0, 4, 4, 4, 4, 3, 3, 1, 2, 5, 5, 7], dtype=np.int32)


def stationary_flag(az: np.ndarray, vr: np.ndarray, tx: float, ty: float, theta: float,
                    vx_odom: np.float64, yawrate: np.float64) -> np.ndarray:
    """Gate of meas_selection.py:53-70 with the ego velocity at the sensor (:22-34)."""
    vxs = vx_odom - yawrate * ty
    vys = 0.0 + yawrate * tx
    a = -theta
    vxs, vys = vxs * np.cos(a) - vys * np.sin(a), vxs * np.sin(a) + vys * np.cos(a)
    pred = -(vxs * np.cos(az) + vys * np.sin(az))
    return np.abs(pred - vr) <= GAMMA_STATIONARY


RANSAC_MIN_SAMPLES, RANSAC_MARGIN, RANSAC_ITERS = 2, 0.25, 30   # data_utils/constants.py:8-10
RANSAC_RATIO, RANSAC_MIN_MEAS = 0.6, 10                         # constants.py:11-12


def ego_vx_vy(theta: np.ndarray, vr: np.ndarray):
    """Least-squares sensor velocity from (azimuth, range rate) pairs (meas_selection.py:72-
    93): normal equations summed in float64 over float32 cos / sin, solved by inversion."""
    A = np.zeros((2, 2))
    rhs = np.zeros((2, 1))
    for t, v in zip(theta, vr):
        c, sn, s2 = np.cos(t), np.sin(t), np.sin(2 * t)
        A[0, 0] += c ** 2
        A[0, 1] += s2
        rhs[0, 0] -= c * v
        rhs[1, 0] -= sn * v
    A[0, 1] *= 0.5
    A[1, 0] = A[0, 1]
    A[1, 1] = len(theta) - A[0, 0]
    sol = np.linalg.inv(A) @ rhs
    return sol[0, 0], sol[1, 0]


def ransac(z: np.ndarray, with_fit: bool = False):
    """meas_selection.py:96-166 on z = [azimuth, vr] rows (float32): (inlier flags, valid,
    inlier ratio) -- with_fit: + the chosen (vx, vy) and every row's |vr - predicted| under
    it.  Draws RANSAC_ITERS np.random.shuffle permutations (global generator) when there are
    more than RANSAC_MIN_MEAS rows, none otherwise (all flags False)."""
    n = z.shape[0]
    if n <= RANSAC_MIN_MEAS:
        out = (np.zeros(n, dtype=bool), False, 0)
        return out + (None, None) if with_fit else out
    order = np.arange(n)
    fits, counts = [], np.zeros(RANSAC_ITERS)
    for it in range(RANSAC_ITERS):
        np.random.shuffle(order)
        cons, test = z[order[:RANSAC_MIN_SAMPLES]], z[order[RANSAC_MIN_SAMPLES:]]
        vx, vy = ego_vx_vy(cons[:, 0], cons[:, 1])
        pred = -(vx * np.cos(test[:, 0]) + vy * np.sin(test[:, 0]))
        counts[it] = np.sum(np.abs(test[:, 1] - pred) <= RANSAC_MARGIN)
        fits.append((vx, vy))
    best = int(np.argmax(counts))
    vx, vy = fits[best]
    ratio = (counts[best] + RANSAC_MIN_SAMPLES) / n
    pred = -(vx * np.cos(z[:, 0]) + vy * np.sin(z[:, 0]))
    err = np.abs(z[:, 1] - pred)
    out = (err <= RANSAC_MARGIN, bool(ratio >= RANSAC_RATIO), ratio)
    return out + ((vx, vy), err) if with_fit else out


def se2(x, y, th) -> np.ndarray:
    T = np.eye(3)
    T[:2, :2] = [[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]]
    T[:2, 2] = (x, y)
    return T


def sync_window(win: dict, reject_outlier_by_ransac: bool = False) -> dict:
    """Per-measurement arrays of extract_frame for a window (synthetic.make_scan_window
    layout); with RANSAC the scans draw from numpy's global generator in window order."""
    ptr = win['scan_ptr']
    W = int(win['n_scans'])
    mount, odo = win['mount'], win['odometry']
    pose = lambda s: (np.float64(odo[s][0]), np.float64(odo[s][1]), np.float64(odo[s][2]))  # noqa: E731
    xc, yc, thc = pose(W - 1)
    cols = {k: [] for k in ('px', 'py', 'vx', 'vy', 'st')}
    for s in range(W):
        a, b = int(ptr[s]), int(ptr[s + 1])
        tx, ty, yaw = (float(v) for v in mount[s])
        az, vr = win['azimuth_sc'][a:b], win['vr'][a:b]
        gate = stationary_flag(az, vr, tx, ty, yaw, np.float64(odo[s][3]), np.float64(odo[s][4]))
        if reject_outlier_by_ransac:   # meas_selection.py:188-199: inliers among the gated
            inl = ransac(np.stack((az, vr), axis=1)[gate])[0]
            gate = gate.copy()
            gate[np.flatnonzero(gate)] = inl
        cols['st'].append(gate)
        ang = az + yaw                                    # float32 (weak python scalar)
        vrc = win['vr_compensated'][a:b]
        cols['vx'].append(vrc * np.cos(ang))
        cols['vy'].append(vrc * np.sin(ang))
        # T_curr^-1 T_prev of the two SE2 poses (meas_sync.py:23-31, 61-65), applied to the
        # float32 positions in float64
        T = np.linalg.inv(se2(xc, yc, thc)) @ se2(*pose(s))
        pos = T[:2, :2] @ np.stack([win['x_cc'][a:b], win['y_cc'][a:b]]) + T[:2, 2:]
        cols['px'].append(pos[0])
        cols['py'].append(pos[1])
    cat = np.concatenate
    return {'meas_px': cat(cols['px']).astype(np.float32),
            'meas_py': cat(cols['py']).astype(np.float32),
            'meas_vx': cat(cols['vx']).astype(np.float32),
            'meas_vy': cat(cols['vy']).astype(np.float32),
            'meas_vr': win['vr_compensated'].astype(np.float32),
            'meas_rcs': win['rcs'].astype(np.float32),
            'meas_timestamp': win['timestamp'],
            'meas_sensorid': win['sensor_id'],
            'meas_label_id': win['label_id'],
            'stationary_meas_flag': cat(cols['st'])}


def ground_truth(d: dict, track_key: np.ndarray) -> dict:
    """compute_node_labels.py:50-105 with integer track keys (0 = the empty track id)."""
    tracked = track_key > 0
    st = d['stationary_meas_flag']
    cls = np.zeros(len(track_key), np.float32)
    cls[tracked] = old_to_new_label_map()[d['meas_label_id']][tracked]
    cls[~tracked & ~st] = LABEL_FALSE
    cls[~tracked & st] = LABEL_STATIC
    ox = np.zeros(len(track_key), np.float32)
    oy = np.zeros(len(track_key), np.float32)
    for k in np.unique(track_key[tracked]):
        f = track_key == k
        ox[f] = np.mean(d['meas_px'][f]) - d['meas_px'][f]
        oy[f] = np.mean(d['meas_py'][f]) - d['meas_py'][f]
    return {'offsetx': ox, 'offsety': oy, 'class_labels': cls}


def select_dynamic(d: dict, gt: dict):
    """Grid selection then the moving measurements, order preserved."""
    x, y = d['meas_px'], d['meas_py']
    keep = (x >= GRID[0]) & (x < GRID[1]) & (y >= GRID[2]) & (y < GRID[3])
    keep &= gt['class_labels'] != LABEL_STATIC
    return ({k: v[keep] for k, v in d.items()}, {k: v[keep] for k, v in gt.items()})
