"""Seeded synthetic RadarScenes-shaped frames.

The real RadarScenes ``.h5`` data is absent from the reference
(``dataset/RadarScenesData/.MISSING_LARGE_BLOBS``), so every test and benchmark
runs on frames drawn here.  A frame is the dict the reference graph builder
consumes after its grid crop and dynamic filter
(``modules/data_generator/datagen_gnn.py:97-102``):

    meas_px, meas_py, meas_vx, meas_vy, meas_vr, meas_rcs : float32[N]
    meas_timestamp                                        : int64[N]  (µs)

plus generator-side ground truth used by the training path
(``cluster_id`` int64[N], cluster centres) and the object-head cluster lists.

Layout (frame f uses ``np.random.default_rng(seed0 + f)``, seed0 = 1234 =
``configuration_radarscenes_gnn.yml:2``):
  * 70 % of points in Gaussian clusters, sigma = 1 m, mean 12 points per
    cluster, centres uniform in [2, 98] x [-48, 48];
  * 30 % uniform clutter in [0, 100) x [-50, 50);
  * everything clipped into the grid ``configuration_radarscenes_gnn.yml:34-38``;
  * vx, vy, vr ~ N(0, 5) m/s, rcs ~ N(0, 10) dBsm;
  * timestamps = 1e12 + sorted uniform ints in [0, 155000) (10 scans).
"""
from __future__ import annotations

import numpy as np

SEED0 = 1234
GRID_MIN_X, GRID_MAX_X = 0.0, 100.0
GRID_MIN_Y, GRID_MAX_Y = -50.0, 50.0


def make_frame(num_nodes: int, seed: int = SEED0, lattice: bool = False) -> dict:
    """One synthetic frame with ``num_nodes`` measurements.

    ``lattice=True`` places the points on an integer lattice (maximal distance
    ties) -- used to document the reference's implementation-defined kNN tie
    order (SURVEY.md §7 "Bit-exact edge_index").
    """
    rng = np.random.default_rng(seed)
    n = int(num_nodes)
    if lattice:
        side = int(np.ceil(np.sqrt(n)))
        ii = np.arange(n)
        px = (ii % side).astype(np.float32) + 10.0
        py = (ii // side).astype(np.float32) - 10.0
        cluster_id = np.arange(n, dtype=np.int64) // 5
    else:
        n_clu = int(round(0.7 * n))
        n_bg = n - n_clu
        n_clusters = max(1, int(round(n_clu / 12.0)))
        centres = np.stack([rng.uniform(2.0, 98.0, n_clusters),
                            rng.uniform(-48.0, 48.0, n_clusters)], axis=-1)
        cid = rng.integers(0, n_clusters, n_clu)
        pts_c = centres[cid] + rng.normal(0.0, 1.0, (n_clu, 2))
        pts_b = np.stack([rng.uniform(GRID_MIN_X, GRID_MAX_X, n_bg),
                          rng.uniform(GRID_MIN_Y, GRID_MAX_Y, n_bg)], axis=-1)
        pts = np.concatenate([pts_c, pts_b], axis=0)
        cluster_id = np.concatenate([cid, n_clusters + np.arange(n_bg)]).astype(np.int64)
        # shuffle so that node order carries no spatial structure
        perm = rng.permutation(n)
        pts = pts[perm]
        cluster_id = cluster_id[perm]
        hi_x = np.nextafter(np.float32(GRID_MAX_X), np.float32(0.0))
        hi_y = np.nextafter(np.float32(GRID_MAX_Y), np.float32(0.0))
        px = np.clip(pts[:, 0], GRID_MIN_X, hi_x).astype(np.float32)
        py = np.clip(pts[:, 1], GRID_MIN_Y, hi_y).astype(np.float32)
    vx = rng.normal(0.0, 5.0, n).astype(np.float32)
    vy = rng.normal(0.0, 5.0, n).astype(np.float32)
    vr = rng.normal(0.0, 5.0, n).astype(np.float32)
    rcs = rng.normal(0.0, 10.0, n).astype(np.float32)
    ts = (np.int64(10**12) + np.sort(rng.integers(0, 155000, n))).astype(np.int64)
    return {
        'meas_px': px, 'meas_py': py, 'meas_vx': vx, 'meas_vy': vy,
        'meas_vr': vr, 'meas_rcs': rcs, 'meas_timestamp': ts,
        'cluster_id': cluster_id,
    }


def make_batch(num_frames: int, num_nodes: int, seed0: int = SEED0) -> list:
    """``num_frames`` frames, frame f seeded with ``seed0 + f`` (§8(d))."""
    return [make_frame(num_nodes, seed0 + f) for f in range(num_frames)]


def cluster_lists(num_nodes: int, group: int = 5) -> list:
    """Object-head cluster lists: consecutive groups of ``group`` nodes (§8(d))."""
    return [np.arange(s, min(s + group, num_nodes), dtype=np.int64)
            for s in range(0, num_nodes, group)]


def other_features(frame: dict) -> np.ndarray:
    """(px, py, vx, vy) per node, ``datagen_gnn.py:110-111``."""
    return np.stack((frame['meas_px'], frame['meas_py'],
                     frame['meas_vx'], frame['meas_vy']), axis=-1).astype(np.float32)


def make_labels(frame: dict, edge_index: np.ndarray, num_classes: int = 7, seed: int = SEED0):
    """Synthetic training labels of one frame in the reference's label layout
    (``datagen_gnn.py:126-139``), from the generator's cluster ids:

      node_class       int64 [N]   class of the node's cluster; clutter (single-point
                                   clusters) gets the last class ('FALSE')
      node_offsets     f32 [N, 2]  cluster centre - point (raw metres; the model
                                   normalises them, compute_offsets.py:6-11)
      edge_class       int64 [U]   link pairs (i < j, row-major = nonzero(triu(adj, 1)),
                                   compute_edge_labels.py:7-20): 1 if both ends are in
                                   the same real cluster
      cluster_node_idx list of int64 member lists of the real clusters (ascending,
                                   clusters ordered by their lowest member)
      cluster_labels   int64 [Ncl] class of each listed cluster
    """
    rng = np.random.default_rng(seed)
    cid = np.asarray(frame['cluster_id'], np.int64)
    n = cid.shape[0]
    px = frame['meas_px'].astype(np.float64)
    py = frame['meas_py'].astype(np.float64)
    ids, inv, counts = np.unique(cid, return_inverse=True, return_counts=True)
    real = counts[inv] > 1
    cls_of = rng.integers(0, num_classes - 1, ids.shape[0])
    node_class = np.where(real, cls_of[inv], num_classes - 1).astype(np.int64)
    cx = np.bincount(inv, px) / counts
    cy = np.bincount(inv, py) / counts
    node_offsets = np.stack((cx[inv] - px, cy[inv] - py), -1).astype(np.float32)
    ei = np.asarray(edge_index)
    m = ei[0] < ei[1]
    s, d = ei[0][m], ei[1][m]
    edge_class = ((cid[s] == cid[d]) & real[s]).astype(np.int64)
    firsts = {}
    for i in range(n):
        if real[i]:
            firsts.setdefault(int(inv[i]), []).append(i)
    groups = sorted(firsts.values(), key=lambda g: g[0])
    cluster_node_idx = [np.asarray(g, np.int64) for g in groups]
    cluster_labels = np.asarray([cls_of[inv[g[0]]] for g in groups], np.int64)
    return {'node_class': node_class, 'node_offsets': node_offsets, 'edge_class': edge_class,
            'cluster_node_idx': cluster_node_idx, 'cluster_labels': cluster_labels}


def batch_labels(frames: list, row_ptr: np.ndarray, col: np.ndarray, num_classes: int = 7):
    """make_labels for every frame of a batch whose disjoint-union CSR (global node ids,
    rows / columns ascending = np.where order) is row_ptr / col: the labels concatenated
    (edge_class in link-pair order, frame by frame) and the per-frame cluster lists."""
    out = {k: [] for k in ('node_class', 'node_offsets', 'edge_class', 'cluster_labels')}
    clusters = []
    base = 0
    for f, fr in enumerate(frames):
        n = fr['meas_px'].shape[0]
        r = np.repeat(np.arange(n), np.diff(row_ptr[base:base + n + 1]))
        c = col[row_ptr[base]:row_ptr[base + n]] - base
        lb = make_labels(fr, np.stack((r, c)), num_classes, f)
        for k in out:
            out[k].append(lb[k])
        clusters.append(lb['cluster_node_idx'])
        base += n
    return {k: np.concatenate(v) for k, v in out.items()}, clusters


def make_objects(num_objects: int, seed: int = SEED0, min_size: int = 2, max_size: int = 24,
                 num_classes: int = 7) -> dict:
    """A synthetic classifier sample (the per-object features of
    datagen_classifier.extract_and_compute_features_and_labels, datagen_classifier.py:62-100):
    for each object, measurements centred on their mean and expressed in the covariance's
    eigenbasis, as (x, y, r = |xy|, th = atan2(y, x), rcs); object sizes >=
    valid_cluster_num_meas_thr (2, configuration_radarscenes_classifier.yml:7); labels
    uniform over the classes.  Returns float32 node_features [N, 5], int64 object_size
    [n_obj], int64 object_class [n_obj]."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(min_size, max_size + 1, num_objects).astype(np.int64)
    feats = []
    for n in sizes:
        ext = rng.uniform(0.3, 2.5, 2)
        xy = rng.normal(0.0, 1.0, (int(n), 2)) * ext
        xy -= xy.mean(0)
        r = np.sqrt(xy[:, 0] ** 2 + xy[:, 1] ** 2)
        th = np.arctan2(xy[:, 1], xy[:, 0])
        rcs = rng.normal(0.0, 10.0, int(n))
        feats.append(np.stack((xy[:, 0], xy[:, 1], r, th, rcs), -1))
    return {'node_features': np.concatenate(feats, 0).astype(np.float32),
            'object_size': sizes,
            'object_class': rng.integers(0, num_classes, num_objects).astype(np.int64)}


def make_scan_window(seed: int, n_scans: int = 10, mean_meas: int = 160) -> dict:
    """A window of radar scans with RadarScenes field names and dtypes (the inputs of
    read_data.extract_and_sync_radar_data, read_data.py:227-303): per measurement
    x_cc, y_cc, azimuth_sc, vr, vr_compensated, rcs (f32), timestamp (int64 us),
    track_id (bytes, b'' = no track) + its integer key, sensor_id, label_id (old ids
    0..11, labels.py:44-58); per scan the radar mount (x, y, yaw) and the odometry
    (x_seq, y_seq, yaw_seq, vx, yaw_rate) as float64.  Static returns carry the range
    rate the ego motion predicts (plus noise) so the stationary gate sees both classes."""
    rng = np.random.default_rng(seed)
    mounts = np.array([[3.66, -0.64, -1.48], [3.86, -0.70, -0.09],
                       [3.86, 0.74, 0.09], [3.66, 0.68, 1.48]])  # 4 corner radars
    sizes = rng.integers(mean_meas // 2, mean_meas * 3 // 2, n_scans)
    ptr = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    N = int(ptr[-1])
    out = {k: np.zeros(N, np.float32) for k in ('x_cc', 'y_cc', 'azimuth_sc', 'vr',
                                                'vr_compensated', 'rcs')}
    out['timestamp'] = np.zeros(N, np.int64)
    out['sensor_id'] = np.zeros(N, np.int64)
    out['label_id'] = np.zeros(N, np.int64)
    out['track_key'] = np.zeros(N, np.int64)
    tid = np.zeros(N, dtype='S8')
    mount = np.zeros((n_scans, 3))
    odo = np.zeros((n_scans, 5))
    x, y, yaw = rng.uniform(-50, 50), rng.uniform(-50, 50), rng.uniform(-np.pi, np.pi)
    t0 = 10 ** 12
    for s in range(n_scans):
        sid = int(rng.integers(1, 5))
        tx, ty, myaw = mounts[sid - 1]
        vx_e, yr = rng.uniform(2, 15), rng.uniform(-0.2, 0.2)
        mount[s] = (tx, ty, myaw)
        odo[s] = (x, y, yaw, vx_e, yr)
        a, b = int(ptr[s]), int(ptr[s + 1])
        n = b - a
        az = rng.uniform(-1.3, 1.3, n)
        r = rng.uniform(1.0, 90.0, n)
        # sensor-frame ego velocity (meas_selection.py:22-34) and the static range rate
        vxs, vys = vx_e - yr * ty, 0.0 + yr * tx
        c, sn = np.cos(-myaw), np.sin(-myaw)
        vxs, vys = vxs * c - vys * sn, vxs * sn + vys * c
        vr_static = -(vxs * np.cos(az) + vys * np.sin(az))
        moving = rng.random(n) < 0.35
        vr = np.where(moving, vr_static + rng.normal(0, 6, n), vr_static + rng.normal(0, 0.5, n))
        out['azimuth_sc'][a:b] = az
        out['vr'][a:b] = vr
        out['vr_compensated'][a:b] = vr - vr_static
        out['x_cc'][a:b] = tx + r * np.cos(az + myaw)
        out['y_cc'][a:b] = ty + r * np.sin(az + myaw)
        out['rcs'][a:b] = rng.normal(0, 10, n)
        out['timestamp'][a:b] = t0 + s * 15500 + rng.integers(0, 200)
        out['sensor_id'][a:b] = sid
        tracked = moving & (rng.random(n) < 0.8)
        keys = np.where(tracked, rng.integers(1, 9, n), 0)
        out['track_key'][a:b] = keys
        tid[a:b] = [b'' if k == 0 else b'trk%d' % k for k in keys]
        out['label_id'][a:b] = np.where(tracked, rng.integers(0, 11, n), 11)
        # ego motion to the next scan (~15.5 ms)
        dt = 0.0155
        x += vx_e * dt * np.cos(yaw)
        y += vx_e * dt * np.sin(yaw)
        yaw += yr * dt
    out.update(n_scans=n_scans, scan_ptr=ptr, mount=mount, odometry=odo, track_id_bytes=tid)
    return out
