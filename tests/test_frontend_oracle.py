"""Front-end oracle (oracle/frontend_ref.py) against the reference's own outputs
(tests/golden/frontend_*.npz, made by tests/golden/make_frontend_golden.py).

Bit-exact: stationary flags, class labels, the dynamic selection (indices) and every
float32 output of the sync step; offsets (numpy float32 means in both) bit-exact too."""
import numpy as np
import pytest

from conftest import golden, golden_names
from oracle import frontend_ref

NAMES = golden_names('frontend_')


def window(d):
    w = {k[3:]: d[k] for k in d.files if k.startswith('in/')}
    w['n_scans'] = int(w['n_scans'])
    return w


@pytest.mark.parametrize('name', NAMES)
def test_frontend_oracle_matches_reference(name):
    d = golden(name)
    w = window(d)
    full = frontend_ref.sync_window(w)
    for k in ('meas_px', 'meas_py', 'meas_vx', 'meas_vy', 'meas_vr', 'meas_rcs',
              'meas_timestamp', 'stationary_meas_flag', 'meas_label_id'):
        np.testing.assert_array_equal(full[k], d['full/' + k], err_msg=k)
    gt = frontend_ref.ground_truth(full, w['track_key'])
    for k in ('class_labels', 'offsetx', 'offsety'):
        np.testing.assert_array_equal(gt[k], d['full_gt/' + k], err_msg=k)
    dd, gd = frontend_ref.select_dynamic(full, gt)
    for k in ('meas_px', 'meas_py', 'meas_vx', 'meas_vy', 'meas_timestamp'):
        np.testing.assert_array_equal(dd[k], d['dyn/' + k], err_msg=k)
    np.testing.assert_array_equal(gd['class_labels'], d['dyn_gt/class_labels'])
    assert 0 < len(dd['meas_px']) < len(full['meas_px'])
    assert 0 < full['stationary_meas_flag'].sum() < len(full['meas_px'])
