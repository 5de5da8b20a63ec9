"""The C ABI library builds, loads and exports every function include/radar_gnn.h
declares; argument validation works without a GPU (no compute calls here)."""
import ctypes

import pytest

from graph_neural_network_for_radar_perception_amd import _native as nat


@pytest.fixture(scope='module')
def lib():
    from graph_neural_network_for_radar_perception_amd import build
    build.build_library()
    return nat.lib()


def test_every_header_function_exported(lib):
    names = nat.header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
        assert n in nat._SIGNATURES, f'{n} declared in radar_gnn.h but not bound in _native.py'


def test_version(lib):
    assert lib.rg_version() >= 1


def test_packed_sizes(lib):
    # f32: 16-row M tiles x 16-deep k groups x 64 lanes x float4, + bias padded to 16
    assert lib.rg_packed_linear_bytes(6, 256, nat.RG_F32) == 16 * 1 * 64 * 16 + 256 * 4
    # bf16: 16-row M tiles x 32-deep k steps x 64 lanes x 8 bf16, + f32 bias
    assert lib.rg_packed_linear_bytes(192, 128, nat.RG_BF16) == 8 * 6 * 64 * 16 + 128 * 4
    assert lib.rg_packed_linear_bytes(64, 7, nat.RG_BF16) == 1 * 2 * 64 * 16 + 16 * 4


def test_chain_argument_errors_are_reported(lib):
    arr = (nat.rg_layer * 1)()
    rc = lib.rg_mlp_chain(nat.RG_F32, arr, 0, 10, None, 0, 0, None, 0, 0, None, 0, 0, None, 0, 0,
                          None, None, None, 0, 0, None, 0, 0, None)
    assert rc == 1
    assert b'n_layers' in lib.rg_last_error()
    arr[0].w_packed = 16
    arr[0].in_dim, arr[0].out_dim = 300, 8
    rc = lib.rg_mlp_chain(nat.RG_F32, arr, 1, 10, None, 0, 0, 16, 300, 300, None, 0, 0, None, 0, 0,
                          None, None, None, 0, 0, 16, 8, 0, None)
    assert rc == 3
    assert b'outside' in lib.rg_last_error()
    with pytest.raises(RuntimeError, match='rg_mlp_chain'):
        nat.check(rc, 'rg_mlp_chain')


def test_graph_build_argument_errors(lib):
    rc = lib.rg_build_graph(None, None, None, 10, 1, 10, 100, 25.0, 0, None, None, 0, None, None,
                            None, 0, None)
    assert rc == 3 and b'k=100' in lib.rg_last_error()
    rc = lib.rg_build_graph(None, None, None, 10, 1, 10, 10, 25.0, 0, None, None, 0, None, None,
                            None, 0, None)
    assert rc == 1 and b'workspace' in lib.rg_last_error()


def test_segment_reduce_rejects_bad_widths(lib):
    rc = lib.rg_segment_reduce(None, 0, 6, None, None, 4, 6, 0, None, 0, 6, None)
    assert rc == 3


def test_training_backward_argument_errors(lib):
    """The round-6 training entries validate before touching the device: an unsupported
    activation, a dz aliasing its input, a short workspace, and rows <= 0 as a no-op."""
    arr = (nat.rg_layer * 1)()
    arr[0].w_packed = 16
    arr[0].in_dim, arr[0].out_dim = 64, 128
    f = 4096  # any non-null address: nothing is dereferenced before the checks fail
    # relu is not fused (the caller runs the two steps)
    rc = lib.rg_dx_norm_backward(arr, 100, f, 64, f + 64, 128, f, f, nat.ACT['relu'], f + 128,
                                 128, f, f, f, 1 << 20, None)
    assert rc == 3 and b'act' in lib.rg_last_error()
    # dz may not alias dz_next / z
    rc = lib.rg_dx_norm_backward(arr, 100, f, 64, f + 64, 128, f, f, nat.ACT['leakyrelu'], f,
                                 128, f, f, f, 1 << 20, None)
    assert rc == 1 and b'alias' in lib.rg_last_error()
    # workspace shorter than rg_dx_norm_backward_workspace_size(rows)
    need = lib.rg_dx_norm_backward_workspace_size(100000)
    assert need >= 16
    rc = lib.rg_dx_norm_backward(arr, 100000, f, 64, f + 64, 128, f, f, nat.ACT['leakyrelu'],
                                 f + 128, 128, f, f, f, need - 8, None)
    assert rc == 1 and b'workspace' in lib.rg_last_error()
    # no rows: nothing to do
    assert lib.rg_dx_norm_backward(arr, 0, f, 64, f + 64, 128, f, f, nat.ACT['leakyrelu'],
                                   f + 128, 128, f, f, f, 0, None) == 0
    # a gathered ffn backward may not write over the rows it gathers
    rc = lib.rg_ffn_backward_gather(f, 64, f + 64, 64, f, None, 10, 64, 1, f, f, 2, f + 64, 64, f,
                                    f, f, None)
    assert rc == 1 and b'alias' in lib.rg_last_error()
    # a column block of dW narrower than the gradient's input width
    rc = lib.rg_linear_grad_ld(f, 64, 10, 64, 64, nat.IN_DENSE, f, 64, 64, None, 0, 0, None, 0,
                               0, None, None, f, 32, None, f, 1 << 20, None)
    assert rc == 1 and b'ld_dw' in lib.rg_last_error()


def test_workspace_queries(lib):
    assert lib.rg_build_graph_workspace_size(3000, 1, 3000, 10, 0) > 3000 * 94 * 4
    assert lib.rg_link_pairs_workspace_size(100) > 0
    assert lib.rg_csr_by_dst_workspace_size(100, 1000) > 0
    assert lib.rg_pairs_from_edge_index_workspace_size(1000) > 0


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(nat, '_lib', None)
    monkeypatch.setattr(nat, '_load_error', None)
    monkeypatch.setattr(nat, 'LIB_PATH', str(tmp_path / 'nope.so'))
    with pytest.raises(nat.NativeLibraryError):
        nat.lib()


@pytest.mark.timeout(1200)
def test_abi_host_code_under_asan_ubsan():
    """The C ABI's host code -- argument checks, workspace-size arithmetic at the BASELINE
    configurations' sizes and past them, the null / negative / short-workspace /
    unsupported-shape paths -- compiled with AddressSanitizer + UndefinedBehaviorSanitizer
    (host side only) and driven by tests/abi_sanitize_main.cpp; any sanitizer report or failed
    check fails the run.  CPU only: no path it takes reaches a kernel launch."""
    import os
    import subprocess
    from graph_neural_network_for_radar_perception_amd import build
    here = os.path.dirname(os.path.abspath(__file__))
    exe = build.build_sanitized_driver(os.path.join(here, 'abi_sanitize_main.cpp'))
    env = dict(os.environ, ASAN_OPTIONS='abort_on_error=1:detect_leaks=0',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    out = r.stdout + r.stderr
    assert 'AddressSanitizer' not in out and 'runtime error' not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
