"""bench.py's presets and the settings its JSON line reports (CPU only: argument parsing).

The driver runs ``python bench.py`` with no flags: that must be the metric configuration M
(BASELINE.json metric: 64 frames x 3000 nodes, k = 10, L = 7, fp32) with two batches in flight
and no overlapping forwards (its conv spans stay the kernel's own); C5 runs three overlapping
forwards with 1536-wave 16-bit conv launches."""
import sys

import pytest

import bench


def _parse(monkeypatch, *argv):
    monkeypatch.setattr(sys, 'argv', ['bench.py', *argv])
    return bench.parse()


def test_default_is_the_metric_configuration(monkeypatch):
    a = _parse(monkeypatch)
    assert (a.config, a.frames, a.nodes, a.k, a.layers, a.dtype) == ('m', 64, 3000, 10, 7, 'fp32')
    assert a.gpus == 1 and a.streams == 2 and not a.concurrent
    assert bench.conv_waves_of(a) is None      # fp32: the x3 conv, no 16-bit schedule


def test_c5_overlaps_forwards(monkeypatch):
    from graph_neural_network_for_radar_perception_amd import pipeline
    a = _parse(monkeypatch, '--config', 'c5')
    assert (a.frames, a.nodes, a.graph, a.dtype) == (1, 20000, 'radius', 'fp16')
    assert a.streams == 3 and a.concurrent == 1
    assert bench.conv_waves_of(a) == pipeline.CONCURRENT_CONV_WAVES == 1536
    assert pipeline.CONCURRENT_CONV_WAVES % 64 == 0   # rg_conv_layer_fused_waves' unit


@pytest.mark.parametrize('cfg', ['c2', 'c3', 'c5b'])
def test_batched_16bit_presets_keep_build_overlap(monkeypatch, cfg):
    a = _parse(monkeypatch, '--config', cfg)
    assert a.streams == 2 and not a.concurrent
    from graph_neural_network_for_radar_perception_amd import engine
    assert bench.conv_waves_of(a) == engine.DeviceGraph.CONV_WAVES
