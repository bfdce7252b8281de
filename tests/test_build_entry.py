"""The built extensions load in this (GPU-less) process: an unresolved symbol
in the gfx950 extension shows up here, not first on the GPU box."""
import importlib
from pathlib import Path

import pytest

PKG = Path(__file__).resolve().parents[1] / 'pytorch-blender_amd' / 'blendtorch'


def test_hip_extension_loads_without_a_gpu():
    if not list(PKG.glob('_hip*.so')):
        pytest.skip('HIP extension not built here')
    import torch  # noqa: F401  (its HIP runtime first, as ops.hip_ext does)
    ext = importlib.import_module('blendtorch._hip')
    for name in ('conv_wgrad', 'conv_dgrad_hold', 'conv_dgrad_flush', 'adam_attach_schedule', 'adam_update',
                 'replay_sample'):
        assert hasattr(ext, name), name


def test_native_extension_loads():
    if not list(PKG.glob('_native*.so')):
        pytest.skip('native extension not built here')
    ext = importlib.import_module('blendtorch._native')
    assert hasattr(ext, 'recv_round')
