"""Consumer models and their fused-op modules on the CPU path (the gfx950
kernels themselves are covered by tests/test_gpu_kernels.py)."""
import sys
from pathlib import Path

import torch
import torch.nn as nn

from blendtorch import ops
from blendtorch.models import Discriminator


def test_ops_import_does_not_need_torch_modules():
    # the fused modules are built lazily and are real nn.Module subclasses
    assert issubclass(ops.BatchNormLeakyReLU2d, nn.BatchNorm2d)
    assert issubclass(ops.AdaptiveAvgPool2d, nn.Module)


def test_bn_leaky_cpu_fallback_matches_unfused():
    torch.manual_seed(0)
    a = ops.BatchNormLeakyReLU2d(16, slope=0.2)
    b = nn.Sequential(nn.BatchNorm2d(16), nn.LeakyReLU(0.2))
    b[0].load_state_dict(a.state_dict())
    x = torch.randn(4, 16, 9, 7)
    for mode in ('train', 'eval'):
        getattr(a, mode)()
        getattr(b, mode)()
        assert torch.allclose(a(x), b(x), atol=1e-6)
    assert torch.allclose(a.running_mean, b[0].running_mean)
    assert int(a.num_batches_tracked) == int(b[0].num_batches_tracked) == 1


def test_adaptive_pool_cpu_fallback():
    x = torch.randn(2, 8, 15, 20)
    assert torch.equal(ops.AdaptiveAvgPool2d((3, 4))(x), nn.functional.adaptive_avg_pool2d(x, (3, 4)))


def test_discriminator_fused_state_dict_interchange():
    torch.manual_seed(1)
    a = Discriminator(adaptive=True)
    b = Discriminator(adaptive=True, fused=False)
    assert a.state_dict().keys() == b.state_dict().keys()
    b.load_state_dict(a.state_dict())
    x = torch.randn(2, 3, 64, 80)
    assert torch.allclose(a(x), b(x), atol=1e-6)


def test_keypoint_net_fused_matches_unfused():
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'examples' / 'datagen'))
    import train_keypoints as tk
    torch.manual_seed(2)
    a, b = tk.KeypointNet(), tk.KeypointNet(fused=False)
    b.load_state_dict(a.state_dict())
    x = torch.randn(2, 3, 96, 128)
    assert torch.allclose(a(x), b(x), atol=1e-5)
