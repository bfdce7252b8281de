#!/usr/bin/env python
"""Launch each gfx950 kernel a few times (no eager-torch baselines) so a
rocprofv3 --pmc pass stays short."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / 'pytorch-blender_amd'))
import numpy as np
import torch

from blendtorch import ops

dev = torch.device('cuda', 0)
x4 = torch.randint(0, 256, (8, 480, 640, 4), dtype=torch.uint8, device=dev)
x3 = x4[..., :3].contiguous()
M = np.random.default_rng(0).normal(size=(4, 4)).astype(np.float32)
for _ in range(3):
    ops.decode(x4, ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2))
    ops.decode(x4, ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2, dtype='bfloat16'))
    ops.decode(x3, ops.DecodeConfig.unit(channels='rgb'))
    ops.decode(x4, ops.DecodeConfig.unit(channels='rgb', layout='nhwc'))
    ops.color4x4(x4, M, [0, 0, 0, 0], gamma=2.2)
torch.cuda.synchronize()
print('ok')
