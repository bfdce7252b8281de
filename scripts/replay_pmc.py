"""Short replay-sampler run for rocprofv3 --pmc passes (fused kernel at
batch 8 and 64, 640x480 RGBA store -> fp32 RGB CHW with gamma)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402
from blendtorch.btt.replay import DeviceReplayBuffer  # noqa: E402

dev = torch.device('cuda', 0)
rb = DeviceReplayBuffer(1024, device=dev, seed=1)
g = torch.Generator(device=dev).manual_seed(0)
for s in range(0, 1024, 256):
    rb.extend(torch.randint(0, 256, (256, 480, 640, 4), dtype=torch.uint8, device=dev, generator=g),
              frameid=torch.arange(s, s + 256, device=dev))
cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
for B in (8, 64):
    for _ in range(10):
        rb.sample(B, cfg)
torch.cuda.synchronize()
print('ok')
