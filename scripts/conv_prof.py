"""Runs the MFMA conv kernels on the bench discriminator's layer shapes (for
rocprofv3 --kernel-trace --stats: per-kernel times of conv_fwd,
conv_wgrad and its slice reduce).  python scripts/conv_prof.py [--blocks 512]"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))
import torch  # noqa: E402

from blendtorch import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--blocks', type=int, default=512)
ap.add_argument('--iters', type=int, default=50)
a = ap.parse_args()
dev = torch.device('cuda', 0)
cl = torch.channels_last
for cin, h, w, cout in [(32, 240, 320, 64), (64, 120, 160, 128), (128, 60, 80, 256)]:
    x = torch.randn(8, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(8, cout, h // 2, w // 2, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w16 = torch.randn(cout, cin, 4, 4, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    out = torch.empty(cout, cin, 4, 4, device=dev).contiguous(memory_format=cl)
    for _ in range(a.iters):
        ops.conv_wgrad(x, dy, out, target_blocks=a.blocks)
        ops.conv_fwd(x, w16)
        ops.conv_dgrad(dy, w16, tuple(x.shape))
torch.cuda.synchronize()
print('done')
