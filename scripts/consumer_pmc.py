"""Short driver for PMC passes over the consumer-model kernels: fused
BatchNorm+LeakyReLU forward/backward and NHWC adaptive pooling on the
discriminator's first-layer activation (8 x 32 x 240 x 320 bf16, 39.3 MB)
and its pooled head input (8 x 256 x 30 x 40).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python scripts/consumer_pmc.py
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402


def main(iters=5):
    dev = torch.device('cuda', 0)
    ops.hip_ext()
    x = torch.randn(8, 32, 240, 320, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    w = torch.ones(32, device=dev, requires_grad=True)
    b = torch.zeros(32, device=dev, requires_grad=True)
    rm, rv = torch.zeros(32, device=dev), torch.ones(32, device=dev)
    gy = torch.randn(8, 240, 320, 32, device=dev, dtype=torch.bfloat16).permute(0, 3, 1, 2)
    p = torch.randn(8, 256, 30, 40, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    p.requires_grad_(True)
    gp = torch.randn(8, 4, 4, 256, device=dev, dtype=torch.bfloat16).permute(0, 3, 1, 2)
    for _ in range(iters):
        y = ops.batch_norm_leaky_relu(x, w, b, rm, rv)
        y.backward(gy)
        q = ops.adaptive_avg_pool_nhwc(p, 4)
        q.backward(gp)
    torch.cuda.synchronize()
    print('ok', float(x.grad.float().abs().sum()), float(p.grad.float().abs().sum()))


if __name__ == '__main__':
    main()
