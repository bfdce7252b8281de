"""Weight-gradient tile shapes on the bench discriminator's 128- and 256-channel
layers: 64-channel tiles (conv_wgrad_body, the default) against 128-channel
tiles (conv_wgrad_co128_body, BT_WGRAD_CO128), alone (kernel + slice reduce)
and as the fused data + weight gradient launch of the training step
(conv_dgrad_hold + conv_wgrad: dgrad_wgrad_kernel), with the max relative
error of each against fp32 PyTorch.  Device time per call from graph replays.

    python scripts/wgrad_tiles_bench.py [--iters 200]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402
from conv_bench import timed  # noqa: E402

LAYERS = [(32, 240, 320, 64), (64, 120, 160, 128), (128, 60, 80, 256)]   # Cin, H, W, Cout (input side), batch 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    ext = ops.hip_ext()
    g = torch.Generator(device=dev).manual_seed(0)
    for cin, H, W, cout in LAYERS:
        x = torch.randn(8, cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
        dy = (torch.randn(8, cout, H // 2, W // 2, device=dev, generator=g) * 0.1).to(torch.bfloat16).contiguous(
            memory_format=cl)
        w = (0.05 * torch.randn(cout, cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(
            memory_format=cl)
        out = torch.empty(cout, cin, 4, 4, device=dev)
        ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 4, 4), dy.float(), stride=2, padding=1)
        # 32 -> 64 (Cout 64): 128-column tiles against 256-column ones (conv_wgrad_wide_body, fused
        # with the patch data gradient); the deeper layers: 64- against 128-channel tiles
        for co128 in ((0, 1) if cout % 128 else (0, 1, 2)):
            if cout % 128:
                ext.conv_set_wgrad_co128(0)
                ext.conv_set_wgrad_wide(co128)
            else:
                ext.conv_set_wgrad_co128(1 if co128 else 0)
                ext.conv_set_wgrad_wide(0)
            # 2: the fused launch's data gradient in 128-channel tiles too (Cin % 128 == 0)
            ext.conv_set_dgrad_bn128(1 if co128 == 2 else 0)
            alone = timed(lambda: ops.conv_wgrad(x, dy, out), a.iters)
            ops.conv_wgrad(x, dy, out)
            err = float((out - ref).abs().max() / ref.abs().max())

            def pair():
                ext.conv_dgrad_hold(1)
                try:
                    ops.conv_dgrad(dy, w, tuple(x.shape))
                finally:
                    ext.conv_dgrad_hold(0)
                ops.conv_wgrad(x, dy, out)
            fused = timed(pair, a.iters)
            dgrad = timed(lambda: ops.conv_dgrad(dy, w, tuple(x.shape)), a.iters)
            print(json.dumps({'layer': f'{cin}->{cout} @{H}x{W}', ('wide' if cout % 128 else 'co128'): co128, 'wgrad_us': round(alone, 2),
                              'fused_pair_us': round(fused, 2), 'dgrad_alone_us': round(dgrad, 2),
                              'rel_err': float(f'{err:.2e}')}), flush=True)
    ext.conv_set_wgrad_co128(-1)
    ext.conv_set_wgrad_wide(-1)
    ext.conv_set_dgrad_bn128(-1)


if __name__ == '__main__':
    main()
