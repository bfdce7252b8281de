"""The first layer's weight gradient (conv_wgrad_c4w_kernel + its slice
reduce) alone, on the bench discriminator's shape: 8 x 480 x 640 RGBA input,
32 output channels.  Variants: raw u8 frames through the decode table or
decoded bf16 frames; with / without the BN1 backward applied to dY while it
is staged (sums given); waves per block; slice (block) targets.  Device time
per call (kernel + reduce) from graph replays (scripts/conv_bench.py's
timer), and the max relative error against fp32 PyTorch.

    python scripts/c4w_bench.py [--iters 200]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--patch-only', action='store_true', help='the c4p kernel against the default c4w only')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    ext = ops.hip_ext()
    g = torch.Generator(device=dev).manual_seed(0)
    N, H, W, C = 8, 480, 640, 32
    raw = torch.randint(0, 256, (N, H, W, 4), dtype=torch.uint8, device=dev, generator=g)
    x_u8 = raw.permute(0, 3, 1, 2)                                  # [N, 4, H, W] channels-last bytes
    dcfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    lut = ops.decode_lut_bf16(dcfg, dev)
    x_bf = ops.decode(raw, dcfg).permute(0, 3, 1, 2)                # decoded bf16, channels-last
    dy = (torch.randn(N, C, H // 2, W // 2, device=dev, generator=g) * 0.1).to(torch.bfloat16).contiguous(memory_format=cl)
    y = torch.randn(N, H // 2, W // 2, C, device=dev, generator=g).to(torch.bfloat16)   # BN input, NHWC
    mean = torch.randn(C, device=dev, generator=g) * 0.1
    invstd = torch.rand(C, device=dev, generator=g) + 0.5
    bw = torch.rand(C, device=dev, generator=g) + 0.5
    bb = torch.randn(C, device=dev, generator=g) * 0.1
    dw = torch.randn(C, device=dev, generator=g) * 1e3
    db = torch.randn(C, device=dev, generator=g) * 1e3
    out = torch.empty(C, 3, 4, 4, device=dev)
    ref = torch.nn.grad.conv2d_weight(x_bf.float()[:, :3], (C, 3, 4, 4), dy.float(), stride=2, padding=1)
    rows = []
    ap_only = a.patch_only
    for bn in (False, True):
        # the decoded-patch kernel (conv_wgrad_c4p_kernel, u8 only): bands of 1, 2, 4 output rows
        for r in (1, 2, 4):
            ext.conv_set_c4p_rows(r)
            x = x_u8
            bnd = (y, mean, invstd, bw, bb, dw, db, 0.2) if bn else None
            fn = lambda: ops.conv_wgrad(x, dy, out, lut=lut, bn_dy=bnd)
            us = timed(fn, a.iters)
            row = {'kernel': 'c4p', 'bn_dy': bn, 'u8': True, 'rows': r, 'us': round(us, 2)}
            if not bn:
                fn()
                row['rel_err'] = float(f'{float((out - ref).abs().max() / ref.abs().max()):.2e}')
            print(json.dumps(row), flush=True)
            rows.append(row)
        ext.conv_set_c4p_rows(0)
        if ap_only:
            for tb in (512,):
                x = x_u8
                bnd = (y, mean, invstd, bw, bb, dw, db, 0.2) if bn else None
                fn = lambda: ops.conv_wgrad(x, dy, out, target_blocks=tb, lut=lut, bn_dy=bnd)
                row = {'kernel': 'c4w', 'bn_dy': bn, 'u8': True, 'waves': 4, 'target_blocks': tb,
                       'us': round(timed(fn, a.iters), 2)}
                print(json.dumps(row), flush=True)
            ext.conv_set_c4p_rows(-1)
            continue
        for u8 in (True, False):
            for nw in (4, 8):
                for tb in (256, 512, 768, 1024):
                    ext.conv_set_c4w_waves(nw)
                    x = x_u8 if u8 else x_bf
                    bnd = (y, mean, invstd, bw, bb, dw, db, 0.2) if bn else None
                    fn = lambda: ops.conv_wgrad(x, dy, out, target_blocks=tb, lut=lut if u8 else None, bn_dy=bnd)
                    us = timed(fn, a.iters)
                    row = {'bn_dy': bn, 'u8': u8, 'waves': nw, 'target_blocks': tb, 'us': round(us, 2)}
                    if not bn:
                        fn()
                        row['rel_err'] = float(f'{float((out - ref).abs().max() / ref.abs().max()):.2e}')
                    print(json.dumps(row), flush=True)
                    rows.append(row)
    ext.conv_set_c4w_waves(-1)
    ext.conv_set_c4p_rows(-1)


if __name__ == '__main__':
    main()
