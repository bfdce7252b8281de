#!/usr/bin/env python
"""Decode value-transform A/B on one box: fp32 LDS table (mode 0) vs the
verified arithmetic form with a lane-private u8 gamma table (16 or 32
copies).  Variant from the environment (BLENDTORCH_DECODE_XFORM=0/1,
BLENDTORCH_GAMMA_COPIES=16/32).  Two inputs: uniform random bytes (worst
case for table lookups) and a smooth synthetic scene (neighbouring pixels
alike, like rendered frames).  Prints one JSON line per (input, config).

    python scripts/decode_ab.py [--iters 200] [--pmc]   (--pmc: few launches, for rocprofv3 --pmc)
"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / 'pytorch-blender_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from blendtorch import ops  # noqa: E402


def scene(B, H, W, seed=0):
    """Smooth frames: gradients, a few flat boxes, mild noise."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W].astype(np.float32)
    out = np.empty((B, H, W, 4), np.uint8)
    for b in range(B):
        img = np.stack([x / W * 200 + 20, y / H * 180 + 30, (x + y) / (W + H) * 150 + 60, np.full_like(x, 255)], -1)
        for _ in range(6):
            x0, y0 = rng.integers(0, W - 80), rng.integers(0, H - 80)
            img[y0:y0 + 80, x0:x0 + 80, :3] = rng.integers(0, 256, 3)
        img[..., :3] += rng.normal(0, 2, (H, W, 3))
        out[b] = np.clip(img, 0, 255).astype(np.uint8)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--pmc', action='store_true')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    B, H, W = 8, 480, 640
    inputs = {'random': torch.randint(0, 256, (B, H, W, 4), dtype=torch.uint8, device=dev),
              'scene': torch.from_numpy(scene(B, H, W)).to(dev)}
    cfgs = {'unit_gamma_bf16_nhwc_rgba': ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16',
                                                               layout='nhwc'),
            'unit_gamma_f32_rgb': ops.DecodeConfig.unit(channels='rgb', gamma=2.2),
            'densityopt_gamma_f32_rgb': ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
            'unit_f32_rgb': ops.DecodeConfig.unit(channels='rgb')}
    variant = {'xform': os.environ.get('BLENDTORCH_DECODE_XFORM', '1'),
               'copies': os.environ.get('BLENDTORCH_GAMMA_COPIES', '32')}
    iters = 3 if a.pmc else a.iters
    for iname, x in inputs.items():
        for cname, cfg in cfgs.items():
            out = ops.decode(x, cfg)
            ref = ops.reference_decode(x.cpu(), cfg)
            exact = bool(torch.equal(out.cpu(), ref))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ops.decode(x, cfg, out=out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            print(json.dumps(dict(variant, input=iname, config=cname, us=round(us, 2), exact=exact)), flush=True)


if __name__ == '__main__':
    main()
