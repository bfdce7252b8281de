#!/usr/bin/env python
"""Micro-benchmark of the gfx950 image kernels vs eager PyTorch.

Times each kernel with HIP events over many iterations on a batch of
8 x 480 x 640 RGBA frames (the headline config) and reports achieved HBM
bandwidth (bytes read + written / time).  `--json` writes results to a file.
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / 'pytorch-blender_amd'))

import numpy as np
import torch

from blendtorch import ops


def timeit(fn, iters=200, warmup=20):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--tag', default='')
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--json', default=None)
    ap.add_argument('--only', default=None)
    ap.add_argument('--no-ref', action='store_true', help='skip the eager-PyTorch reference timings')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    B, H, W = a.batch, 480, 640
    x4 = torch.randint(0, 256, (B, H, W, 4), dtype=torch.uint8, device=dev)
    x3 = x4[..., :3].contiguous()
    res = {}
    cases = {
        'decode_rgba_rgb_f32_gamma_norm': (x4, ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2), 4, 12),
        'decode_rgba_rgb_bf16_gamma_norm': (x4, ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2, dtype='bfloat16'), 4, 6),
        'decode_rgb_rgb_f32_unit': (x3, ops.DecodeConfig.unit(channels='rgb'), 3, 12),
        'decode_rgba_u8_gamma': (x4, ops.DecodeConfig(channels='rgba', gamma=2.2, dtype='uint8'), 4, 4),
        'decode_rgba_rgb_f32_nhwc': (x4, ops.DecodeConfig.unit(channels='rgb', layout='nhwc'), 4, 12),
    }
    ext = ops.hip_ext()
    for name, (x, cfg, inb, outb) in cases.items():
        if a.only and a.only not in name:
            continue
        out = ops.decode(x, cfg)
        lut = ops.device_lut(cfg, dev)
        # kernel-only time (C++ launch loop between HIP events)
        us = ext.bench_decode(x.data_ptr(), out.data_ptr(), lut.data_ptr(), B, H, W, x.shape[-1], cfg.cout,
                              list(cfg.cmap), ops.OUT_DTYPES[cfg.dtype], ops.LAYOUTS[cfg.layout], a.iters)
        ref_us = float('nan') if a.no_ref else timeit(lambda: ops.reference_decode(x, cfg), max(10, a.iters // 10), 3)
        nbytes = B * H * W * (inb + outb)
        res[name] = {'us': round(us, 2), 'GBps': round(nbytes / us / 1e3, 1), 'torch_eager_us': round(ref_us, 1),
                     'speedup_vs_eager': round(ref_us / us, 1)}
        print(a.tag, name, res[name], flush=True)
    if not a.only or 'color' in a.only:
        M = np.random.default_rng(0).normal(size=(4, 4)).astype(np.float32)
        cfg = ops.DecodeConfig(channels='rgba', gamma=2.2, color_matrix=M)
        out = ops.color4x4(x4, M, [0, 0, 0, 0], gamma=2.2)
        lut = ops.device_lut(cfg, dev)
        Mt = torch.as_tensor(M, device=dev).contiguous()
        bt = torch.zeros(4, dtype=torch.float32, device=dev)
        us = ext.bench_color4x4(x4.data_ptr(), out.data_ptr(), lut.data_ptr(), Mt.data_ptr(), bt.data_ptr(),
                                B, H, W, 4, a.iters)   # kernel-only (C++ launch loop between HIP events)
        py_us = timeit(lambda: ops.color4x4(x4, M, [0, 0, 0, 0], gamma=2.2), a.iters)   # incl. Python op overhead
        ref_us = timeit(lambda: ops.reference_color4x4(x4, M, [0, 0, 0, 0], gamma=2.2), 20, 3)
        nbytes = B * H * W * (4 + 16)
        res['color4x4_mfma_rgba_f32'] = {'us': round(us, 2), 'GBps': round(nbytes / us / 1e3, 1),
                                         'python_op_us': round(py_us, 1),
                                         'torch_eager_us': round(ref_us, 1), 'speedup_vs_eager': round(ref_us / us, 1)}
        print('color4x4_mfma_rgba_f32', res['color4x4_mfma_rgba_f32'], flush=True)
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=2))


if __name__ == '__main__':
    main()
