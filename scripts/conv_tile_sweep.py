"""Per-layer tile / staging sweep of the tap-gather GEMM (forward with the BN
accumulator epilogue, and the data gradient) on the bench discriminator's
layers (batch 8, 640x480 input): every (BM, BN, staging) the kernel builds,
device time per call from graph replays (scripts/conv_bench.py's timer).
Prints one JSON row per (layer, op, variant) and the best per (layer, op).

    python scripts/conv_tile_sweep.py [--iters 200]
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

LAYERS = [(64, 120, 160, 128), (128, 60, 80, 256), (32, 240, 320, 64)]   # Cin, H, W, Cout (input side)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--batch', type=int, default=8)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    ext = ops.hip_ext()
    best = {}
    for cin, h, w, cout in LAYERS:
        x = torch.randn(a.batch, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(a.batch, cout, h // 2, w // 2, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        w16 = (torch.randn(cout, cin, 4, 4, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        acc = ops.BnAccumulator(cout, dev)
        wt = torch.empty(cin * 16 * cout, dtype=torch.bfloat16, device=dev)   # the transposed weight, once
        ext.conv_weight_t(w16.data_ptr(), wt.data_ptr(), cout, cin, torch.cuda.current_stream().cuda_stream)
        yref = ops.conv_fwd(x, w16)
        dref = ops.conv_dgrad(dy, w16, tuple(x.shape), wt=wt)
        layer = f'{cin}->{cout} @ {h}x{w}'
        for staging in (0, 2, 3, 4):
            for bm in (64, 128):
                for bn in (64, 128):
                    if cout % bn:
                        continue
                    ext.conv_set_tiles(bm, bn, staging, 0)
                    for op in ('fwd', 'dgrad'):
                        if op == 'fwd':
                            fn = lambda: ops.conv_fwd(x, w16, acc.fwd, acc_r=acc.R)
                            ok = torch.equal(ops.conv_fwd(x, w16), yref)
                        else:
                            fn = lambda: ops.conv_dgrad(dy, w16, tuple(x.shape), wt=wt)
                            ok = torch.equal(ops.conv_dgrad(dy, w16, tuple(x.shape), wt=wt), dref)
                        try:
                            us = timed(fn, a.iters)
                        except RuntimeError as e:
                            print(json.dumps({'layer': layer, 'op': op, 'staging': staging, 'bm': bm, 'bn': bn,
                                              'error': str(e)[:200]}), flush=True)
                            continue
                        row = {'layer': layer, 'op': op, 'staging': staging, 'bm': bm, 'bn': bn,
                               'us': round(us, 2), 'bit_exact_vs_default': ok}
                        print(json.dumps(row), flush=True)
                        k = (layer, op)
                        if k not in best or us < best[k]['us']:
                            best[k] = row
        ext.conv_set_tiles(0, 0, -1, 0)
    for k, v in best.items():
        print('BEST', json.dumps(v), flush=True)


if __name__ == '__main__':
    main()
