"""Split-K forward (tap_gemm_body SPLIT = 2, BT_CONV_FWD_SPLIT) against the
default tap-GEMM forward on the bench discriminator's 128- and 256-channel
layers, with and without the BN statistics, and the max relative error of each
against fp32 conv2d.  Device time per call from graph replays.

    python scripts/fwd_split_bench.py [--iters 200]
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

LAYERS = [(64, 120, 160, 128), (128, 60, 80, 256)]   # Cin, H, W, Cout (input side), batch 8


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
        w = (0.05 * torch.randn(cout, cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(
            memory_format=cl)
        ref = torch.nn.functional.conv2d(x.float(), w.float(), stride=2, padding=1)
        acc = ops.BnAccumulator(cout, dev)
        for split in (0, 1, 0, 1):
            ext.conv_set_fwd_split(split)
            n0 = ext.conv_fwd_split_launches()
            y = ops.conv_fwd(x, w)
            took = ext.conv_fwd_split_launches() > n0
            err = float((y.float() - ref).abs().max() / ref.abs().max())
            plain = timed(lambda: ops.conv_fwd(x, w), a.iters)
            stats = timed(lambda: ops.conv_fwd(x, w, acc.fwd, acc.R), a.iters)
            print(json.dumps({'layer': f'{cin}->{cout} @{H}x{W}', 'split': split, 'split_ran': took,
                              'fwd_us': round(plain, 2), 'fwd_stats_us': round(stats, 2),
                              'rel_err': float(f'{err:.2e}')}), flush=True)
    ext.conv_set_fwd_split(-1)


if __name__ == '__main__':
    main()
