"""conv2's forward (8 x 32 x 240 x 320 -> 64 channels, BN sums into an
accumulator) on the persistent patch GEMM against the tap GEMM, and the patch
kernel with parts switched off (dbg bits: 1 no patch fills, 2 no MFMAs, 4 no
stores) or a different grid -- which part sets its time.

    python scripts/fwd_patch_bench.py [--iters 400]
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
    ap.add_argument('--iters', type=int, default=400)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    ext = ops.hip_ext()
    x = torch.randn(8, 32, 240, 320, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.05 * torch.randn(64, 32, 4, 4, device=dev)).to(torch.bfloat16).contiguous(memory_format=cl)
    acc = ops.BnAccumulator(64, dev)
    variants = [('tap', 0, 0, 0), ('patch', 1, 0, 0), ('patch_nofill', 1, 1, 0), ('patch_nomfma', 1, 2, 0),
                ('patch_nostore', 1, 4, 0), ('patch_only_mfma', 1, 5, 0), ('patch_only_fill', 1, 6, 0),
                ('patch_none', 1, 7, 0), ('patch_g240', 1, 0, 240), ('patch_g128', 1, 0, 128),
                ('patch_g200', 1, 0, 200), ('tap2', 0, 0, 0), ('patch2', 1, 0, 0)]
    for name, on, dbg, blocks in variants:
        ext.conv_set_fwd_patch(on, dbg, blocks)
        try:
            us = timed(lambda: ops.conv_fwd(x, w, acc.fwd, acc.R), a.iters)
        finally:
            ext.conv_set_fwd_patch(-1, 0, 0)
        acc.fwd.zero_()
        print(json.dumps({'variant': name, 'us': round(us, 2)}), flush=True)


if __name__ == '__main__':
    main()
