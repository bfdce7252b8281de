"""Where a BatchNorm+LeakyReLU apply launch of the disc step spends its time:
for each of the step's six applies (forward BN1-3, backward BN4-2 at batch 8,
640x480), device time per call (graph replays, scripts/conv_bench.py's timer)
of
  fold     the accumulator form the step runs (every block folds the fp64
           replicas, takes a release ticket, the last block clears);
  norel    the same without the release (BT_BN_RELEASE=0 -- run this script
           once with it set; the accumulator is then never cleared, so only
           the timing is meaningful);
  plain    the apply pass alone with the coefficients given (no fold);
and the bytes each moves, as TB/s.

    python scripts/bn_apply_bench.py [--iters 200]
"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402
from conv_bench import timed  # noqa: E402

# (name, backward?, pixels M, channels C)
APPLIES = [('bn1_fwd', False, 8 * 240 * 320, 32), ('bn2_fwd', False, 8 * 120 * 160, 64),
           ('bn3_fwd', False, 8 * 60 * 80, 128), ('bn4_bwd', True, 8 * 30 * 40, 256),
           ('bn3_bwd', True, 8 * 60 * 80, 128), ('bn2_bwd', True, 8 * 120 * 160, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    ext = ops.hip_ext()
    bf = ops.OUT_DTYPES['bfloat16']
    mode = 'norel' if os.environ.get('BT_BN_RELEASE', '1') == '0' else 'fold'
    g = torch.Generator(device=dev).manual_seed(0)
    for name, bwd, M, C in APPLIES:
        x = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
        gy = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
        out = torch.empty_like(x)
        w = torch.rand(C, device=dev, generator=g) + 0.5
        b = torch.randn(C, device=dev, generator=g) * 0.1
        mean = torch.zeros(C, device=dev)
        invstd = torch.ones(C, device=dev)
        dw = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        acc = ops.BnAccumulator(C, dev)
        s = ops._stream(dev)
        a_ = acc.fwd if not bwd else acc.bwd
        if bwd:
            fold = lambda: ext.bn_backward_acc(x.data_ptr(), gy.data_ptr(), out.data_ptr(), M, C, bf, a_.data_ptr(),
                                               acc.R, mean.data_ptr(), invstd.data_ptr(), w.data_ptr(), b.data_ptr(),
                                               dw.data_ptr(), db.data_ptr(), 0.2, ops._stream(dev), False)
            plain = lambda: ext.bn_bwd_apply(x.data_ptr(), gy.data_ptr(), out.data_ptr(), M, C, bf, mean.data_ptr(),
                                             invstd.data_ptr(), w.data_ptr(), b.data_ptr(), dw.data_ptr(),
                                             db.data_ptr(), 0.2, ops._stream(dev))
            nbytes = 3 * M * C * 2
        else:
            fold = lambda: ext.bn_forward_acc(x.data_ptr(), out.data_ptr(), M, C, bf, a_.data_ptr(), acc.R, 1e-5, 0.1,
                                              mean.data_ptr(), invstd.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                                              w.data_ptr(), b.data_ptr(), 0.2, ops._stream(dev), 0)
            plain = lambda: ext.bn_fwd_apply(x.data_ptr(), out.data_ptr(), M, C, bf, mean.data_ptr(),
                                             invstd.data_ptr(), w.data_ptr(), b.data_ptr(), 0.2, ops._stream(dev))
            nbytes = 2 * M * C * 2
        del s
        for v, fn in ((mode, fold), ('plain', plain)):
            us = timed(fn, a.iters)
            print(json.dumps({'apply': name, 'variant': v, 'M': M, 'C': C, 'us': round(us, 2),
                              'tbps': round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == '__main__':
    main()
