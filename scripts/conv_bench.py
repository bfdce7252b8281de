"""Tap-GEMM forward / data-gradient and weight-gradient kernel timing on the bench discriminator's layers (batch 8,
640x480 input): gfx950 MFMA ``ops.conv_wgrad`` (over several grid sizes) vs
MIOpen's bf16 weight gradient (``aten.convolution_backward``, weight only).

    python scripts/conv_bench.py [--iters 200]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402

LAYERS = [(32, 240, 320, 64), (64, 120, 160, 128), (128, 60, 80, 256)]
   # Cin, H, W, Cout (input side)


GRAPH = True


def timed(fn, iters):
    """Device time per call: ``fn`` captured 20 times in a HIP graph and the
    graph replayed (eager calls measure the host's launch path instead --
    ~20 us per call, more than most of these kernels take)."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    reps = 20
    g = None
    if GRAPH:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(1, iters // reps)
    e0.record()
    if g is not None:
        for _ in range(n):
            g.replay()
    else:
        for _ in range(n * reps):
            fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (n * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--eager', action='store_true', help='time eager calls (host launch path included)')
    a = ap.parse_args()
    global GRAPH
    GRAPH = not a.eager
    torch.backends.cudnn.benchmark = True
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    for cin, h, w, cout in LAYERS:
        x = torch.randn(a.batch, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(a.batch, cout, h // 2, w // 2, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        w16 = torch.randn(cout, cin, 4, 4, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        out = torch.empty(cout, cin, 4, 4, device=dev).contiguous(memory_format=cl)
        row = {'layer': f'{cin}->{cout} @ {h}x{w}', 'gflop': round(2 * a.batch * (h // 2) * (w // 2) * cout * cin * 16 / 1e9, 2)}
        row['miopen_us'] = round(timed(lambda: torch.ops.aten.convolution_backward(
            dy, x, w16, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]), a.iters), 2)
        import torch.nn.functional as F
        row['miopen_fwd_us'] = round(timed(lambda: F.conv2d(x, w16, None, 2, 1), a.iters), 2)
        rows = ops.conv_fwd_stats_rows(a.batch * (h // 2) * (w // 2), cout)
        stats = torch.empty(rows * 2 * cout, device=dev)
        row['mfma_fwd_us'] = round(timed(lambda: ops.conv_fwd(x, w16), a.iters), 2)
        row['mfma_fwd_stats_us'] = round(timed(lambda: ops.conv_fwd(x, w16, stats), a.iters), 2)
        yref = F.conv2d(x.float(), w16.float(), None, 2, 1)
        row['fwd_rel_err'] = float(f'{float((ops.conv_fwd(x, w16).float() - yref).abs().max() / yref.abs().max()):.2e}')
        row['miopen_dgrad_us'] = round(timed(lambda: torch.ops.aten.convolution_backward(
            dy, x, w16, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]), a.iters), 2)
        row['mfma_dgrad_us'] = round(timed(lambda: ops.conv_dgrad(dy, w16, tuple(x.shape)), a.iters), 2)
        dref = torch.nn.grad.conv2d_input(tuple(x.shape), w16.float(), dy.float(), stride=2, padding=1)
        row['dgrad_rel_err'] = float(f'{float((ops.conv_dgrad(dy, w16, tuple(x.shape)).float() - dref).abs().max() / dref.abs().max()):.2e}')
        ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 4, 4), dy.float(), stride=2, padding=1)
        for tb in (256, 512, 1024, 2048):
            us = timed(lambda: ops.conv_wgrad(x, dy, out, target_blocks=tb), a.iters)
            err = float((out - ref).abs().max() / ref.abs().max())
            row[f'mfma_us_b{tb}'] = round(us, 2)
            row[f'rel_err_b{tb}'] = float(f'{err:.2e}')
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
