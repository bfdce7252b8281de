"""Consumer-step microbenchmark: DCGAN discriminator training step (forward,
backward, Adam) on a batch of 8 x 3 x 480 x 640 frames, in the layouts and
dtypes the bench consumer can use.  Input is a random HBM tensor, so the
number is the model step alone (no streaming).

    python scripts/disc_step_bench.py [--iters 200] [--only bf16-nhwc]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402

from blendtorch.models import Discriminator  # noqa: E402

VARIANTS = {
    'bf16-nhwc': (torch.bfloat16, torch.channels_last),
    'bf16-nchw': (torch.bfloat16, torch.contiguous_format),
    'fp32-nhwc': (torch.float32, torch.channels_last),
    'fp32-nchw': (torch.float32, torch.contiguous_format),
}


def run(name, iters, batch, graph, fused_adam=False, fused_bn=True, dma=0, cast='autocast', u8=False, optim='torch',
        dma_phase='none', split=False, head='torch'):
    dt, fmt = VARIANTS[name]
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = Discriminator(nc=3, ndf=32, adaptive=True, fused=fused_bn).to(dev).to(memory_format=fmt)
    if optim == 'gfx950':
        from blendtorch import ops
        opt = ops.FusedAdam(model.parameters(), lr=2e-4)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=2e-4, capturable=graph, fused=fused_adam or None)
    crit = torch.nn.BCELoss()
    x = torch.rand(batch, 3, 480, 640, device=dev).to(memory_format=fmt)
    amp = dt == torch.bfloat16
    if amp:
        x = x.to(torch.bfloat16)
    if u8:
        # what bench.py --consumer disc trains on: raw RGBA u8 NHWC frames,
        # decoded (gamma, /255, bf16 NHWC) inside the step
        from blendtorch import ops
        raw = torch.randint(0, 256, (batch, 480, 640, 4), dtype=torch.uint8, device=dev)
        dcfg = ops.DecodeConfig.unit(channels='rgba' if (amp and cast == 'fused') else 'rgb', gamma=2.2,
                                     dtype='bfloat16' if amp else 'float32', layout='nhwc')

    def inputs():
        if not u8:
            return x
        y = ops.decode(raw, dcfg).permute(0, 3, 1, 2)
        return y if amp else y.contiguous(memory_format=torch.channels_last)

    def step():
        opt.zero_grad(set_to_none=True)
        xi = inputs()
        if amp and cast == 'fused' and head == 'fused':
            model.bce_loss_bf16(xi, 1.0).backward()
            opt.step()
            return
        if amp and cast == 'fused':
            out = model.forward_bf16(xi)
        else:
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp, cache_enabled=not graph):
                out = model(xi)
        loss = crit(out.float(), torch.ones(batch, device=dev))
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    # optional background H2D traffic shaped like the stream loader's copy path:
    # 8 frames of 640x480 RGBA (9.8 MB) per step from pinned host memory, spread
    # over `dma` side streams -- isolates what DMA alone does to the step
    side = [torch.cuda.Stream() for _ in range(dma)]
    hsrc = [torch.empty(1228800, dtype=torch.uint8).pin_memory() for _ in range(8)] if dma else []
    ddst = [torch.empty(1228800, dtype=torch.uint8, device=dev) for _ in range(8)] if dma else []

    def copies():
        # dma_phase: none = issued unordered (they run whenever the DMA engines
        # are free); start = gated on the step's start, so they overlap the
        # forward (what the stream loader's post events do); mid = gated
        # between the forward and the backward graph
        t0 = time.perf_counter()
        ev = None
        if dma_phase != 'none':
            ev = torch.cuda.Event()
            ev.record()
            evs.append(ev)
        if dma_phase == 'start_prev':   # gate on the event of two steps ago (already passed, usually)
            ev = evs[-3] if len(evs) >= 3 else None
        if dma_phase == 'record':       # record only: no cross-stream wait
            ev = None
        for i in range(8 if dma else 0):
            with torch.cuda.stream(side[i % dma]):
                if ev is not None:
                    torch.cuda.current_stream().wait_event(ev)
                ddst[i].copy_(hsrc[i], non_blocking=True)
        del evs[:-4]
        host_copy_s[0] += time.perf_counter() - t0
    evs = []
    host_copy_s = [0.0]
    fn = step
    if graph and split:
        from blendtorch.parallel.step import CapturedStep

        def loss_fn(m, _):
            xi = inputs()
            if amp and cast == 'fused':
                out = m.forward_bf16(xi)
            else:
                with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
                    out = m(xi)
            return crit(out.float(), torch.ones(batch, device=dev))
        stepper = CapturedStep(model, opt, loss_fn, allreduce=False, split=True)
        probe = torch.zeros(1, device=dev)
        fn = (lambda: stepper(probe, mid=copies)) if dma_phase == 'mid' else (lambda: stepper(probe))
        for _ in range(3):
            fn()
    elif graph:
        g = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            step()
        fn = g.replay
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    host_copy_s[0] = 0.0
    t0 = time.perf_counter()
    for _ in range(iters):
        if dma and dma_phase != 'mid':
            copies()
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1000
    copy_ms = host_copy_s[0] / iters * 1000
    return {'variant': name, 'graph': graph, 'fused_adam': fused_adam, 'fused_bn': fused_bn, 'dma_streams': dma,
            'cast': cast, 'u8_input': u8, 'optim': optim, 'head': head, 'dma_phase': dma_phase if dma else None, 'split': split,
            'ms_per_step': round(ms, 4), 'images_per_s': round(batch / ms * 1000, 1),
            'host_ms_issuing_copies': round(copy_ms, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--only', default='')
    ap.add_argument('--graph', choices=['both', 'on', 'off'], default='both')
    ap.add_argument('--no-fused-adam', dest='fused_adam', action='store_false',
                    help='foreach Adam instead of torch.optim.Adam(fused=True) (one multi-tensor kernel)')
    ap.add_argument('--dma', type=int, default=0, help='side streams of background H2D traffic (9.8 MB per step)')
    ap.add_argument('--cpu-load', type=int, default=0, help='busy-looping CPU processes alongside (producer load)')
    ap.add_argument('--no-fused-bn', dest='fused_bn', action='store_false',
                    help='MIOpen BatchNorm + PyTorch LeakyReLU instead of the fused gfx950 op')
    ap.add_argument('--cast', choices=['autocast', 'fused'], default='autocast',
                    help='fused = Discriminator.forward_bf16 (one weight-cast launch per direction)')
    ap.add_argument('--optim', choices=['torch', 'gfx950'], default='torch')
    ap.add_argument('--head', choices=['torch', 'fused'], default='torch')
    ap.add_argument('--dma-phase', choices=['none', 'record', 'start', 'start_prev', 'mid'], default='none')
    ap.add_argument('--split', action='store_true', help='forward and backward as two graphs (CapturedStep split)')
    ap.add_argument('--u8', action='store_true', help='train on raw u8 RGBA frames decoded inside the step')
    args = ap.parse_args()
    import subprocess
    hogs = [subprocess.Popen([sys.executable, '-c', 'while True: pass']) for _ in range(args.cpu_load)]
    torch.backends.cudnn.benchmark = True
    names = [args.only] if args.only else list(VARIANTS)
    graphs = {'both': (False, True), 'on': (True,), 'off': (False,)}[args.graph]
    for n in names:
        for g in graphs:
            r = run(n, args.iters, args.batch, g, args.fused_adam, args.fused_bn, args.dma, args.cast, args.u8, args.optim,
                    args.dma_phase, args.split or args.dma_phase == 'mid', args.head)
            r['cpu_load'] = args.cpu_load
            print(json.dumps(r), flush=True)
    for h in hogs:
        h.kill()


if __name__ == '__main__':
    main()
