"""FusedAdam variants on the bench discriminator's parameters (0.7 M), each
captured in a HIP graph and replayed: device time per optimizer step.

    python scripts/adam_bench.py [--iters 300]

Variants: two launches (adam_schedule + adam_update), one launch, one
launch + bf16 conv shadows (+ transposes), + gradient clearing.
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402
from blendtorch.models import Discriminator  # noqa: E402


def run(variant, iters):
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    opt = ops.FusedAdam(m.parameters(), lr=2e-4)
    for p in m.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    if variant == 'one_launch':
        opt._one_launch = True
    if variant in ('shadows', 'shadows_zero'):
        m.use_optimizer_shadows(opt)
    if variant == 'shadows_zero':
        opt.set_zero_grads(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            opt.step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        opt.step()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=300)
    a = ap.parse_args()
    out = {v: round(run(v, a.iters), 2) for v in ('two_launch', 'one_launch', 'shadows', 'shadows_zero')}
    print(json.dumps({'adam_us_per_step': out}), flush=True)


if __name__ == '__main__':
    main()
