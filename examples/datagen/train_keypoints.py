#!/usr/bin/env python
"""Supervised training on streamed renderings: regress the 8 projected cube
corners (the ``xy`` annotation every Cube frame carries) from the image.

This is the workload blendtorch exists for: Blender (or the C++ stand-in)
renders random poses, the annotations come with the frames, and a network
trains on them live. The reference shows only the data side
(examples/datagen/generate.py). On MI355X the whole consumer stays on the GPU:

* ``DeviceLoader`` lands the frames in HBM. The fused decode kernel writes them as
  bf16 channels-last (NHWC) tensors, scaled to [0, 1] with gamma 2.2, which is
  exactly what the first convolution reads;
* the model runs under bf16 autocast (MFMA convolutions);
* one process per GPU. ``torchrun --nproc-per-node N`` gives data parallelism with
  DDP (RCCL all-reduce of gradient buckets, overlapped with backward), and every
  rank streams from its own producers (shard mode).

    python examples/datagen/train_keypoints.py [--steps 300] [--batch 32] [--producers 8]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/datagen/train_keypoints.py

Prints one JSON line: samples/s, and the first and last loss (mean squared error of
the corner positions, in units of the image size).
"""
import argparse
import functools
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'pytorch-blender_amd'))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from blendtorch import btt, ops, parallel  # noqa: E402
from blendtorch.btt.gpu import DeviceLoader  # noqa: E402


def _block_factory(cin, cout, stride, fused=True):
    if fused:
        # BN + ReLU (a LeakyReLU of slope 0) as one gfx950 op on GPU training steps:
        # 8 passes over the activation per step instead of 13 (csrc/gpu/kernels.hip bn_*)
        norm_act = [ops.BatchNormLeakyReLU2d(cout, slope=0.0), nn.Identity()]
    else:
        norm_act = [nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]
    return nn.Sequential(nn.Conv2d(cin, cout, 3, stride, 1, bias=False), *norm_act)


class KeypointNet(nn.Module):
    """Small strided CNN: 3x480x640 -> 8 corners (x, y) in [0, 1]."""

    def __init__(self, width=32, corners=8, fused=True):
        super().__init__()
        w = width
        block = functools.partial(_block_factory, fused=fused)
        self.features = nn.Sequential(
            block(3, w, 2), block(w, w, 1),            # 240x320
            block(w, 2 * w, 2), block(2 * w, 2 * w, 1),  # 120x160
            block(2 * w, 4 * w, 2), block(4 * w, 4 * w, 1),  # 60x80
            block(4 * w, 8 * w, 2),                    # 30x40
            block(8 * w, 8 * w, 2),                    # 15x20
        )
        self.head = nn.Sequential(ops.AdaptiveAvgPool2d((3, 4)) if fused else nn.AdaptiveAvgPool2d((3, 4)), nn.Flatten(), nn.Linear(8 * w * 12, 256),
                                  nn.ReLU(inplace=True), nn.Linear(256, 2 * corners))

    def forward(self, x):
        return self.head(self.features(x))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--batch', type=int, default=32, help='per GPU')
    ap.add_argument('--producers', type=int, default=8, help='per GPU')
    ap.add_argument('--lr', type=float, default=2e-3)
    ap.add_argument('--start-port', type=int, default=0)
    ap.add_argument('--json', default=None)
    ap.add_argument('--no-fused-bn', dest='fused_bn', action='store_false',
                    help='MIOpen BatchNorm + ReLU instead of the fused gfx950 op')
    a = ap.parse_args(argv)

    rank, world, dev = parallel.init_distributed()
    W, H = 640, 480
    model = KeypointNet(fused=a.fused_bn).to(dev).to(memory_format=torch.channels_last)
    if world > 1:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.AdamW(model.parameters(), lr=a.lr, fused=dev.type == 'cuda')   # one multi-tensor kernel
    scale = torch.tensor([W, H], dtype=torch.float32, device=dev)
    port = a.start_port or (25000 + (os.getpid() % 100) * 40 if world == 1 else 25000 + rank * 40)
    with btt.BlenderLauncher(producer='cubesim', num_instances=a.producers, named_sockets=['DATA'], proto='ipc',
                             start_port=port, seed=1000 * rank + 1,
                             instance_args=[['--mode', 'rgba', '--shm', '32']] * a.producers) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=a.batch, device=dev,
                          max_items=(a.steps + 5) * a.batch, meta_to_device=True,
                          decode=ops.DecodeConfig.unit(channels='rgb', gamma=2.2, dtype='bfloat16', layout='nhwc'))
        losses = []
        t0 = None
        for step, b in enumerate(dl):
            if step == 5:           # warm-up: MIOpen kernel selection, producer start-up
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
            x = b['image'].permute(0, 3, 1, 2)                       # NHWC storage, NCHW view
            target = (b['xy'].to(torch.float32) / scale).flatten(1)  # [B, 16] in [0, 1]
            with torch.autocast('cuda', dtype=torch.bfloat16):
                pred = model(x)
            loss = nn.functional.mse_loss(pred.float(), target)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            losses.append(loss.detach())
            if step + 1 >= a.steps + 5:
                break
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
    losses = torch.stack(losses).float().cpu()
    stats = {'samples_per_s': a.steps * a.batch / dt}
    agg = parallel.all_gather_stats(stats, dev)
    if rank == 0:
        head, tail = float(losses[:10].mean()), float(losses[-10:].mean())
        res = {'metric': 'keypoint training samples/s (whole job)', 'value': round(sum(s['samples_per_s'] for s in agg), 1),
               'n_gpus': world, 'batch_per_gpu': a.batch, 'steps': a.steps, 'dtype': 'bf16',
               'loss_first10': round(head, 5), 'loss_last10': round(tail, 5), 'ms_per_step': round(dt / a.steps * 1e3, 3)}
        print(json.dumps(res), flush=True)
        if a.json:
            Path(a.json).write_text(json.dumps(res, indent=2))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
