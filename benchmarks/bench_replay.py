#!/usr/bin/env python
"""HBM replay throughput: frames resident in a DeviceReplayBuffer, random
batches gathered + decoded by one fused kernel per batch.

    python benchmarks/bench_replay.py [--frames 4096] [--batch 8] [--steps 2000] [--fill producers|synthetic]

``--fill producers`` streams the frames from headless Cube producers through
a raw-u8 DeviceLoader (the record-once, train-many-epochs workflow);
``synthetic`` writes random frames (same shape) straight into the store.
Prints one JSON line (images/s of decoded fp32 CHW batches).
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'pytorch-blender_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=4096)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--fill', choices=['producers', 'synthetic'], default='synthetic')
    ap.add_argument('--dtype', choices=['float32', 'bfloat16'], default='float32')
    ap.add_argument('--graph', action='store_true', help='replay a HIP-graph-captured sampler')
    ap.add_argument('--sampler', choices=['fused', 'legacy'], default='fused',
                    help='fused: ONE launch (Philox draw + gather + decode + metadata); legacy: randint, '
                         'decode_gather and one index_select per metadata key (the round-1 path)')
    a = ap.parse_args()

    import torch
    from blendtorch import btt, ops
    from blendtorch.btt.replay import DeviceReplayBuffer
    dev = torch.device('cuda', 0)
    rb = DeviceReplayBuffer(a.frames, device=dev)
    t0 = time.perf_counter()
    if a.fill == 'synthetic':
        g = torch.Generator(device=dev).manual_seed(0)
        for s in range(0, a.frames, 256):
            n = min(256, a.frames - s)
            rb.extend(torch.randint(0, 256, (n, 480, 640, 4), dtype=torch.uint8, device=dev, generator=g),
                      frameid=torch.arange(s, s + n, device=dev))
    else:
        from blendtorch.btt.gpu import DeviceLoader
        with btt.BlenderLauncher(producer='cubesim', num_instances=8, named_sockets=['DATA'], proto='ipc',
                                 start_port=24000, instance_args=[['--mode', 'rgba', '--shm', '32']] * 8) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=64, max_items=a.frames, device=dev,
                              decode=ops.DecodeConfig.raw())
            rb.fill_from(dl, a.frames)
    torch.cuda.synchronize()
    fill_s = time.perf_counter() - t0
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2, dtype=a.dtype)
    def legacy():
        idx = torch.randint(0, len(rb), (a.batch,), device=dev)
        out = {'image': ops.decode_gather(rb.store, idx, cfg), 'index': idx}
        out.update({k: v.index_select(0, idx) for k, v in rb.meta.items()})
        return out

    if a.sampler == 'legacy':
        sample = legacy
    else:
        sample = rb.graphed_sampler(a.batch, cfg) if a.graph else (lambda: rb.sample(a.batch, cfg))
    for _ in range(a.warmup):
        sample()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        b = sample()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    H, W, C = rb.frame_shape
    moved = a.batch * H * W * (C + cfg.cout * (4 if a.dtype == 'float32' else 2))   # bytes read + written
    print(json.dumps({'metric': 'replay images/s (HBM store -> gather+decode)', 'value': round(a.steps * a.batch / dt, 1),
                      'sampler': a.sampler, 'us_per_batch': round(dt / a.steps * 1e6, 2),
                      'effective_tbps': round(moved * a.steps / dt / 1e12, 3),
                      'unit': 'images/s', 'batch': a.batch, 'frames': a.frames, 'store_gb': round(rb.nbytes / 1e9, 2),
                      'fill': a.fill, 'fill_s': round(fill_s, 2), 'ms_per_batch': round(dt / a.steps * 1e3, 4),
                      'dtype': a.dtype, 'graph': a.graph, 'out_shape': list(b['image'].shape)}), flush=True)


if __name__ == '__main__':
    main()
