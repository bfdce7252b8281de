#!/usr/bin/env python
"""Host-resident frames -> decoded HBM batch, per path (the stream loader's
two ways in, without producers or sockets): ``ext.bench_frames_to_device``.

  copy   : B hipMemcpyAsync into a device staging buffer + decode kernel,
           frames spread over 1-4 streams (separate SDMA engines), per-batch
           host sync (latency) or pipelined over two staging buffers;
  direct : the decode kernel reads the registered host frames over PCIe.

Each line: path, streams, pipelined, us per batch, GB/s of frame bytes and a
staleness check (the host rewrites a byte per frame each iteration; a stale
read would show).  python benchmarks/frames_to_device.py [--batch 8,32]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', default='8,32')
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--kind', default='register', choices=['register', 'hostmalloc', 'register_thp'])
    a = ap.parse_args()
    import torch  # noqa: F401
    from blendtorch import ops
    e = ops.hip_ext()
    for B in (int(b) for b in a.batch.split(',')):
        for cin in (4, 3):
            rows = [('direct', 1, False)] + [('copy', k, pl) for k in (1, 2, 3, 4) for pl in (False, True)]
            for mode, k, pl in rows:
                us, gbs, stale = e.bench_frames_to_device(mode, a.kind, B, 480, 640, cin, a.iters, 0, k, pl)
                print(json.dumps({'path': mode, 'copy_streams': k if mode == 'copy' else None, 'pipelined': pl,
                                  'batch': B, 'cin': cin, 'host_memory': a.kind, 'us_per_batch': round(us, 1),
                                  'gbytes_per_s': round(gbs, 2), 'stale': stale}), flush=True)


if __name__ == '__main__':
    main()
