"""Host frames -> HBM over both PCIe read paths at once: the decode kernel's
own loads (direct) for the first n frames of each batch, SDMA copies for the
rest (``bench_frames_to_device('hybrid:<n>', ...)``).  Prints one JSON line
per configuration.   python scripts/f2d_hybrid.py [--batch 32]"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))
import torch  # noqa: E402,F401

from blendtorch import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--batch', type=int, default=32)
ap.add_argument('--iters', type=int, default=300)
a = ap.parse_args()
e = ops.hip_ext()
B = a.batch
for streams in (2, 4):
    for nd in (B, B * 7 // 8, B * 3 // 4, B // 2, 0):
        mode = 'direct' if nd == B else f'hybrid:{nd}'
        us, gbs, stale = e.bench_frames_to_device(mode, 'register', B, 480, 640, 4, a.iters, 0, streams, True)
        print(json.dumps({'mode': mode, 'batch': B, 'direct_frames': nd, 'copy_streams': streams,
                          'us_per_batch': round(us, 1), 'gbytes_per_s': round(gbs, 2), 'stale': stale}), flush=True)
