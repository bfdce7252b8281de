#!/usr/bin/env python
"""Short driver for rocprofv3 --pmc passes over the two frames->device paths
(8 x 640x480 RGBA frames in registered host memory):
  copy   -- 8 hipMemcpyAsync + decode from HBM staging
  direct -- decode kernel reads the host frames over PCIe itself
so the counters show where the decode kernel's bytes come from (TCC_EA0_RDREQ_IO_* vs _DRAM_*)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / 'pytorch-blender_amd'))
from blendtorch import ops  # noqa: E402

e = ops.hip_ext()
for mode in ('copy', 'direct'):
    us, gbs, stale = e.bench_frames_to_device(mode, 'register', 8, 480, 640, 4, 10, 0, 1, False)
    print(mode, round(us, 1), 'us/batch', round(gbs, 1), 'GB/s', 'stale', stale, flush=True)
