#!/usr/bin/env python
"""Minimal streaming example: 2 producer instances, 16 items, batch 4
(reference: examples/datagen/minimal.py).  Uses Blender when available,
else the native cube producer."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'pytorch-blender_amd'))
from torch.utils import data  # noqa: E402

from blendtorch import btt  # noqa: E402


def main():
    here = Path(__file__).parent
    launch = dict(scene=here / 'cube.blend', script=here / 'cube.blend.py', num_instances=2, named_sockets=['DATA'])
    if btt.discover_blender() is None:
        launch = dict(producer='cubesim', num_instances=2, named_sockets=['DATA'])
    with btt.BlenderLauncher(**launch) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'])
        ds.stream_length(16)
        dl = data.DataLoader(ds, batch_size=4, num_workers=4)
        for item in dl:
            print('Received', item['image'].shape, item['xy'].shape, item['btid'].tolist())


if __name__ == '__main__':
    main()
