#!/usr/bin/env python
"""Generate, record and replay synthetic data (reference: examples/datagen/generate.py).

    python generate.py [--scene cube|falling_cubes] [--record] [--replay] [--gpu]

--record writes one .btr file per DataLoader worker to tmp/record_*.btr;
--replay reads them back (shuffled) without any producer running;
--gpu streams through the native GPU loader (gamma on the device) instead
of DataLoader workers.  Figures of the first batches go to tmp/.
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'pytorch-blender_amd'))
import numpy as np  # noqa: E402
from torch.utils import data  # noqa: E402

from blendtorch import btt  # noqa: E402

HERE = Path(__file__).resolve().parent


def gamma_correct(x):
    """The reference's item-level gamma (same float32 math as the GPU LUT)."""
    return np.uint8(255.0 * (x.astype(np.float32) / 255) ** (1 / 2.2))


def item_transform(item):
    item['image'] = gamma_correct(item['image'])
    return item


def iterate(dl, n):
    for i, item in enumerate(dl):
        img, xy = item['image'], item['xy']
        print(f'batch {i}: image {tuple(img.shape)} xy {tuple(xy.shape)} btid {item["btid"].tolist()}')
        if i == 0:
            save_figure(img, xy)
        if i + 1 >= n:
            break


def save_figure(img, xy):
    try:
        import matplotlib
        matplotlib.use('Agg')
        import matplotlib.pyplot as plt
    except ImportError:
        return
    (HERE / 'tmp').mkdir(exist_ok=True)
    img = img.cpu().numpy() if hasattr(img, 'cpu') else img
    if img.shape[1] in (3, 4) and img.ndim == 4:
        img = img.transpose(0, 2, 3, 1)
    fig, axs = plt.subplots(1, min(4, len(img)), figsize=(12, 3))
    for k, ax in enumerate(np.atleast_1d(axs)):
        ax.imshow(img[k][..., :3])
        ax.scatter(xy[k][:, 0], xy[k][:, 1], s=4, c='r')
        ax.axis('off')
    fig.savefig(HERE / 'tmp' / 'output.png')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scene', default='cube', choices=['cube', 'falling_cubes'])
    ap.add_argument('--replay', action='store_true')
    ap.add_argument('--record', action='store_true')
    ap.add_argument('--gpu', action='store_true')
    ap.add_argument('--batches', type=int, default=16)
    a = ap.parse_args()
    prefix = HERE / 'tmp' / 'record'
    if a.replay:
        ds = btt.FileDataset(prefix, item_transform=item_transform)
        iterate(data.DataLoader(ds, batch_size=4, num_workers=4, shuffle=True), a.batches)
        return
    launch = dict(scene=HERE / f'{a.scene}.blend', script=HERE / f'{a.scene}.blend.py', num_instances=4,
                  named_sockets=['DATA'])
    if btt.discover_blender() is None:
        launch = dict(producer='cubesim', num_instances=4, named_sockets=['DATA'],
                      instance_args=[['--scene', a.scene]] * 4)
    with btt.BlenderLauncher(**launch) as bl:
        addr = bl.launch_info.addresses['DATA']
        if a.gpu:
            dl = btt.DeviceLoader(addr, batch_size=4, max_items=4 * a.batches,
                                  decode=btt.DecodeConfig(channels='rgb', gamma=2.2, dtype='uint8'))
            iterate(dl, a.batches)
            return
        ds = btt.RemoteIterableDataset(addr, item_transform=item_transform)
        ds.stream_length(4 * a.batches)
        if a.record:
            ds.enable_recording(prefix)
        iterate(data.DataLoader(ds, batch_size=4, num_workers=4, shuffle=False), a.batches)


if __name__ == '__main__':
    main()
