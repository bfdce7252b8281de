#!/usr/bin/env python
"""Reference-harness benchmark: the same measurement as the reference's
``benchmarks/benchmark.py:7-47`` (4 producer instances, ``stream_length(512)``,
batch 8, 5 s start-up sleep, first batch excluded, ``sec/image`` over 504
images and ``sec/batch`` over 63 batches), on either consumer path:

* ``--path cpu``  -- exactly the reference's consumer: ``RemoteIterableDataset``
  + ``torch.utils.data.DataLoader(num_workers=4)`` (pickle + default_collate +
  worker shared-memory transfer), items stay on the host;
* ``--path gpu``  -- the MI355X path: :class:`blendtorch.btt.DeviceLoader`
  (native receive into pinned memory, zero-copy fused decode into HBM).

Producers are the C++ headless stand-ins (``--producer cubesim``, default) or
the scene scripts under a Blender executable (``--producer blender``: real
Blender if on PATH, else the bundled headless emulation).

    python benchmarks/benchmark.py [--scene cube|falling_cubes] [--path cpu|gpu]
                                   [--instances 4] [--mode rgb|rgba] [--json]

The headline, driver-facing benchmark (steady state, many batches, JSON) is
``bench.py`` at the repository root.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'pytorch-blender_amd'))

BATCH = 8
INSTANCES = 4
WORKER_INSTANCES = 4
NUM_ITEMS = 512
EXAMPLES_DIR = ROOT / 'examples' / 'datagen'


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument('--scene', default='cube', choices=['cube', 'falling_cubes'])
    ap.add_argument('--path', default='cpu', choices=['cpu', 'gpu'])
    ap.add_argument('--producer', default='cubesim', choices=['cubesim', 'blender'])
    ap.add_argument('--instances', type=int, default=INSTANCES)
    ap.add_argument('--workers', type=int, default=WORKER_INSTANCES)
    ap.add_argument('--items', type=int, default=NUM_ITEMS)
    ap.add_argument('--batch', type=int, default=BATCH)
    ap.add_argument('--mode', default='rgb', choices=['rgb', 'rgba'],
                    help="frame format (the reference's cube.blend.py renders 'rgb'; its README says RGBA)")
    ap.add_argument('--sleep', type=float, default=5.0, help='start-up wait before consuming (reference: 5 s)')
    ap.add_argument('--start-port', type=int, default=11000)
    ap.add_argument('--json', action='store_true', help='print one JSON line instead of the reference text')
    ap.add_argument('--shm-slots', type=int, default=0,
                    help='>0: producers use the same-host shared-memory frame ring (BlenderLauncher(shm_slots=N))')
    args = ap.parse_args(argv)

    import torch
    import torch.utils.data as data
    from blendtorch import btt

    script_args = ['--mode', args.mode]
    if args.producer == 'cubesim':
        launch_args = dict(producer='cubesim', instance_args=[['--scene', args.scene] + script_args] * args.instances)
    else:
        import shutil
        from blendtorch import btb
        # real Blender when installed, else the bundled headless emulation
        blend_path = None if shutil.which('blender') else str(Path(btb.__file__).parent / 'headless' / 'bin')
        launch_args = dict(scene=EXAMPLES_DIR / f'{args.scene}.blend', script=EXAMPLES_DIR / f'{args.scene}.blend.py',
                           blend_path=blend_path, instance_args=[script_args] * args.instances)
    launch_args.update(num_instances=args.instances, named_sockets=['DATA'], start_port=args.start_port,
                       shm_slots=args.shm_slots)

    with btt.BlenderLauncher(**launch_args) as bl:
        addrs = bl.launch_info.addresses['DATA']
        if args.path == 'cpu':
            ds = btt.RemoteIterableDataset(addrs)
            ds.stream_length(args.items)
            dl = data.DataLoader(ds, batch_size=args.batch, num_workers=args.workers, shuffle=False)
        else:
            from blendtorch.btt.gpu import DeviceLoader
            from blendtorch.ops import DecodeConfig
            dl = DeviceLoader(addrs, batch_size=args.batch, max_items=args.items,
                              decode=DecodeConfig.unit(channels='rgb', gamma=2.2))

        # Wait to avoid timing startup times of the producers
        time.sleep(args.sleep)

        t0 = None
        imgshape = None
        n = 0
        for item in dl:
            if t0 is None:  # 1st is warmup
                t0 = time.time()
                imgshape = tuple(item['image'].shape)
            n += len(item['image'])
        if args.path == 'gpu':
            torch.cuda.synchronize()
        assert n == args.items, n
        t1 = time.time()

    N = args.items - args.batch
    B = args.items // args.batch - 1
    if args.json:
        print(json.dumps({'path': args.path, 'scene': args.scene, 'mode': args.mode, 'instances': args.instances,
                          'shm_slots': args.shm_slots,
                          'sec_per_image': (t1 - t0) / N, 'sec_per_batch': (t1 - t0) / B,
                          'images_per_sec': N / (t1 - t0), 'shape': list(imgshape)}))
    else:
        print(f'Time {(t1 - t0) / N:.3f}sec/image, {(t1 - t0) / B:.3f}sec/batch, shape {imgshape}')


if __name__ == '__main__':
    main()
