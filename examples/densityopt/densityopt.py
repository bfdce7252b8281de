#!/usr/bin/env python
"""Adapt simulation parameters to a target image distribution (densityopt).

MI355X-native version of the reference example
(examples/densityopt/densityopt.py): supershape producers render 64x64
images for parameters sent over the duplex channel; rendered batches are
decoded straight into HBM by the GPU loader ((x - 127.5) / 127.5, HWC->CHW
on the gfx950 decode kernel); a DCGAN discriminator tells target from
simulated images, and the simulation parameters (LogNormal over the
supershape frequencies m1, m2) follow the score-function gradient
(blendtorch_stochopt.pdf eq. 4-5).

Producers: the native ``supershapesim`` stand-in (default) or real Blender
with ``supershape.blend.py`` (``--producer blender``; needs the external
supershape package inside Blender).

    python examples/densityopt/densityopt.py [--num-epochs 70] [--random-start] [--json out.json]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'pytorch-blender_amd'))

import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim

from blendtorch import btt
from blendtorch.btt.gpu import DeviceLoader
from blendtorch.models import Discriminator, ProbModel
from blendtorch.ops import DecodeConfig

BATCH = 64
TARGET_LABEL = 1
SIM_LABEL = 0
SIM_INSTANCES = 4
DEFAULT_MEAN_TARGET = 2.25
DEFAULT_STD_TARGET = 0.1
BASELINE_ALPHA = 0.9


def update_simulations(remotes, params):
    """Split N parameter samples into one chunk per instance (with their ids)."""
    ids = torch.arange(params.shape[0]).long()
    for remote, subset, subset_ids in zip(remotes, torch.chunk(params, len(remotes)),
                                          torch.chunk(ids, len(remotes))):
        remote.send(shape_params=subset.cpu().numpy(), shape_ids=subset_ids.numpy())


def item_transform(item):
    """CPU path: the reference's per-item numpy transform."""
    x = (item['image'].astype(np.float32) - 127.5) / 127.5
    return np.transpose(x, (2, 0, 1)), item['shape_id']


def cpu_stream(addresses):
    """CPU fallback: RemoteIterableDataset + DataLoader, as the reference does."""
    from torch.utils import data
    ds = btt.RemoteIterableDataset(addresses, item_transform=item_transform, timeoutms=30000)
    for img, sid in data.DataLoader(ds, batch_size=BATCH, num_workers=0):
        yield {'image': img, 'shape_id': sid}


def run(args):
    dev = torch.device(args.device)
    netD = Discriminator(fused=args.fused_bn).to(dev)
    here = Path(__file__).resolve().parent
    launch = dict(num_instances=args.instances, named_sockets=['DATA', 'CTRL'], start_port=args.start_port)
    if args.producer == 'blender':
        launch.update(scene=here / 'supershape.blend', script=here / 'supershape.blend.py')
    else:
        launch.update(producer='supershapesim')
    with btt.BlenderLauncher(**launch) as bl:
        if dev.type == 'cuda':
            sim = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=BATCH, device=dev, prefetch=2,
                               decode=DecodeConfig.densityopt(channels='rgb'), timeoutms=30000)
            gen_sim = iter(sim)
        else:
            gen_sim = cpu_stream(bl.launch_info.addresses['DATA'])
        remotes = [btt.DuplexChannel(a) for a in bl.launch_info.addresses['CTRL']]

        if args.random_start:
            mu_target = np.random.uniform(0.0, 3, size=2).astype(np.float32)
        else:
            mu_target = [DEFAULT_MEAN_TARGET, DEFAULT_MEAN_TARGET]
        std_target = [DEFAULT_STD_TARGET, DEFAULT_STD_TARGET]
        print('Target params:', mu_target, std_target)
        # one batch of target images (kept resident on the device)
        target = ProbModel(mu_target, std_target)
        update_simulations(remotes, ProbModel.to_supershape(target.sample(BATCH)))
        real_img = next(gen_sim)['image'].clone()

        mu = np.asarray(mu_target) + np.random.randn(2) if args.random_start else [1.2, 3.0]
        pm = ProbModel(mu, [0.4, 0.4])
        optD = optim.Adam(netD.parameters(), lr=5e-5, betas=(0.5, 0.999), fused=dev.type == 'cuda')
        optS = optim.Adam(pm.parameters(), lr=5e-2, betas=(0.7, 0.999))
        crit = nn.BCELoss(reduction='none')
        b = 0.7
        first = True
        history = []
        samples = pm.sample(BATCH)
        update_simulations(remotes, pm.to_supershape(samples))
        t0 = time.time()
        epoch = 0
        wait_s = 0.0
        while True:
            tw = time.time()
            sim_batch = next(gen_sim)
            wait_s += time.time() - tw
            sim_img, sim_shape_id = sim_batch['image'], sim_batch['shape_id']
            # discriminator step
            label = torch.full((BATCH,), TARGET_LABEL, dtype=torch.float32, device=dev)
            netD.zero_grad()
            out = netD(real_img)
            crit(out, label).mean().backward()
            D_real = out.mean().item()
            label.fill_(SIM_LABEL)
            out = netD(sim_img)
            crit(out, label).mean().backward()
            D_sim = out.mean().item()
            if (D_real - D_sim) < 0.7:
                optD.step()
                if args.verbose:
                    print('D step: mean real', D_real, 'mean sim', D_sim)
            # simulation-parameter step (score-function gradient)
            if not first or (D_real - D_sim) >= 0.7:
                optS.zero_grad()
                label.fill_(TARGET_LABEL)
                with torch.no_grad():
                    out = netD(sim_img)
                    errS_sim = crit(out, label).cpu()
                log_probs = pm.log_prob(samples)
                loss = log_probs[sim_shape_id] * (errS_sim - b)
                loss.mean().backward()
                optS.step()
                b = errS_sim.mean() if first else BASELINE_ALPHA * errS_sim.mean() + (1 - BASELINE_ALPHA) * b
                if args.verbose:
                    print('S step:', pm.m1m2_mean.detach().numpy(), torch.exp(pm.m1m2_log_std).detach().numpy())
                first = False
            samples = pm.sample(BATCH)
            update_simulations(remotes, pm.to_supershape(samples))
            history.append(pm.readable_params())
            epoch += 1
            if epoch > args.num_epochs:
                break
        dt = time.time() - t0
        tgt = torch.tensor(np.concatenate((mu_target, std_target))).float()
        diff = (tgt - history[-1]).abs()
        print('Abs.Diff to true params', diff)
        return {'iterations': epoch, 'seconds': dt, 'iterations_per_s': epoch / dt, 'sim_wait_s': wait_s,
                'images_per_s': epoch * BATCH / dt, 'final_params': history[-1].tolist(),
                'target': tgt.tolist(), 'abs_diff': diff.tolist()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--random-start', action='store_true')
    ap.add_argument('--num-epochs', default=70, type=int)
    ap.add_argument('--instances', default=SIM_INSTANCES, type=int)
    ap.add_argument('--producer', choices=['supershapesim', 'blender'], default='supershapesim')
    ap.add_argument('--device', default='cuda' if torch.cuda.is_available() else 'cpu')
    ap.add_argument('--start-port', default=26000, type=int)
    ap.add_argument('--json', default=None)
    ap.add_argument('--no-fused-bn', dest='fused_bn', action='store_false',
                    help='discriminator with MIOpen BatchNorm + PyTorch LeakyReLU instead of the fused gfx950 op')
    ap.add_argument('--verbose', action='store_true')
    args = ap.parse_args()
    res = run(args)
    print(json.dumps(res))
    if args.json:
        Path(args.json).write_text(json.dumps(res, indent=2))


if __name__ == '__main__':
    main()
