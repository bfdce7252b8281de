#!/usr/bin/env python
"""Adapt simulation parameters to a target image distribution (densityopt).

MI355X-native version of the reference example
(examples/densityopt/densityopt.py): supershape producers render 64x64
images for parameters sent over the duplex channel; rendered batches are
decoded straight into HBM by the GPU loader ((x - 127.5) / 127.5 on the
gfx950 decode kernel, bf16 channels-last for the MFMA discriminator); a DCGAN
discriminator tells target from simulated images, and the simulation
parameters (LogNormal over the supershape frequencies m1, m2) follow the
score-function gradient (blendtorch_stochopt.pdf eq. 4-5).

The whole iteration -- gated D step, gated S step, baseline, resampling --
is one device program (:class:`blendtorch.models.densityopt.DensityOptStep`),
replayed from a HIP graph; the only host synchronisation per iteration is
the copy of the next parameters the producers must render.

Data parallel: run with ``torchrun --nproc-per-node N`` (or ``--gpus N``):
every rank launches its own producers, rank 0 draws the parameter samples
and broadcasts them over RCCL, each rank sends its chunk to its producers
(the reference's partition of work over instances, densityopt.py:95-107),
and gradients / gate statistics are averaged in-graph.

Producers: the native ``supershapesim`` stand-in (default) or real Blender
with ``supershape.blend.py`` (``--producer blender``; needs the external
supershape package inside Blender).

    python examples/densityopt/densityopt.py [--num-epochs 70] [--random-start] [--json out.json]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / 'pytorch-blender_amd'))

from blendtorch.utils import ensure_hw_queues  # noqa: E402

# before the HIP runtime starts: HIP's 4 queues for a training step with in-graph
# RCCL collectives (8 slowed the bench's graphed DP step by 27 %, profiles/r4/pg_tax.md)
ensure_hw_queues(4, exact=True)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from blendtorch import btt, parallel  # noqa: E402
from blendtorch.models import Discriminator, ProbModel  # noqa: E402
from blendtorch.models.densityopt import DensityOptStep  # noqa: E402
from blendtorch.ops import DecodeConfig  # noqa: E402
from blendtorch.utils.images import save_image  # noqa: E402

BATCH = 64
SIM_INSTANCES = 4
DEFAULT_MEAN_TARGET = 2.25
DEFAULT_STD_TARGET = 0.1
# supershape row template: (m, a=1, b=1, n1=n2=n3=3), m from the samples (densityopt.py:82-93)
_ROW = np.array([0, 1, 1, 3, 3, 3], dtype=np.float32)


def supershape_params(m1, m2):
    """(N, 2, 6) float32 supershape parameters for frequency samples m1, m2."""
    p = np.tile(_ROW, (len(m1), 2, 1)).astype(np.float32)
    p[:, 0, 0] = m1
    p[:, 1, 0] = m2
    return p


def update_simulations(remotes, m1, m2, ids):
    """Split this rank's samples into one chunk per local instance, with their
    global ids (reference: densityopt.py:95-107)."""
    params = supershape_params(m1, m2)
    for remote, sub, sub_ids in zip(remotes, np.array_split(params, len(remotes)), np.array_split(ids, len(remotes))):
        remote.send(shape_params=sub, shape_ids=np.asarray(sub_ids, dtype=np.int64))


def item_transform(item):
    """CPU path: the reference's per-item numpy transform."""
    x = (item['image'].astype(np.float32) - 127.5) / 127.5
    return np.transpose(x, (2, 0, 1)), item['shape_id']


def cpu_stream(addresses, batch):
    """CPU fallback: RemoteIterableDataset + DataLoader, as the reference does."""
    from torch.utils import data
    ds = btt.RemoteIterableDataset(addresses, item_transform=item_transform, timeoutms=30000)
    # the dataset's default max_items=100000 (reference dataset.py:22) ends the
    # stream after 1562 iterations of 64 with a short batch of 32: the
    # reference's own loop cannot run past epoch 1562; stream without bound
    ds.stream_length(1 << 62)
    for img, sid in data.DataLoader(ds, batch_size=batch, num_workers=0):
        yield {'image': img, 'shape_id': sid}


def run(args):
    rank, world, dev = parallel.init_distributed(backend=args.backend)
    if args.device == 'cpu':
        dev = torch.device('cpu')
    comm = parallel.DeviceComm(device=dev if dev.type == 'cuda' else None, dedicated=True) if world > 1 else None
    if comm is not None and comm.backend == 'nccl':
        comm.selfcheck()
    B = args.batch
    bf16 = dev.type == 'cuda' and not args.fp32
    here = Path(__file__).resolve().parent
    launch = dict(num_instances=args.instances, named_sockets=['DATA', 'CTRL'],
                  start_port=args.start_port + 50 * rank, seed=1000 * rank + 17)
    if args.producer == 'blender':
        launch.update(scene=here / 'supershape.blend', script=here / 'supershape.blend.py')
    else:
        launch.update(producer='supershapesim')
    rng = np.random.default_rng(args.seed)
    with btt.BlenderLauncher(**launch) as bl:
        if dev.type == 'cuda':
            from blendtorch.btt.gpu import DeviceLoader
            # bf16 channels-last with the blue channel repeated as a 4th: the
            # first MFMA conv reads 8-byte pixels and its weight ignores channel 3
            dec = (DecodeConfig.densityopt(channels=(0, 1, 2, 2), dtype='bfloat16', layout='nhwc') if bf16
                   else DecodeConfig.densityopt(channels='rgb'))
            # a fixed ring of output tensors: the fused step keeps a sim-half graph per
            # ring tensor and reads each batch where the loader decoded it (no copy)
            sim = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=B, device=dev, prefetch=2,
                               decode=dec, timeoutms=30000, reuse_buffers=True)
            gen_sim = iter(sim)
        else:
            gen_sim = cpu_stream(bl.launch_info.addresses['DATA'], B)

        def as_input(img):
            return img.permute(0, 3, 1, 2) if bf16 else img.to(dev)

        remotes = [btt.DuplexChannel(a) for a in bl.launch_info.addresses['CTRL']]
        if args.random_start:
            mu_target = rng.uniform(0.0, 3, size=2).astype(np.float32)
            if comm is not None:        # one target for every rank
                t = torch.as_tensor(mu_target, device=comm.device)
                mu_target = comm.broadcast_(t, 0).cpu().numpy()
        else:
            mu_target = np.array([DEFAULT_MEAN_TARGET, DEFAULT_MEAN_TARGET], dtype=np.float32)
        std_target = np.array([DEFAULT_STD_TARGET, DEFAULT_STD_TARGET], dtype=np.float32)
        if rank == 0:
            print('Target params:', mu_target, std_target, flush=True)
        # one batch of target images per rank, kept resident on the device
        target = ProbModel(mu_target, std_target)
        ts = target.sample(B)
        update_simulations(remotes, ts['m1'].numpy(), ts['m2'].numpy(), np.arange(B))
        real = as_input(next(gen_sim)['image']).clone()

        torch.manual_seed(args.seed)
        netD = Discriminator(fused=not args.no_fused_bn).to(dev)
        mu = (np.asarray(mu_target) + rng.standard_normal(2)) if args.random_start else [1.2, 3.0]
        pm = ProbModel(mu, [0.4, 0.4]).to(dev)
        if comm is not None:   # identical initial D and ProbModel on every rank
            for t in list(netD.state_dict().values()) + list(pm.state_dict().values()):
                if t.is_floating_point():
                    comm.broadcast_(t, 0)
        if bf16:
            netD = netD.to(memory_format=torch.channels_last)
        step = DensityOptStep(netD, pm, real, B, comm=comm, bf16=bf16, graph=not args.no_graph,
                              fused=None if not args.unfused_sstep else False, seed=args.seed)
        pin = dev.type == 'cuda'
        host_samples = torch.empty((2, B), dtype=torch.float32, pin_memory=pin)
        host_params = torch.empty(4, dtype=torch.float32, pin_memory=pin)
        host_stats = torch.empty(4, dtype=torch.float32, pin_memory=pin)
        ids = np.arange(rank * B, (rank + 1) * B)

        def fetch():
            """The one device->host hand-off per iteration: next samples (+ logging scalars).
            Fused step: its kernel wrote them to host-mapped memory -- wait and read."""
            if step.fused:
                torch.cuda.current_stream(dev).synchronize()
                hs = step.host_state()
                host_params.copy_(hs['params'])
                host_stats[:2].copy_(hs['stats'])
                host_stats[2:3].copy_(hs['gate_d'])
                host_stats[3:4].copy_(hs['gate_s'])
                return hs['samples'].numpy().copy()
            mine, _ = step.my_samples()
            host_samples.copy_(mine, non_blocking=pin)
            host_params.copy_(step.params_out, non_blocking=pin)
            host_stats[:2].copy_(step.stats, non_blocking=pin)
            host_stats[2:3].copy_(step.gate_d, non_blocking=pin)
            host_stats[3:4].copy_(step.gate_s, non_blocking=pin)
            if pin:
                torch.cuda.current_stream(dev).synchronize()
            return host_samples.numpy()

        step.start()
        s = fetch()
        update_simulations(remotes, s[0], s[1], ids)
        if not args.no_prefetch:
            step.prefetch()    # the D step's real-batch half runs while the producers render
        history = []
        d_steps = s_steps = 0
        # rank 0 writes the reference's outputs: image grids of the target and
        # the simulated batch every --image-every epochs (densityopt.py:321-323),
        # encoded on a writer thread so the loop does not wait for zlib
        out_dir = Path(args.out_dir) if args.out_dir else None
        writer = None
        if out_dir is not None and rank == 0:
            out_dir.mkdir(parents=True, exist_ok=True)
            from concurrent.futures import ThreadPoolExecutor
            writer = ThreadPoolExecutor(max_workers=1)
        pending = []
        # steady state: iterations after the warm-up / capture ones, timed per phase
        steady_from = max(args.steady_skip, step.warmup + 2)
        ph = dict.fromkeys(('sim_wait', 'step_enqueue', 'fetch', 'send', 'prefetch', 'images', 'gpu_iteration',
                            'gpu_real_half'), 0.0)
        ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) if pin else None
        n_steady, t_steady = 0, None
        real_rec = False       # ev[2:] hold a prefetched real half whose time is not yet read
        t0 = time.time()
        wait_s = 0.0
        epoch = 0
        cpu0 = None
        prod_pids = [p.pid for p in bl.launch_info.processes] if bl.launch_info is not None else []
        while True:
            steady = epoch >= steady_from
            if steady and t_steady is None:
                t_steady = time.perf_counter()
                cpu0 = _cpu_snapshot(prod_pids)
            ta = time.perf_counter()
            batch = next(gen_sim)
            tb = time.perf_counter()
            wait_s += tb - ta
            sid = batch['shape_id']
            sid = sid if isinstance(sid, torch.Tensor) else torch.as_tensor(np.asarray(sid))
            sim_img = as_input(batch['image'])
            if ev is not None and steady:
                ev[0].record()
            step(sim_img, sid)
            if ev is not None and steady:
                ev[1].record()
            tc = time.perf_counter()
            s = fetch()
            td = time.perf_counter()
            if real_rec:       # fetch() synchronised: the real half prefetched last iteration is done
                ph['gpu_real_half'] += ev[2].elapsed_time(ev[3]) * 1e-3
                real_rec = False
            update_simulations(remotes, s[0], s[1], ids)
            te = time.perf_counter()
            if not args.no_prefetch:
                if ev is not None and steady:
                    ev[2].record()
                step.prefetch()
                if ev is not None and steady:
                    ev[3].record()
                    real_rec = True
            tp = time.perf_counter()
            d_steps += int(host_stats[2] > 0)
            s_steps += int(host_stats[3] > 0)
            history.append(host_params.clone())
            if args.verbose and rank == 0:
                print(f'it {epoch}: D_real {float(host_stats[0]):.3f} D_sim {float(host_stats[1]):.3f} '
                      f'D step {int(host_stats[2])} S step {int(host_stats[3])} params {host_params.tolist()}',
                      flush=True)
            epoch += 1
            if writer is not None and args.image_every > 0 and epoch % args.image_every == 0:
                r_img, s_img = real[:, :3].float().cpu(), sim_img[:, :3].float().cpu()
                pending.append(writer.submit(save_image, r_img, out_dir / f'real_{epoch:03d}.png', normalize=True))
                pending.append(writer.submit(save_image, s_img, out_dir / f'sim_samples_{epoch:03d}.png',
                                             normalize=True))
            tf = time.perf_counter()
            if steady:
                n_steady += 1
                ph['sim_wait'] += tb - ta
                ph['step_enqueue'] += tc - tb
                ph['fetch'] += td - tc
                ph['send'] += te - td
                ph['prefetch'] += tp - te
                ph['images'] += tf - tp
                if ev is not None:
                    ph['gpu_iteration'] += ev[0].elapsed_time(ev[1]) * 1e-3   # fetch() synchronised
            if epoch > args.num_epochs:
                break
        t_end = time.perf_counter()
        cpu1 = _cpu_snapshot(prod_pids) if cpu0 is not None else None
        dt = time.time() - t0
        for f in pending:
            f.result()
        if writer is not None:
            writer.shutdown()
        tgt = torch.tensor(np.concatenate((mu_target, std_target))).float()
        diff = (tgt - history[-1]).abs()
        if rank == 0:
            print('Abs.Diff to true params', diff, flush=True)
        res = {'iterations': epoch, 'seconds': dt, 'iterations_per_s': epoch / dt, 'sim_wait_s': wait_s,
               'images_per_s': epoch * B * world / dt, 'world': world, 'batch_per_rank': B,
               'final_params': history[-1].tolist(), 'target': tgt.tolist(), 'abs_diff': diff.tolist(),
               'd_steps': d_steps, 's_steps': s_steps, 'graph': step.graph is not None, 'fused_sstep': step.fused,
               'dtype': 'bf16' if bf16 else 'fp32', 'collectives': ('rccl-direct' if comm is not None and comm.native
                                                                   else ('gloo' if comm is not None else None))}
        if n_steady:
            st = t_end - t_steady
            res['steady'] = {
                'first_iteration': steady_from, 'iterations': n_steady, 'seconds': st,
                'iterations_per_s': n_steady / st, 'images_per_s': n_steady * B * world / st,
                # per-iteration means (ms): host time blocked on the next simulated batch, enqueueing
                # the (graph-replayed) iteration, the D->H fetch incl. waiting for the GPU, duplex
                # sends, image bookkeeping; gpu_iteration = device time of the iteration (events)
                'ms_per_iteration': {k: round(v * 1e3 / n_steady, 4) for k, v in ph.items()},
                'ms_per_iteration_total': round(st * 1e3 / n_steady, 4),
            }
            if ev is None:
                res['steady']['ms_per_iteration'].pop('gpu_iteration')
                res['steady']['ms_per_iteration'].pop('gpu_real_half')
            if cpu1 is not None:
                res['steady']['cpu'] = _cpu_report(cpu0, cpu1, n_steady, st)
        # the reference's record of convergence: parameter history with the
        # target appended as the last row (densityopt.py:326-331, 350-354)
        hist = torch.stack(history + [tgt]).numpy()
        res['history_rows'] = int(hist.shape[0])
        if out_dir is not None and rank == 0:
            hp = out_dir / f'run_{args.timestr}_{args.run_index:02d}_densityopt.txt'
            # the reference's call as it stands (densityopt.py:350-354): its note is
            # savetxt's comments= prefix, so the first line reads
            # 'last entry corresponds to target paramsmu_m1, ...' (np.loadtxt(skiprows=1))
            np.savetxt(hp, hist, header='mu_m1, mu_m2, std_m1, std_m2',
                       comments='last entry corresponds to target params')
            res['history_file'] = str(hp)
        if comm is not None:
            w = torch.cat([p.detach().reshape(-1).float() for p in list(netD.parameters()) + list(pm.parameters())])
            res['weights_checksum'] = float(w.double().sum())
            res['weights_sha'] = __import__('hashlib').sha1(w.cpu().numpy().tobytes()).hexdigest()[:16]
        return res


def _cpu_snapshot(pids=()):
    """(this process's threads {tid: (name, cpu seconds)}, the producer processes' cpu
    seconds, the host's busy and total jiffies from /proc/stat): where the CPU of the steady
    window goes -- this process's threads (main, loader IO / worker, HIP runtime), the
    producers, and the whole machine (which on a shared host includes other tenants)."""
    import os
    tick = os.sysconf('SC_CLK_TCK')
    prod = 0.0
    for pid in pids:
        try:
            with open(f'/proc/{pid}/stat') as f:
                parts = f.read().rsplit(')', 1)[1].split()
            prod += sum(int(x) for x in parts[11:15]) / tick   # utime stime cutime cstime
        except (OSError, ValueError, IndexError):
            pass
    th = {}
    try:
        for tid in os.listdir('/proc/self/task'):
            try:
                with open(f'/proc/self/task/{tid}/stat') as f:
                    parts = f.read().rsplit(')', 1)[1].split()
                with open(f'/proc/self/task/{tid}/comm') as f:
                    name = f.read().strip()
                th[int(tid)] = (name, (int(parts[11]) + int(parts[12])) / tick)
            except (OSError, ValueError, IndexError):
                pass
        with open('/proc/stat') as f:
            v = [int(x) for x in f.readline().split()[1:]]
        busy, total = sum(v) - v[3] - (v[4] if len(v) > 4 else 0), sum(v)
    except OSError:
        busy = total = 0
    return th, busy, total, prod


def _cpu_report(a, b, iters, seconds):
    """CPU-ms per iteration of this process (total and its 5 busiest threads) and the
    host's busy CPUs over the window."""
    import os
    th = {}
    for tid, (name, t1) in b[0].items():
        t0 = a[0].get(tid, (name, 0.0))[1]
        th[f'{name}:{tid}'] = t1 - t0
    top = sorted(th.items(), key=lambda kv: -kv[1])[:5]
    ncpu = os.cpu_count() or 1
    frac = (b[1] - a[1]) / max(1, b[2] - a[2])
    return {'process_ms_per_iteration': round(sum(th.values()) * 1e3 / iters, 4),
            'threads_ms_per_iteration': {k: round(v * 1e3 / iters, 4) for k, v in top},
            'producers_ms_per_iteration': round((b[3] - a[3]) * 1e3 / iters, 4),
            'host_busy_cpus': round(frac * ncpu, 2), 'host_cpus': ncpu}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--random-start', action='store_true')
    ap.add_argument('--num-epochs', default=70, type=int)
    ap.add_argument('--instances', default=SIM_INSTANCES, type=int, help='producer instances per rank')
    ap.add_argument('--batch', default=BATCH, type=int, help='images per rank per iteration')
    ap.add_argument('--producer', choices=['supershapesim', 'blender'], default='supershapesim')
    ap.add_argument('--device', default='cuda' if torch.cuda.is_available() else 'cpu')
    ap.add_argument('--backend', default=None, help='process-group backend (default: nccl on GPUs, gloo on CPU)')
    ap.add_argument('--start-port', default=26000, type=int)
    ap.add_argument('--seed', default=0, type=int)
    ap.add_argument('--json', default=None)
    ap.add_argument('--fp32', action='store_true', help='fp32 discriminator (PyTorch/MIOpen) instead of bf16 MFMA')
    ap.add_argument('--no-graph', action='store_true', help='eager iterations (no HIP graph)')
    ap.add_argument('--unfused-sstep', action='store_true',
                    help='the S step / gates in PyTorch ops (ProbModel + autograd) instead of the gfx950 kernels')
    ap.add_argument('--no-fused-bn', action='store_true',
                    help='discriminator with MIOpen BatchNorm + PyTorch LeakyReLU instead of the fused gfx950 op')
    ap.add_argument('--num-runs', default=1, type=int, help='independent runs (one history file each)')
    ap.add_argument('--out-dir', default='tmp',
                    help='where the parameter history and image grids go (reference: tmp/); "" writes nothing')
    ap.add_argument('--image-every', default=5, type=int,
                    help='write real_/sim_samples_ PNG grids every N epochs (reference: 5; 0 = never)')
    ap.add_argument('--steady-skip', default=5, type=int,
                    help='iterations excluded from the steady-state rate (at least warm-up + capture + 1)')
    ap.add_argument('--prefetch', action='store_true',
                    help='enqueue the D step\'s real-batch half while the producers render (DensityOptStep.'
                         'prefetch); default off: in a same-box A/B the inline iteration ran 179 / 166 it/s '
                         'against 166 / 150 (profiles/r5/b8/dopt_ab.jsonl)')
    ap.add_argument('--no-prefetch', action='store_true',
                    help='the real-batch half with the rest of the iteration, after the sim batch arrives '
                         '(the default; kept for scripts)')
    ap.add_argument('--verbose', action='store_true')
    args = ap.parse_args(argv)
    args.no_prefetch = args.no_prefetch or not args.prefetch
    args.timestr = time.strftime('%Y%m%d_%H%M%S')
    rank = int(os.environ.get('RANK', '0'))
    runs = []
    for i in range(args.num_runs):
        args.run_index = i
        if i > 0:
            args.seed += 1
            args.start_port += 7     # fresh producer ports (the previous ones may linger in TIME_WAIT)
        res = run(args)
        runs.append(res)
        if rank == 0:
            print(json.dumps(res), flush=True)
    res = runs[-1] if len(runs) == 1 else dict(runs[-1], runs=runs)
    if rank == 0:
        if args.json:
            Path(args.json).write_text(json.dumps(res, indent=2))
    elif args.json:
        Path(args.json).with_suffix(f'.rank{rank}.json').write_text(json.dumps(res, indent=2))
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    return res


if __name__ == '__main__':
    main()
