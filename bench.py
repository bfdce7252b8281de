#!/usr/bin/env python
"""Headline benchmark: Cube scene 640x480 RGBA, batch 8, streamed into HBM.

Mirrors the reference harness (benchmarks/benchmark.py:7-47: 4 producer
instances, batch 8, warm-up batch excluded, sec/image + sec/batch) on the
MI355X-native path:

  K headless Cube producers per GPU (csrc/sim/cubesim, C++ rasteriser; same
  launch contract and message dict as examples/datagen/cube.blend.py)
  render into a shared-memory frame ring --ZMTP PUSH/PULL descriptors-->
  native loader --> fused gfx950 decode kernel reading the pinned ring slots
  over PCIe itself (zero-copy; RGBA->RGB, gamma 2.2, /255, HWC->CHW, fp32)
  -> batch tensor resident on the GPU.  (--shm 0: frames inline in the
  messages, received into pinned slots; --h2d copy: DMA to HBM first.)

One process per GPU (``torch.distributed.run``); each rank owns its own
producers (shard mode, weak scaling), ranks are synchronised with RCCL
barriers around the timed region and the slowest rank's time is reported.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--producers P]
                    [--mode rgba|rgb] [--consumer none|disc] [--codec none|tile16]
                    [--h2d auto|copy] [--graph auto|on|off] [--dist shard|pool|scatter]

--consumer disc adds a DCGAN discriminator training step per batch (bf16,
fused gfx950 BN+LeakyReLU and pooling kernels, fused Adam, one HIP graph per
step on a single rank; profiles/consumer_step.md).

Rank 0 prints ONE JSON line (see README "Benchmark").
"""
import argparse
import fcntl
import json
import os
import signal
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / 'pytorch-blender_amd'
sys.path.insert(0, str(PKG))

# Best published reference row: 5 Blender instances, no UI refresh,
# 0.011 s/image -> 90.9 images/s (Readme.md:93).
BASELINE_IMAGES_PER_SEC = 90.9
METRIC = 'images/sec (whole node) + sec/batch, 640x480 RGBA Cube scene, batch=8'
# What vs_baseline compares: our producers are C++ stand-ins for Blender, so
# the ratio is NOT a framework speedup over blendtorch on equal producers.
PRODUCER = 'cubesim (C++ stand-in for Blender/Eevee, dirty-rect incremental CPU raster)'
BASELINE_NOTE = ('vs_baseline = value / 90.9 img/s, the reference\'s best row: 5 Blender/Eevee instances '
                 '(Readme.md:93). The producers differ (C++ stand-in vs Blender), so the ratio reflects the whole '
                 'pipeline incl. rendering, not the streaming framework alone.')


def ensure_built():
    """Incremental in-tree build, serialised across ranks with a file lock."""
    from blendtorch import _build
    lock = ROOT / 'build' / '.bench.lock'
    lock.parent.mkdir(parents=True, exist_ok=True)
    with open(lock, 'w') as fp:
        fcntl.flock(fp, fcntl.LOCK_EX)
        try:
            _build.build_all()
        finally:
            fcntl.flock(fp, fcntl.LOCK_UN)


def cpu_budget():
    """(affinity, budget, pin): CPUs this process may run on, how many of them
    it may keep busy (cgroup CPU quota), and whether pinning producers to
    single cores isolates anything.  With a quota far below the affinity mask
    (a shared host) the quota is the budget and per-core pinning would only
    pile producers onto cores other tenants also use."""
    cpus = sorted(os.sched_getaffinity(0))
    budget = len(cpus)
    try:
        quota, period = Path('/sys/fs/cgroup/cpu.max').read_text().split()[:2]
        if quota != 'max':
            budget = max(1, min(budget, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return cpus, budget, budget * 2 > len(cpus)


def thread_cpu():
    """{tid: (name, utime + stime ticks)} of this process's threads (Linux)."""
    out = {}
    for tid in os.listdir('/proc/self/task'):
        try:
            with open(f'/proc/self/task/{tid}/stat') as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index('(') + 1:st.rindex(')')]
        if int(tid) == os.getpid():
            name = 'main'       # the Python thread (native threads name themselves bt-*)
        rest = st[st.rindex(')') + 2:].split()
        out[int(tid)] = (name, int(rest[11]) + int(rest[12]))
    return out


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters (usage/throttling) -- producer-bound runs
    are CPU-quota sensitive, so report them next to the throughput."""
    try:
        kv = dict(line.split() for line in Path('/sys/fs/cgroup/cpu.stat').read_text().splitlines())
        return {k: int(v) for k, v in kv.items()}
    except (OSError, ValueError):
        return {}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=int(os.environ.get('WORLD_SIZE', '1')),
                    help='GPUs (= ranks).  Without a torchrun environment and N > 1 this process becomes a '
                         'supervisor that starts N ranks itself (blendtorch/parallel/launch.py)')
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--producers', type=int, default=0, help='producer processes per GPU (0 = auto)')
    ap.add_argument('--mode', choices=['rgba', 'rgb'], default='rgba')
    ap.add_argument('--resolution', default='640x480',
                    help='frame size WxH (the headline config is 640x480; smaller frames probe per-message costs)')
    ap.add_argument('--proto', choices=['tcp', 'ipc'], default='ipc',
                    help='ipc (Unix-domain ZMTP, same-host producers; default) or tcp')
    ap.add_argument('--consumer', choices=['none', 'disc'], default='none')
    ap.add_argument('--consumer-dtype', choices=['bf16', 'fp32'], default='bf16',
                    help='disc consumer: bf16 = decode kernel emits bf16 channels-last frames and the DCGAN step runs '
                         'under bf16 autocast (MFMA); fp32 = fp32 NCHW frames, fp32 step')
    ap.add_argument('--graph', choices=['auto', 'on', 'off'], default='auto',
                    help='disc consumer: capture the whole training step (forward, backward, Adam) in one HIP graph '
                         'and replay it per batch (auto: on for a single rank; DDP steps stay eager)')
    ap.add_argument('--io-threads', type=int, default=0)
    ap.add_argument('--shm', type=int, default=48,
                    help='>0 (default 48): producers render into an N-slot shared-memory ring (same host) and '
                         'send descriptors; 0: images inline in the ZMTP messages')
    ap.add_argument('--inline-producers', type=int, default=0,
                    help='with --shm: this many of each rank\'s producers send their images inline in the ZMTP '
                         'messages instead (a mixed fleet: inline frames land in pinned slots, batches stay direct)')
    ap.add_argument('--color-jitter', action='store_true',
                    help='photometric augmentation in the decode: a random colour transform per image '
                         '(brightness/contrast/saturation 0.4, hue 0.1) on the MFMA colour kernel, fp32 RGB out')
    ap.add_argument('--codec', choices=['none', 'tile16'], default='none',
                    help='shm frames: none = raw HWC; tile16 = key-frame deltas (the background crosses PCIe once, '
                         'then only the 16x16 tiles that differ from it; csrc/codec/tiledelta.h)')
    ap.add_argument('--h2d', choices=['auto', 'copy'], default=None,
                    help='auto: decode kernel reads pinned host frames directly (zero-copy); copy: DMA first. '
                         'Default: auto, but copy for the disc consumer -- its graphed training step runs faster '
                         'when the copy engines, not CUs waiting on PCIe reads, move the frames '
                         '(profiles/consumer_step.md)')
    ap.add_argument('--copy-streams', type=int, default=None,
                    help='copy path: HIP streams a batch\'s frame copies are spread over (several DMA engines); '
                         'default 2, or 1 for the disc consumer (it needs ~12 GB/s, and one DMA stream '
                         'disturbs its step least: 9.72k vs 9.59k img/s, profiles/r2/host_sync.txt)')
    ap.add_argument('--prefetch', type=int, default=None,
                    help='output buffers posted to the loader (batches assembled/decoding/ready ahead of the consumer); '
                         'default 8 (host-ordered hand-off, profiles/r4/cpu_per_frame.md), 6 for the disc consumer.  Deeper queues coalesce larger decode launches (8: +0.7 %%, 16: +1-2 %% on '
                         'long runs), but a short timed window then ends with more in-flight decode work inside '
                         'its closing device sync (20 steps, 8: 37.9k, 16: 34k vs 40.0k img/s); '
                         'profiles/r2/loader_depth_ab.txt')
    ap.add_argument('--launch-depth', type=int, default=2,
                    help='direct-path decode launches queued before new batches coalesce into one launch')
    ap.add_argument('--backend', choices=['nccl', 'gloo'], default='nccl',
                    help='process-group backend (nccl = RCCL over xGMI; gloo only to rehearse several ranks on one GPU)')
    ap.add_argument('--start-port', type=int, default=0)
    ap.add_argument('--sustain-s', type=float, default=2.0,
                    help='after the timed steps, time about this many more seconds of steps and report them as '
                         '"sustained" (a short timed window is served from the warm-up backlog); 0: off')
    ap.add_argument('--host-sync', choices=['auto', 'on', 'off'], default='auto',
                    help='loader/consumer ordering by host-side event checks (on) or cross-stream waits (off); '
                         'auto = on (a stream of cross-stream waits keeps a HIP runtime thread busy: 43 -> 20 '
                         'consumer CPU-us per frame, profiles/r4/cpu_per_frame.md)')
    ap.add_argument('--dma-phase', choices=['start', 'mid'], default='start',
                    help='disc consumer: when the next frames\' host->device DMA may start -- start = when the '
                         'step begins (overlapping the memory-bound forward); mid = between the forward and the '
                         'backward graph (DeviceLoader(defer_post=True) + CapturedStep(split=True))')
    ap.add_argument('--head', choices=['fused', 'torch'], default='fused',
                    help='disc consumer: fused = pool/conv/sigmoid/BCE head as gfx950 kernels (ops.disc_head_bce); '
                         'torch = the library layers + BCELoss')
    ap.add_argument('--optim', choices=['gfx950', 'torch'], default='gfx950',
                    help='disc consumer optimizer: gfx950 = ops.FusedAdam (two launches per step); '
                         'torch = torch.optim.Adam(fused=True, capturable=True)')
    ap.add_argument('--cast', choices=['fused', 'autocast'], default='fused',
                    help='disc consumer, bf16: fused = all conv weights cast in one gfx950 launch per direction '
                         '(Discriminator.forward_bf16); autocast = torch.autocast (a cast per layer each way)')
    ap.add_argument('--step-decode', choices=['on', 'off'], default='on',
                    help='disc consumer with --h2d copy: on = the loader only DMAs raw frames into the batch '
                         'tensor and the decode kernel runs inside the captured training step (one queue, no '
                         'loader kernels competing with the step); off = the loader decodes')
    ap.add_argument('--static-inputs', choices=['on', 'off'], default='on',
                    help='disc consumer: on = the loader cycles a fixed ring of output tensors and the captured '
                         'step has a graph per tensor that reads the batch in place; off = each batch is copied '
                         'into the graph\'s static input buffer')
    ap.add_argument('--fuse-decode', choices=['on', 'off'], default='on',
                    help='disc consumer with the in-step decode (bf16, fused cast and head): on = the first '
                         'convolution reads the raw u8 RGBA frames through the decode table inside its MFMA '
                         'kernels; off = a decode launch writes bf16 frames first')
    ap.add_argument('--graph-steps', type=int, choices=[1, 2], default=2,
                    help='disc consumer with static inputs: training steps per graph replay (2: consecutive '
                         'batches run in pairs from one captured graph -- halves the GPU idle between replays; '
                         '+0.4-1.3 %% in three same-call A/Bs, profiles/r4/b38/).  Not more than 2: the '
                         'loader re-posts a ring tensor two batches after handing it out, so a held step must '
                         'be enqueued by then')
    ap.add_argument('--grad-overlap', choices=['on', 'off'], default='on',
                    help='disc consumer, data parallel: on = two gradient buckets, each all-reduced as soon as its '
                         'gradients are written; off = one bucket after the whole backward')
    ap.add_argument('--consumer-input', choices=['stream', 'resident'], default='stream',
                    help='diagnostic: resident = the consumer trains on one fixed batch while the stream keeps running')
    ap.add_argument('--force-pg', action='store_true',
                    help='initialise a process group even for one rank (rehearses the collective code paths)')
    ap.add_argument('--pg-backend', choices=['auto', 'nccl', 'gloo'], default='auto',
                    help='process-group backend: auto = nccl only where a device collective runs (disc '
                         'consumer, scatter), else a gloo control plane (barriers, timing); nccl = always RCCL')
    ap.add_argument('--rccl-selfcheck', choices=['on', 'off'], default='on',
                    help='with a gloo control plane and --backend nccl: run the RCCL P2P-ring + all-reduce '
                         'self-check on a temporary nccl group at start-up, then destroy it')
    ap.add_argument('--dist', choices=['shard', 'pool', 'scatter'], default='shard',
                    help='shard: every rank owns its producers; pool: every rank launches producers and connects '
                         'to all of them (PUSH round-robin across GPUs); scatter: rank 0 receives world*B per step '
                         'and scatters B-image shards over RCCL')
    args = ap.parse_args(argv)
    if args.h2d is None:
        args.h2d = 'copy' if args.consumer == 'disc' else 'auto'
    if args.prefetch is None:
        args.prefetch = 6 if args.consumer == 'disc' else 8
    return args


def supervise(args, argv) -> int:
    """``--gpus N`` without torchrun: start N ranks of this script and relay.

    Runs BEFORE anything touches the GPU in this process (the device count
    comes from a child interpreter); the ranks inherit stdout, so rank 0's
    JSON line reaches the caller unchanged.  Never silently runs fewer ranks:
    with RCCL every rank needs its own GPU; ``--backend gloo`` may rehearse N
    ranks on fewer GPUs (ranks share devices round-robin)."""
    import importlib.util   # by path: the blendtorch.parallel package imports torch
    spec = importlib.util.spec_from_file_location('bt_launch', PKG / 'blendtorch' / 'parallel' / 'launch.py')
    launch = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(launch)
    ensure_built()          # once, before the ranks race for the build lock
    n = args.gpus
    have = launch.visible_gpu_count()
    if have < 1 or (args.backend == 'nccl' and have < n):
        print(f'[bench] --gpus {n} needs {n} visible GPUs for RCCL, found {have} '
              f'(use --backend gloo to rehearse several ranks on fewer GPUs)', file=sys.stderr, flush=True)
        return 3
    codes, rc = launch.spawn_ranks([sys.executable, '-u', str(Path(__file__).resolve())] + list(argv), n)
    if rc:
        print(f'[bench] rank exit codes {codes}', file=sys.stderr, flush=True)
    return rc


def _r(v, nd):
    return None if v is None else round(v, nd)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return supervise(args, argv)
    # a supervisor stops ranks with SIGTERM: unwind so the producer processes
    # this rank launched are torn down by BlenderLauncher.__exit__
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))

    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))

    ensure_built()
    # before the HIP runtime starts: streaming alone gets 8 hardware queues, so
    # the loader's copy / decode streams never share one with RCCL's; a training
    # consumer keeps HIP's 4 -- its captured step with the in-graph all-reduce
    # ran 27 % slower with 8 (profiles/r4/pg_tax.md; blendtorch.utils.ensure_hw_queues)
    from blendtorch.utils import ensure_hw_queues
    hw_queues = ensure_hw_queues(8 if args.consumer == 'none' else 4, exact=args.consumer != 'none')
    import torch
    import torch.distributed as dist
    from blendtorch import btt
    from blendtorch.btt.gpu import DeviceLoader
    from blendtorch.ops import DecodeConfig

    gpu = local_rank % max(1, torch.cuda.device_count())    # == local_rank on a full node
    torch.cuda.set_device(gpu)
    device = torch.device('cuda', gpu)
    world_seen, allreduce, comm = 1, None, None
    if world == 1 and args.force_pg:
        # a 1-rank process group: rehearses the collective path (e.g. RCCL
        # all-reduce captured in the step graph) on a single GPU
        from blendtorch.parallel.launch import free_port
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(free_port()))
        os.environ.setdefault('RANK', '0')
        os.environ['WORLD_SIZE'] = '1'
    # Which backend the process group needs.  Streaming in shard / pool mode
    # runs no device collective: the ranks only meet at the barriers around
    # the timed region and for the timing all-reduce, which a gloo control
    # plane carries.  A live RCCL communicator costs streaming 4-8 % on one
    # GPU even when it is never used (profiles/r3/pg_ab.md; why:
    # profiles/r4/pg_tax.md), so nccl is only built where a device
    # collective runs (the training step's gradient all-reduce, scatter).
    # With --backend nccl a shard/pool run still proves RCCL over xGMI at
    # start-up: a temporary nccl group runs the P2P-ring + all-reduce
    # self-check and is destroyed before streaming starts.
    device_coll = args.consumer == 'disc' or args.dist == 'scatter'
    if args.pg_backend == 'auto':
        pg_backend = args.backend if device_coll else 'gloo'
    else:
        pg_backend = args.pg_backend
    if pg_backend == 'nccl' and args.backend != 'nccl':
        pg_backend = 'gloo'
    pg_dev = device if pg_backend == 'nccl' else torch.device('cpu')
    if world > 1 or args.force_pg:
        if pg_backend == 'nccl':
            dist.init_process_group('nccl', device_id=device)
        else:
            dist.init_process_group('gloo')
        world_seen = dist.get_world_size()
        # collective sanity check: sum over ranks of (rank + 1) == w (w + 1) / 2
        chk = torch.tensor([float(rank + 1)], device=pg_dev)
        dist.all_reduce(chk)
        allreduce = {'value': float(chk.item()), 'expected': world_seen * (world_seen + 1) / 2,
                     'pg_backend': pg_backend}
        if allreduce['value'] != allreduce['expected']:
            raise RuntimeError(f'all_reduce sanity check failed: {allreduce}')
        # the communicator the training step and scatter mode use (RCCL called on
        # the compute stream), checked before anything depends on it: a P2P ring
        # over xGMI plus an all-reduce, each with a timeout that names this rank
        # and its peers (blendtorch/parallel/comm.py)
        if os.environ.get('BT_NO_DEVICECOMM') != '1':      # (diagnostic switch)
            from blendtorch.parallel import DeviceComm
            if pg_backend == 'nccl':
                # a communicator of its own for the training step's in-graph all-reduce
                # (16 % step tax on the group's shared one; profiles/r3/pg_ab.md)
                ded = os.environ.get('BT_DEVICECOMM_DEDICATED', '1' if args.consumer == 'disc' else '0') == '1'
                comm = DeviceComm(device=device, dedicated=ded)
                allreduce['selfcheck'] = {k: (round(v, 3) if isinstance(v, float) else v)
                                          for k, v in comm.selfcheck().items()}
            elif args.backend == 'nccl' and args.rccl_selfcheck == 'on':
                # streaming needs no device collective: prove RCCL anyway, then tear it down
                sub = dist.new_group(backend='nccl')
                tmp = DeviceComm(group=sub, device=device)
                res = tmp.selfcheck()
                tmp.close()
                torch.cuda.synchronize()
                dist.destroy_process_group(sub)
                res['torn_down'] = True
                allreduce['selfcheck'] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}

    # place each rank's producers on CPUs local to its GPU (same NUMA domain as
    # the GPU's PCIe root: frames are written there and read back by the GPU),
    # with disjoint port blocks and a /dev/shm share per rank
    # (blendtorch/parallel/topology.py::plan_rank_resources)
    from blendtorch.parallel import plan_rank_resources
    cpus, budget, pin = cpu_budget()
    res_w, res_h = (int(v) for v in args.resolution.lower().split('x'))
    try:
        st = os.statvfs('/dev/shm')
        shm_free = st.f_bavail * st.f_frsize
    except OSError:
        shm_free = None
    rp = plan_rank_resources(rank, local_rank, local_world, world, cpus, budget, pin, producers=args.producers,
                             dist_mode=args.dist, shm_slots=args.shm, shm_free_bytes=shm_free,
                             frame_bytes=res_w * res_h * (4 if args.mode == 'rgba' else 3))
    plan = {'cpus': rp['cpus'], 'domain': rp['domain'], 'numa_local': rp['numa_local']}
    share, nprod, affinity, shm_slots = rp['share'], rp['producers'], rp['affinity'], rp['shm_slots']
    if plan['numa_local']:
        os.sched_setaffinity(0, plan['domain'])           # loader threads next to the GPU too
    start_port = args.start_port or rp['start_port']

    decode = DecodeConfig.unit(channels='rgb', gamma=2.2)
    if args.color_jitter:
        if args.consumer != 'none' or args.mode != 'rgba':
            raise SystemExit('--color-jitter: RGBA frames, no consumer (fp32 RGB output)')
        from blendtorch.ops import ColorJitter
        decode = DecodeConfig.unit(channels='rgb', gamma=2.2,
                                   color_jitter=ColorJitter(0.4, 0.4, 0.4, 0.1, seed=rank))
    amp = args.consumer == 'disc' and args.consumer_dtype == 'bf16'
    # decode inside the consumer's captured step (frames arrive by DMA only)
    step_decode = (args.consumer == 'disc' and args.h2d == 'copy' and args.dist != 'scatter'
                   and args.step_decode == 'on')
    # RGBA frames decoded to 4-channel bf16: the first conv's MFMA kernel reads
    # 8-byte pixels and ignores alpha (weight 0) -- cheaper than a 3-channel layout
    rgba_in = amp and args.cast == 'fused' and args.mode == 'rgba'
    if amp:
        # the decode kernel writes what the model's first conv reads: bf16, channels-last
        decode = DecodeConfig.unit(channels='rgba' if rgba_in else 'rgb', gamma=2.2, dtype='bfloat16', layout='nhwc')
    # graphs per loader output tensor (disc consumer, one graph per step): the
    # step reads each batch where the loader put it
    static_in = (args.prefetch + 2) if (args.consumer == 'disc' and args.static_inputs == 'on'
                                        and args.dma_phase != 'mid' and args.dist != 'scatter') else 0
    # the in-step decode folded into the first convolution's MFMA kernels (raw u8 frames in)
    fuse_decode = (step_decode and args.fuse_decode == 'on' and amp and args.cast == 'fused'
                   and args.head == 'fused' and decode.channels == 'rgba' and decode.dtype == 'bfloat16')
    launch = dict(producer='cubesim', num_instances=nprod, named_sockets=['DATA'], start_port=start_port,
                  proto=args.proto, seed=1000 * rank, cpu_affinity=affinity,
                  instance_args=[['--mode', args.mode, '--sndhwm', '10', '--resolution', f'{res_w}x{res_h}']
                                 + (['--shm', str(shm_slots), '--codec', args.codec]
                                    if shm_slots and i >= args.inline_producers else [])
                                 for i in range(nprod)])
    model = opt = None
    copy_streams = args.copy_streams or (1 if args.consumer == 'disc' else 2)
    # the next frames' DMA starts between the step's forward and backward graphs
    dma_mid = args.consumer == 'disc' and args.dma_phase == 'mid' and args.dist != 'scatter'
    if args.consumer == 'disc':
        if os.environ.get('BT_CUDNN_BENCHMARK', '1') == '1':
            torch.backends.cudnn.benchmark = True   # MIOpen find: best conv kernels for these fixed shapes
        from blendtorch.models import Discriminator
        model = Discriminator(nc=3, ndf=32, adaptive=True).to(device).to(memory_format=torch.channels_last)
        if dist.is_initialized():
            # data parallel: identical initial weights on every rank; gradients are
            # averaged inside the (captured) step, see CapturedStep
            for p_ in model.state_dict().values():
                dist.broadcast(p_, 0)
        use_graph = args.graph == 'on' or (args.graph == 'auto' and (world == 1 or args.backend == 'nccl'))
        # fused Adam: one multi-tensor kernel for the whole update (0.95 -> 0.84 ms graphed step,
        # profiles/consumer_step.md); capturable keeps its step counters on the GPU for the graph
        if args.optim == 'gfx950':
            # ops.FusedAdam: ONE update kernel over all parameters (device step
            # counter: capturable), which also rewrites the bf16 conv weights and
            # their data-gradient transposes the next forward reads (no per-step
            # cast / transpose launches) and clears the gradients it consumed
            from blendtorch import ops
            opt = ops.FusedAdam(model.parameters(), lr=2e-4)
            if args.cast == 'fused':
                model.use_optimizer_shadows(opt)
        else:
            opt = torch.optim.Adam(model.parameters(), lr=2e-4, capturable=use_graph, fused=True)
        crit = torch.nn.BCELoss()

    WARM_RESERVE = 2000   # extra warm-up batches allowed while producers come up
    SUSTAIN_RESERVE = 12000 if args.sustain_s > 0 else 0   # batches the sustained window may draw (bound only)
    total_batches = args.warmup + args.steps + (WARM_RESERVE + SUSTAIN_RESERVE if args.dist != 'scatter' else 0)
    last = {'btid': None}
    from contextlib import ExitStack
    from blendtorch.parallel import ScatterLoader
    with ExitStack() as es:
        dl = None
        if nprod > 0:
            bl = es.enter_context(btt.BlenderLauncher(**launch))
            per_step = args.batch * (world if args.dist == 'scatter' else 1)
            addrs = bl.launch_info.addresses['DATA']
            if args.dist in ('pool', 'scatter'):
                from blendtorch.parallel import pool_addresses
                addrs = pool_addresses(addrs)
            if args.dist != 'scatter' or rank == 0:
                # scatter: the root's loader lands raw u8 RGBA frames -- the bytes
                # that cross xGMI (4-pixel lanes read host memory at the PCIe rate;
                # dropping alpha would save 25 % of the xGMI bytes but forces
                # 16-pixel lanes that read host memory ~30 % slower)
                ldec = decode if args.dist != 'scatter' else DecodeConfig.raw(channels='rgba')
                if step_decode:
                    # the loader only DMAs the frames into the consumer's tensor
                    # (identity decode = no kernel on the loader's queue); the
                    # decode runs inside the captured training step
                    ldec = DecodeConfig.raw(channels=args.mode)
                dl = DeviceLoader(addrs, batch_size=per_step, decode=ldec, device=device,
                                  max_items=total_batches * per_step, prefetch=args.prefetch,
                                  io_threads=args.io_threads or None, timeoutms=60000, h2d=args.h2d,
                                  launch_depth=args.launch_depth,
                                  copy_streams=copy_streams,
                                  defer_post=dma_mid,
                                  host_sync=None if args.host_sync == 'auto' else args.host_sync == 'on',
                                  # a fixed ring of output tensors: the captured step keeps a
                                  # graph per tensor and reads the batch in place (no copy)
                                  reuse_buffers=static_in > 0)
        if args.dist == 'scatter':
            it = iter(ScatterLoader(dl, args.batch, decode, device, total_batches))
        else:
            it = iter(dl)

        def as_input(img):
            if step_decode:
                return img                  # raw u8 NHWC frames: decoded in loss_fn
            # NHWC bf16 storage -> NCHW view with channels-last strides; fp32 NCHW -> channels-last copy
            return img.permute(0, 3, 1, 2) if amp else img.contiguous(memory_format=torch.channels_last)

        def loss_fn(m, x):
            if fuse_decode:
                # the raw u8 RGBA frames go straight into the first convolution,
                # which decodes them in its MFMA kernels' tile loads (no decode
                # launch, no bf16 copy of the batch)
                return m.bce_loss_bf16(x.permute(0, 3, 1, 2), 1.0, decode=decode)
            if step_decode:
                from blendtorch import ops
                x = ops.decode(x, decode)   # gfx950 decode, captured with the step
                x = x.permute(0, 3, 1, 2) if amp else x.contiguous(memory_format=torch.channels_last)
            if amp and args.cast == 'fused' and args.head == 'fused':
                # pool -> conv -> sigmoid -> BCE in 2 + 2 gfx950 launches (ops.disc_head_bce)
                return m.bce_loss_bf16(x.to(torch.bfloat16), 1.0)
            if amp and args.cast == 'fused':
                out = m.forward_bf16(x.to(torch.bfloat16)).float()   # one cast launch per direction
            elif amp:
                # no autocast weight cache: a captured graph must recast the live weights on every replay
                with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=not use_graph):
                    out = m(x)
                out = out.float()
            else:
                out = m(x)
            return crit(out, torch.ones_like(out))

        # whole-step HIP graph (forward, backward, gradient all-reduce over RCCL
        # when world > 1, fused Adam): the batch is copied into a static input
        # buffer and ~100 kernels replay as one launch, which takes the Python /
        # autograd / MIOpen dispatch cost off the critical path
        # (blendtorch/parallel/step.py; DDP's host-side reducer cannot be captured)
        stepper = None
        if model is not None:
            from blendtorch.parallel.step import CapturedStep
            # data parallel: two gradient buckets, the last layers' all-reduced as soon as
            # written, ahead of the first layers' weight gradients (GradBuckets.arm)
            stepper = CapturedStep(model, opt, loss_fn, graph=use_graph, comm=comm,
                                   allreduce='always' if args.force_pg else dist.is_initialized(), split=dma_mid,
                                   static_inputs=static_in, overlap=args.grad_overlap == 'on',
                                   group_steps=args.graph_steps)

        def graphed(x):
            stepper(x, mid=dl.release if (dma_mid and dl is not None) else None)
            if stepper.error:
                print(f'[bench] HIP graph capture failed, eager steps: {stepper.error}', file=sys.stderr, flush=True)
                stepper.error = None

        fixed = {}

        from blendtorch.utils import trace_range

        def step():
            with trace_range('bench.next'):
                b = next(it)
            img = b['image']
            last['btid'] = b.get('btid')
            if model is not None:
                if args.consumer_input == 'resident':
                    # diagnostic: keep streaming, but train on one fixed batch (no
                    # dependency on the loader's events) -- separates contention
                    # from waiting in the streamed-vs-resident step-time gap
                    if 'x' not in fixed:
                        x0 = as_input(img)
                        fixed['x'] = x0.clone() if step_decode else x0.clone(memory_format=torch.channels_last)
                    graphed(fixed['x'])
                else:
                    with trace_range('bench.train'):
                        graphed(as_input(img))
            return img

        # warm-up: at least W batches, and (shard/pool) until every local producer
        # has delivered a frame, so the timed region starts in steady state on every rank
        seen = set()
        n_warm, t_warm = 0, time.time()
        while n_warm < args.warmup or (args.dist != 'scatter' and len(seen) < nprod and n_warm < WARM_RESERVE
                                       and time.time() - t_warm < 20):
            step()
            n_warm += 1
            if last['btid'] is not None:
                seen.update(int(x) for x in last['btid'])
        if stepper is not None:
            stepper.flush()          # --graph-steps 2: no warm-up step carried into the timed region
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        cg0 = cgroup_cpu_stat()
        th0 = thread_cpu() if os.environ.get('BT_THREAD_REPORT') == '1' else None
        ru0 = os.times()
        snap0 = dl.snapshot() if dl is not None else {}
        t0 = time.perf_counter()
        for _ in range(args.steps):
            img = step()
        if stepper is not None:
            stepper.flush()          # --graph-steps 2: the last step of an odd count runs on its own
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        snap1 = dl.snapshot() if dl is not None else {}
        ru1 = os.times()
        cg1 = cgroup_cpu_stat()
        # Sustained rate, reported next to (never instead of) the timed K steps:
        # a short driver window (e.g. 20 steps) is served from the frames the
        # producers queued during warm-up (backlog_covers_window), so the same
        # run also times ~--sustain-s more seconds of steps that the backlog
        # cannot cover, with its own loader window.  Every rank runs the same
        # number of steps (the data-parallel step all-reduces per step).
        sustained = None
        if args.sustain_s > 0 and args.dist != 'scatter':
            te = torch.tensor([elapsed], dtype=torch.float64, device=pg_dev)
            if world > 1:
                dist.all_reduce(te, op=dist.ReduceOp.MAX)
            per = float(te.item()) / max(1, args.steps)
            left = total_batches - n_warm - args.steps - 2
            n_sus = int(min(left, max(0, args.sustain_s / max(per, 1e-6))))
            if n_sus * args.batch * (1 + world) > 16 * args.batch and n_sus >= 4 * args.steps:
                sa = dl.snapshot() if dl is not None else {}
                ts = time.perf_counter()
                for _ in range(n_sus):
                    step()
                if stepper is not None:
                    stepper.flush()
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                tsx = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=pg_dev)
                if world > 1:
                    dist.all_reduce(tsx, op=dist.ReduceOp.MAX)
                sb = dl.snapshot() if dl is not None else {}
                ws = DeviceLoader.window(sa, sb) if dl is not None else {}
                sustained = {'steps': n_sus, 'seconds': round(float(tsx.item()), 4),
                             'images_per_s': round(n_sus * args.batch * world / float(tsx.item()), 2),
                             'ms_per_step': round(float(tsx.item()) / n_sus * 1e3, 4),
                             'backlog_covers_window': ws.get('backlog_covers_window') if ws else None,
                             'producer_share_max_over_min': ws.get('producer_share_max_over_min') if ws else None}
        cpu = {'consumer_cpu_s': round((ru1.user - ru0.user) + (ru1.system - ru0.system), 3)}
        for k in ('usage_usec', 'throttled_usec', 'nr_throttled'):
            if k in cg0 and k in cg1:
                cpu['cgroup_' + k] = cg1[k] - cg0[k]
        # CPU per delivered frame (what plan_rank_resources budgets with): the
        # cgroup holds every local rank's consumer and producers; the consumer
        # process (loader IO threads + the Python main thread) is this rank's
        frames_here = args.steps * args.batch
        per = {'consumer': round(cpu['consumer_cpu_s'] * 1e6 / max(1, frames_here), 2)}
        if 'cgroup_usage_usec' in cpu:
            node_frames = frames_here * (local_world if args.dist != 'scatter' else 1)
            per['total'] = round(cpu['cgroup_usage_usec'] / max(1, node_frames), 2)
            per['producers'] = round(per['total'] - per['consumer'], 2)
        cpu['us_per_frame'] = per
        if snap1.get('cpu_recv_ms'):
            # BT_LOADER_CPU=1: the loader worker's thread CPU per loop stage, per frame
            cpu['loader_us_per_frame'] = {k[4:-3]: round((snap1[k] - snap0.get(k, 0)) * 1e3 / max(1, frames_here), 2)
                                          for k in ('cpu_poll_ms', 'cpu_recv_ms', 'cpu_launch_ms', 'cpu_reap_ms')}
        if th0 is not None:
            # (diagnostic) this process's busiest threads over the timed region
            th1 = thread_cpu()
            wt = snap1.get('worker_tid')
            name = {t: ('bt-loader(worker)' if t == wt else th1[t][0]) for t in th1}
            busy = sorted(((th1[t][1] - th0.get(t, ('', 0))[1], name[t]) for t in th1), reverse=True)
            cpu['threads_cpu_s'] = [[name, round(d / os.sysconf('SC_CLK_TCK'), 3)] for d, name in busy[:12] if d > 0]
        shape = tuple(img.shape)
        if args.dist == 'scatter':
            try:            # run the source to its end so its stats are final
                next(it)
            except StopIteration:
                pass
        else:
            it.close()      # stops the native loader and publishes its stats
        stats = dict(dl.stats) if dl is not None else {}
        metrics = dl.metrics() if dl is not None else {}
        if world > 1 and args.dist in ('pool', 'scatter'):
            dist.barrier()   # other ranks may still be drawing on this rank's producers

    win = DeviceLoader.window(snap0, snap1)
    t = torch.tensor([elapsed], dtype=torch.float64, device=pg_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tmax = float(t.item())
    images = args.steps * args.batch * world
    value = images / tmax
    mine_info = {
        'rank': rank, 'gpu': gpu, 'pid': os.getpid(),
        'elapsed_s': round(elapsed, 6),
        'images_per_s': round(args.steps * args.batch / elapsed, 1),
        'producers': nprod,
        'cpus': share,
        'numa_local': plan['numa_local'],
        'cpu_domain': [min(plan['domain']), max(plan['domain'])] if plan['domain'] else None,
        'loader_frames_per_s': round(win['frames_per_s'], 1) if win else None,
        'h2d_gbytes_per_s': round(win['h2d_gbytes_per_s'], 2) if win else None,
    }
    per_rank = [mine_info]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine_info)
    if rank == 0:
        print(json.dumps({
            'metric': METRIC,
            'value': round(value, 2),
            'unit': 'images/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(tmax / args.steps * 1000, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': round(value / BASELINE_IMAGES_PER_SEC, 3),
            'producer': PRODUCER,
            'baseline_note': BASELINE_NOTE,
            'world_size_seen': world_seen,
            'backend': (args.backend if world > 1 else None),
            'pg_backend': (pg_backend if dist.is_initialized() else None),
            'hw_queues': hw_queues,
            'allreduce_check': allreduce,
            'rank_time_s': {'min': round(min(r['elapsed_s'] for r in per_rank), 6),
                            'max': round(max(r['elapsed_s'] for r in per_rank), 6)},
            'per_rank': per_rank,
            'dtype': 'bf16' if amp else 'fp32',
            'data': 'synthetic (headless C++ Cube-scene producers, random rotations)',
            'config': {
                'model': f'cube-scene-{res_w}x{res_h}-' + args.mode + (' + dcgan-disc' if model is not None else ''),
                'global_batch': args.batch * world,
                'seq_len': None,
                'parallelism': f'dp{world}' + ('' if args.dist == 'shard' else '-' + args.dist),
                'producers_per_gpu': nprod,
                'cpus_per_gpu': share,
                'numa_local': plan['numa_local'],
                'decode': ('rgba->rgb, gamma 2.2, /255, bf16 NHWC (gfx950 kernel)' if amp else
                           'rgba->rgb, gamma 2.2, /255, per-image colour jitter (MFMA), HWC->CHW fp32 (gfx950 kernel)'
                           if args.color_jitter else 'rgba->rgb, gamma 2.2, /255, HWC->CHW fp32 (gfx950 kernel)'),
                'out_shape': list(shape),
                'proto': args.proto,
                'pinned_producers': pin,
                'shm_slots': shm_slots,
                'h2d': args.h2d,
                'launch_depth': args.launch_depth, 'prefetch': args.prefetch,
                'copy_streams': copy_streams if args.h2d == 'copy' else None,
                'codec': args.codec if shm_slots else 'none',
                'inline_producers': min(nprod, args.inline_producers) if shm_slots else nprod,
                'consumer_step': stepper.state if stepper is not None else None,
                'decode_in_step': step_decode,
                'decode_fused_in_conv': fuse_decode,
                'static_input_graphs': static_in,
                'cast': args.cast if amp else None,
                'optim': args.optim if model is not None else None,
                'dma_phase': args.dma_phase if model is not None else None,
                'graph_steps': args.graph_steps if model is not None else None,
                'head': args.head if model is not None else None,
                'host_sync': args.host_sync,
                'consumer_collectives_per_step': stepper.collectives if stepper is not None else None,
                'grad_buckets_issue_order': (stepper.grads.order if stepper is not None and stepper.overlap
                                             and stepper.grads is not None else None),
                'collectives': ('rccl-direct' if comm is not None and comm.native else
                                ('c10d' if comm is not None else None)),
            },
            'sec_per_image': round(tmax / images, 7),
            'sec_per_batch': round(tmax / args.steps, 6),
            'loader_stats': {k: stats.get(k) for k in ('frames', 'batches', 'bad', 'pool_fallbacks', 'direct_batches',
                                                       'launches', 'shm_frames', 'shm_torn', 'tiled_frames',
                                                       'staged_frames')},
            # rank 0's loader over the TIMED WINDOW only (snapshots at t0 / t1):
            # device time per image (H2D + decode, sampled launches after the cold
            # start), image bytes host -> device per second (tile16 moves only the
            # changed tiles), per-producer rates and ring occupancy at both ends
            'gpu_us_per_image': _r(win.get('gpu_us_per_image'), 3),
            'h2d_gbytes_per_s': _r(win.get('h2d_gbytes_per_s'), 2),
            'loader_frames_per_s': _r(win.get('frames_per_s'), 1),
            'producer_frames_per_s': win.get('producer_frames_per_s'),
            'producer_share_max_over_min': win.get('producer_share_max_over_min'),
            'producers_starved': win.get('producers_starved'),
            'window_frames': win.get('frames'),
            'backlog_covers_window': win.get('backlog_covers_window'),
            'ring_t0': win.get('ring_t0'),
            'ring_t1': win.get('ring_t1'),
            'consumer_wait_ms_per_batch': _r(win.get('consumer_wait_ms_per_batch'), 4),
            # ~--sustain-s more steps right after the timed ones (not part of value)
            'sustained': sustained,
            # whole run incl. start-up (for comparison with the window)
            'run_frames_per_producer': metrics.get('frames_per_producer'),
            'cpu': cpu,
        }), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    sys.exit(main() or 0)
