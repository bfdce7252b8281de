"""RCCL/xGMI distribution helpers, exercised with gloo on CPU (world_size 2)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from blendtorch import parallel


def test_shard_addresses_disjoint_cover():
    addrs = [f'tcp://h:{p}' for p in range(10)]
    shards = [parallel.shard_addresses(addrs, r, 4) for r in range(4)]
    flat = sorted(a for s in shards for a in s)
    assert flat == sorted(addrs)
    assert all(len(s) in (2, 3) for s in shards)
    assert parallel.shard_addresses(addrs[:2], 3, 4) == [addrs[1]]


def test_partition_cpus():
    cpus = list(range(16))
    parts = [parallel.partition_cpus(cpus, r, 4) for r in range(4)]
    assert parts[0] == [0, 1, 2, 3] and parts[3] == [12, 13, 14, 15]


def test_parse_cpulist():
    assert parallel.parse_cpulist('0-3,8,10-11\n') == [0, 1, 2, 3, 8, 10, 11]
    assert parallel.parse_cpulist('') == []


def _fake_sysfs(root, layout):
    for bdf, cpulist in layout.items():
        (root / bdf).mkdir(parents=True)
        (root / bdf / 'local_cpulist').write_text(cpulist + '\n')
    return root


def test_plan_rank_cpus_numa_local(tmp_path):
    # 8 GPUs, 4 per socket; socket 0 = CPUs 0-31, socket 1 = CPUs 32-63
    bus = [f'0000:{0x10 * (i + 1):02x}:00.0' for i in range(8)]
    sysfs = _fake_sysfs(tmp_path, {b: ('0-31' if i < 4 else '32-63') for i, b in enumerate(bus)})
    allowed = list(range(64))
    plans = [parallel.plan_rank_cpus(r, 8, allowed, bus_ids=bus, sysfs=sysfs) for r in range(8)]
    assert all(p['numa_local'] for p in plans)
    assert plans[0]['cpus'] == list(range(0, 8)) and plans[3]['cpus'] == list(range(24, 32))
    assert plans[4]['cpus'] == list(range(32, 40)) and plans[7]['domain'] == list(range(32, 64))
    flat = sorted(c for p in plans for c in p['cpus'])
    assert flat == allowed                          # disjoint, covering
    # GPU order need not follow socket order: rank 0 on socket 1
    sysfs2 = _fake_sysfs(tmp_path / 'b', {b: ('32-63' if i % 2 == 0 else '0-31') for i, b in enumerate(bus)})
    p0 = parallel.plan_rank_cpus(0, 8, allowed, bus_ids=bus, sysfs=sysfs2)
    assert p0['numa_local'] and set(p0['cpus']) <= set(range(32, 64))


def test_plan_rank_cpus_fallback(tmp_path):
    allowed = list(range(16))
    p = parallel.plan_rank_cpus(1, 4, allowed, bus_ids=[None] * 4, sysfs=tmp_path)
    assert not p['numa_local'] and p['cpus'] == [4, 5, 6, 7]
    # local set disjoint from the allowed CPUs -> fallback
    sysfs = _fake_sysfs(tmp_path / 'x', {'0000:01:00.0': '100-107'})
    p = parallel.plan_rank_cpus(0, 1, allowed, bus_ids=['0000:01:00.0'], sysfs=sysfs)
    assert not p['numa_local'] and p['cpus'] == allowed


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, dev = parallel.init_distributed(backend='gloo')
        B = 3
        full = torch.arange(world * B * 2, dtype=torch.float32).view(world * B, 2) if r == 0 else None
        shard = parallel.scatter_batch(full, (B, 2), torch.float32, torch.device('cpu'))
        ok_scatter = torch.equal(shard, torch.arange(r * B * 2, (r + 1) * B * 2, dtype=torch.float32).view(B, 2))
        t = torch.full((4,), float(r))
        parallel.broadcast_tensor(t, src=1)
        ok_bcast = torch.equal(t, torch.full((4,), 1.0))
        stats = parallel.all_gather_stats({'fps': 10.0 * (r + 1), 'n': r})
        ok_stats = [s['fps'] for s in stats] == [10.0 * (i + 1) for i in range(world)]

        # scatter mode: u8 frames + packed metadata in one P2P round, decoded per rank
        from blendtorch import ops
        cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
        H, W = 6, 8

        def frames(step):
            g = torch.Generator().manual_seed(step)
            return torch.randint(0, 256, (world * B, H, W, 4), dtype=torch.uint8, generator=g)

        def source():
            for step in range(3):
                yield {'image': frames(step), 'btid': torch.arange(world * B) + 100 * step,
                       'xy': torch.arange(world * B * 16, dtype=torch.float64).view(world * B, 8, 2) + step,
                       'name': [f's{step}i{i}' for i in range(world * B)]}
        sl = parallel.ScatterLoader(source() if r == 0 else None, B, cfg, torch.device('cpu'), 3)
        ok_loader = True
        for step, b in enumerate(sl):
            full = frames(step)[r * B:(r + 1) * B]
            ok_loader &= torch.equal(b['image'], ops.reference_decode(full, cfg))   # bit-exact
            ok_loader &= b['btid'].tolist() == [100 * step + i for i in range(r * B, (r + 1) * B)]
            xy = torch.arange(world * B * 16, dtype=torch.float64).view(world * B, 8, 2)[r * B:(r + 1) * B] + step
            ok_loader &= b['xy'].dtype == torch.float64 and torch.equal(b['xy'], xy)
            ok_loader &= b['name'] == [f's{step}i{i}' for i in range(r * B, (r + 1) * B)]
        ok_loader &= sl.stats['steps'] == 3 and sl.stats['object_scatters'] == 3
        q.put((r, ok_scatter, ok_bcast, ok_stats, ok_loader))
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface failures to the parent
        q.put((rank, repr(e)))


def _pool_worker(rank, world, port, prod_port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from blendtorch import btt
        parallel.init_distributed(backend='gloo')
        with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'],
                                 start_port=prod_port + 10 * rank, seed=rank,
                                 instance_args=[['--mode', 'rgb', '--resolution', '64x48',
                                                 '--frame-range', str(1000 * rank), str(1000 * rank + 100)]]) as bl:
            addrs = parallel.pool_addresses(bl.launch_info.addresses['DATA'])
            # producers start at different times on a loaded host: read until both
            # have delivered (at least 40 items, at most the 2 x 100 they render)
            ds = btt.RemoteIterableDataset(addrs, max_items=200, timeoutms=30000)
            torch.distributed.barrier()   # both ranks' producers launched
            sources = []
            for item in ds:
                sources.append(int(item['frameid']) // 1000)   # which rank's producer
                if len(sources) >= 40 and len(set(sources)) == 2:
                    break
            torch.distributed.barrier()   # keep producers alive until both ranks are done
        q.put((rank, len(addrs), sorted(set(sources)), len(sources)))
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface failures to the parent
        q.put((rank, repr(e)))


def test_pool_mode_gloo_world2():
    """Pool mode: each rank launches one producer (frame ids 0.. on rank 0,
    1000.. on rank 1) and connects to both; every rank receives frames from
    both producers (PUSH round-robin across ranks)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    base = 36000 + (os.getpid() % 500) * 20
    procs = [ctx.Process(target=_pool_worker, args=(r, 2, port, base, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 4, r
        assert r[1] == 2 and r[3] >= 40 and r[2] == [0, 1], r


def test_pack_meta_roundtrip():
    b = {'btid': torch.arange(4), 'xy': torch.rand(4, 8, 2, dtype=torch.float64),
         'f': torch.rand(4).half(), 'flag': torch.tensor([True, False, True, True])}
    tensors, objects = parallel.__dict__['_meta_schema'](dict(b, image=None), 4, 'image')
    assert objects == [] and [k for k, _, _ in tensors] == ['btid', 'xy', 'f', 'flag']
    packed = parallel.pack_meta(b, tensors, 4)
    assert packed.dtype == torch.uint8 and packed.shape == (4, 8 + 128 + 2 + 1)
    out = parallel.unpack_meta(packed[2:4], tensors)
    for k, v in b.items():
        assert out[k].dtype == v.dtype and torch.equal(out[k], v[2:4]), k


def test_collectives_gloo_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1:] == (True, True, True, True), r


def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from blendtorch.parallel.step import CapturedStep, allreduce_gradients
        parallel.init_distributed(backend='gloo')
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.ReLU(), torch.nn.Linear(3, 1))
        for p in m.parameters():
            p.grad = torch.full_like(p, float(rank + 1))
        n = allreduce_gradients(m.parameters(), bucket_mb=1e-5)      # tiny buckets: one per tensor
        ok_avg = n == 4 and all(torch.equal(p.grad, torch.full_like(p, 1.5)) for p in m.parameters())
        # data-parallel step without DDP: ranks see different data, weights stay identical
        opt = torch.optim.SGD(m.parameters(), lr=0.1)
        step = CapturedStep(m, opt, lambda mod, x: mod(x).pow(2).mean(), graph=False)
        for i in range(3):
            step(torch.randn(8, 4, generator=torch.Generator().manual_seed(10 * rank + i)))
        w = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        allw = [torch.empty_like(w) for _ in range(world)]
        torch.distributed.all_gather(allw, w)
        ok_sync = all(torch.equal(allw[0], x) for x in allw) and step.collectives == 1
        q.put((rank, ok_avg, ok_sync))
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface failures to the parent
        q.put((rank, repr(e)))


def test_manual_grad_allreduce_gloo_world2():
    """allreduce_gradients / CapturedStep (eager here): averaged gradients and
    weights that stay bit-identical across ranks without DDP."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1:] == (True, True), r


def test_captured_step_split_mid_hook_eager():
    """split/mid: the hook runs between forward and backward, and the update
    equals the unsplit step (eager on the CPU; GPU graph replay in
    tests/test_gpu_consumer.py)."""
    from blendtorch.parallel.step import CapturedStep
    order = []
    torch.manual_seed(0)
    a = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.ReLU(), torch.nn.Linear(3, 1))
    b = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.ReLU(), torch.nn.Linear(3, 1))
    b.load_state_dict(a.state_dict())

    def loss_fn(mod, x):
        order.append('fwd')
        return mod(x).pow(2).mean()

    sa = CapturedStep(a, torch.optim.SGD(a.parameters(), lr=0.1), loss_fn, allreduce=False, graph=False, split=True)
    sb = CapturedStep(b, torch.optim.SGD(b.parameters(), lr=0.1), loss_fn, allreduce=False, graph=False)
    x = torch.randn(8, 4, generator=torch.Generator().manual_seed(1))
    sa(x, mid=lambda: order.append('mid'))
    assert order == ['fwd', 'mid']
    sb(x)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)


def test_pack_meta_rejects_schema_drift():
    """A metadata tensor whose dtype or per-item shape changes after the
    schema was agreed raises instead of sending rows of another width."""
    b = {'btid': torch.arange(4), 'xy': torch.rand(4, 8, 2, dtype=torch.float64)}
    schema, _ = parallel.__dict__['_meta_schema'](b, 4, 'image')
    out = torch.empty((4, 8 + 128), dtype=torch.uint8)
    assert parallel.pack_meta(b, schema, 4, out=out) is out
    assert torch.equal(out, parallel.pack_meta(b, schema, 4))
    with pytest.raises(ValueError, match="'xy' changed"):
        parallel.pack_meta({'btid': torch.arange(4), 'xy': torch.rand(4, 9, 2, dtype=torch.float64)}, schema, 4)
    with pytest.raises(ValueError, match="'btid' changed"):
        parallel.pack_meta({'btid': torch.arange(4, dtype=torch.int32), 'xy': b['xy']}, schema, 4)


def test_device_comm_refuses_a_destroyed_process_group(monkeypatch):
    """A DeviceComm whose process group was destroyed raises instead of
    calling RCCL through the dangling borrowed communicator; a nonblocking
    communicator (TORCH_NCCL_USE_COMM_NONBLOCKING) is never borrowed."""
    import os
    import torch
    import torch.distributed as dist
    from blendtorch.parallel import comm as commmod
    from blendtorch.parallel.launch import free_port
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    monkeypatch.setenv('MASTER_PORT', str(free_port()))
    dist.init_process_group('gloo', rank=0, world_size=1)
    try:
        c = commmod.DeviceComm()
        assert not c.native
        c._comm = 1                      # pretend a borrowed communicator
        c._live()                        # group alive: fine
    finally:
        dist.destroy_process_group()
    with pytest.raises(RuntimeError, match='destroyed'):
        c._live()
    assert not c.native
    monkeypatch.setenv('TORCH_NCCL_USE_COMM_NONBLOCKING', '1')
    assert commmod._nonblocking()
    monkeypatch.setenv('TORCH_NCCL_USE_COMM_NONBLOCKING', '0')
    assert not commmod._nonblocking()


class _FakeEvent:
    def __init__(self, done_after):
        self.n = done_after

    def query(self):
        self.n -= 1
        return self.n < 0


def test_replay_watchdog_passes_finished_steps():
    """Events that complete (at once or after a few polls) never raise; the
    queue keeps at most ``depth`` steps in flight."""
    from blendtorch.parallel.step import ReplayWatchdog
    now = [0.0]
    wd = ReplayWatchdog(5.0, depth=3, make_event=lambda: _FakeEvent(2), clock=lambda: now[0],
                        sleep=lambda s: now.__setitem__(0, now[0] + s))
    for _ in range(10):
        wd.record()
        assert len(wd._q) <= 3
    wd.drain()
    assert wd.steps == 10 and not wd._q and wd.max_wait_s < 5.0


def test_replay_watchdog_names_the_rank_of_a_hung_step():
    """a replay that hangs on a collective raises with the
    rank and RCCL's asynchronous error instead of hanging the job."""
    from blendtorch.parallel.step import ReplayWatchdog
    now = [0.0]
    wd = ReplayWatchdog(2.0, depth=2, describe=lambda: 'rank 3/8, RCCL async error: unhandled system error',
                        make_event=lambda: _FakeEvent(10 ** 9), clock=lambda: now[0],
                        sleep=lambda s: now.__setitem__(0, now[0] + 0.25))
    wd.record()
    wd.record()
    with pytest.raises(RuntimeError, match=r'step 0 did not complete within 2 s .*rank 3/8.*unhandled system error'):
        wd.record()


def test_captured_step_strict_capture_and_watchdog_defaults(monkeypatch):
    """world > 1 all-reducing steps: strict capture (no silent eager fallback)
    and a watchdog by default; a 1-rank step keeps both off.  A strict step
    whose capture fails raises with the rank in the message."""
    import torch.distributed as dist
    from blendtorch.parallel import step as stepmod
    net = torch.nn.Linear(4, 1)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    s1 = stepmod.CapturedStep(net, opt, lambda m, x: m(x).sum(), allreduce=False, graph=False)
    assert not s1.strict and s1.watchdog is None
    s2 = stepmod.CapturedStep(net, opt, lambda m, x: m(x).sum(), allreduce=False, graph=False, strict=True)
    assert s2.strict
    s2.state = 'pending'

    def _graph(*a, **k):
        raise RuntimeError('operation not permitted when stream is capturing')
    fake_stream = type('S', (), {'wait_stream': lambda *a: None})
    monkeypatch.setattr(torch.cuda, 'Stream', lambda *a, **k: fake_stream())
    monkeypatch.setattr(torch.cuda, 'current_stream', lambda *a, **k: fake_stream())
    monkeypatch.setattr(torch.cuda, 'stream', lambda s: __import__('contextlib').nullcontext())
    monkeypatch.setattr(torch.cuda, 'CUDAGraph', lambda *a, **k: object())
    monkeypatch.setattr(torch.cuda, 'graph', _graph)
    with pytest.raises(RuntimeError, match=r'capture failed \(rank 0/1'):
        s2._capture(torch.ones(2, 4))
    assert s2.state == 'eager'
    assert not dist.is_initialized()
