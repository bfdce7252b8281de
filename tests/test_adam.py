"""ops.FusedAdam: the CPU reference path against torch.optim.Adam/AdamW, and
(GPU) the two-launch gfx950 update against that reference, in eager mode and
replayed from a captured HIP graph."""
import copy

import pytest
import torch

from blendtorch import ops


def _model(seed=0, device='cpu'):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 4, 2, 1), torch.nn.BatchNorm2d(8), torch.nn.Conv2d(8, 1, 3),
                               torch.nn.Flatten(), torch.nn.Linear(49, 3)).to(device)


def _grads(model, k, device='cpu'):
    g = torch.Generator().manual_seed(100 + k)
    for p in model.parameters():
        p.grad = torch.randn(p.shape, generator=g).to(device)


@pytest.mark.parametrize('wd,decoupled,maximize', [(0.0, False, False), (0.01, False, False), (0.05, True, False),
                                                   (0.0, False, True)])
def test_reference_path_matches_torch(wd, decoupled, maximize):
    a, b = _model(), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=wd,
                         decoupled=decoupled, maximize=maximize)
    cls = torch.optim.AdamW if decoupled else torch.optim.Adam
    ref = cls(b.parameters(), lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=wd, maximize=maximize)
    for k in range(6):
        _grads(a, k)
        _grads(b, k)
        ours.step()
        ref.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)


def test_state_dict_roundtrip_keeps_step():
    a = _model()
    opt = ops.FusedAdam(a.parameters(), lr=1e-2)
    for k in range(3):
        _grads(a, k)
        opt.step()
    sd = copy.deepcopy(opt.state_dict())   # state_dict() shares the live buffers
    assert all(float(s['step']) == 3 for s in sd['state'].values())
    b = _model()
    b.load_state_dict(a.state_dict())
    opt2 = ops.FusedAdam(b.parameters(), lr=1e-2)
    opt2.load_state_dict(sd)
    _grads(a, 7)
    _grads(b, 7)
    opt.step()
    opt2.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=0, atol=0)


def test_set_lr_and_param_group_lr():
    a, b = _model(), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2)
    ref = torch.optim.Adam(b.parameters(), lr=1e-2)
    _grads(a, 0)
    _grads(b, 0)
    ours.step()
    ref.step()
    ours.set_lr(3e-3)
    ref.param_groups[0]['lr'] = 3e-3
    _grads(a, 1)
    _grads(b, 1)
    ours.step()
    ref.step()
    ours.param_groups[0]['lr'] = 1e-3     # plain torch-style edit is honoured too
    ref.param_groups[0]['lr'] = 1e-3
    _grads(a, 2)
    _grads(b, 2)
    ours.step()
    ref.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)


def test_rejects_bad_hyperparameters():
    with pytest.raises(ValueError):
        ops.FusedAdam(_model().parameters(), lr=-1)
    with pytest.raises(ValueError):
        ops.FusedAdam(_model().parameters(), betas=(1.0, 0.9))


# ---------------------------------------------------------------------------
# GPU: the gfx950 kernels


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    ops.hip_ext()
    return torch.device('cuda', 0)


@pytest.mark.gpu
@pytest.mark.parametrize('wd,decoupled', [(0.0, False), (0.01, False), (0.05, True)])
def test_gpu_update_matches_reference(dev, wd, decoupled):
    a, b = _model(device=dev), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2, betas=(0.8, 0.95), weight_decay=wd, decoupled=decoupled,
                         bf16_shadow=True)
    ref = ops.FusedAdam(b.parameters(), lr=1e-2, betas=(0.8, 0.95), weight_decay=wd, decoupled=decoupled)
    before = ops.KERNEL_CALLS.get('adam_update', 0)
    for k in range(5):
        _grads(a, k, dev)
        _grads(b, k)
        ours.step()
        ref.step()
    assert ops.KERNEL_CALLS['adam_update'] == before + 5          # one launch per step for the whole model
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.cpu(), pb, rtol=1e-5, atol=1e-6)
        assert torch.equal(ours.shadow(pa), pa.detach().to(torch.bfloat16))
    assert float(ours.state[next(a.parameters())]['step']) == 5


@pytest.mark.gpu
def test_gpu_channels_last_parameters(dev):
    a, b = _model(device=dev).to(memory_format=torch.channels_last), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2)
    ref = ops.FusedAdam(b.parameters(), lr=1e-2)
    for k in range(3):
        _grads(a, k, dev)                # contiguous grads on channels-last weights: restrided
        _grads(b, k)
        ours.step()
        ref.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.cpu(), pb, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_gpu_bf16_grads_and_odd_sizes(dev):
    torch.manual_seed(3)
    ps = [torch.randn(n, device=dev, requires_grad=True) for n in (1, 3, 5, 1023, 4096 + 2)]
    qs = [p.detach().cpu().clone().requires_grad_(True) for p in ps]
    for p in ps:
        p.grad_dtype = None                # allow bf16 gradients on fp32 parameters
    ours = ops.FusedAdam(ps, lr=5e-3)
    ref = ops.FusedAdam(qs, lr=5e-3)
    for k in range(3):
        for p, q in zip(ps, qs):
            g = torch.randn(p.shape).to(torch.bfloat16)
            p.grad = g.to(dev)
            q.grad = g.float()
        ours.step()
        ref.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.detach().cpu(), q.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_gpu_graph_replay_advances_step_and_follows_set_lr(dev):
    a, b = _model(device=dev), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2)
    ref = ops.FusedAdam(b.parameters(), lr=1e-2)
    grads = [torch.zeros_like(p) for p in a.parameters()]   # static gradient buffers the graph reads
    for p, g in zip(a.parameters(), grads):
        p.grad = g

    def feed(k):
        _grads(b, k)
        for g, q in zip(grads, b.parameters()):
            g.copy_(q.grad)

    feed(0)
    ours.step()                          # eager step: allocates the state outside the capture
    ref.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):        # capture records, it does not run the update
        ours.step()
    for k in range(1, 6):
        if k == 3:
            ours.set_lr(2e-3)
            ref.set_lr(2e-3)
        feed(k)
        graph.replay()
        ref.step()
    torch.cuda.synchronize()
    assert float(ours.state[next(a.parameters())]['step']) == 6
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.detach().cpu(), pb.detach(), rtol=1e-5, atol=1e-6)


def test_reference_grad_scale_and_gate():
    """grad_scale multiplies the gradient inside the update; a closed gate
    leaves counter, moments and weights untouched."""
    a, b = _model(), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2, grad_scale=0.25)
    ref = torch.optim.Adam(b.parameters(), lr=1e-2)
    for k in range(4):
        _grads(a, k)
        _grads(b, k)
        for q in b.parameters():
            q.grad.mul_(0.25)
        ours.step(gate=torch.ones(1))
        ref.step()
        before = [p.detach().clone() for p in a.parameters()]
        _grads(a, 50 + k)
        ours.step(gate=torch.zeros(1))        # skipped entirely
        assert all(torch.equal(x, p) for x, p in zip(before, a.parameters()))
    assert float(ours.state[next(a.parameters())]['step']) == 4
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
    ours.set_grad_scale(1.0)
    assert ours.grad_scale == 1.0


def test_load_state_dict_twice_into_stepped_optimizer():
    """Loading a state dict (twice, into an optimizer that already stepped)
    takes the loaded step counter, never a stale per-group counter."""
    a = _model()
    opt = ops.FusedAdam(a.parameters(), lr=1e-2)
    for k in range(3):
        _grads(a, k)
        opt.step()
    sd3 = copy.deepcopy(opt.state_dict())
    _grads(a, 3)
    opt.step()
    sd4 = copy.deepcopy(opt.state_dict())
    b = _model()
    opt2 = ops.FusedAdam(b.parameters(), lr=1e-2)
    _grads(b, 9)
    opt2.step()
    opt2.load_state_dict(sd3)
    opt2.load_state_dict(sd4)
    b.load_state_dict(a.state_dict())
    _grads(a, 5)
    _grads(b, 5)
    opt.step()
    opt2.step()
    assert float(opt2.state[next(b.parameters())]['step']) == 5
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=0, atol=0)


@pytest.mark.gpu
def test_gpu_grad_scale_and_gate_in_graph(dev):
    """Captured: the gate tensor is read on every replay (skip without a host
    sync), grad_scale matches the reference path."""
    a, b = _model(device=dev), _model()
    ours = ops.FusedAdam(a.parameters(), lr=1e-2, grad_scale=0.5)
    ref = ops.FusedAdam(b.parameters(), lr=1e-2, grad_scale=0.5)
    grads = [torch.zeros_like(p) for p in a.parameters()]
    for p, g in zip(a.parameters(), grads):
        p.grad = g
    gate = torch.ones(1, device=dev)

    def feed(k):
        _grads(b, k)
        for g, q in zip(grads, b.parameters()):
            g.copy_(q.grad)

    feed(0)
    ours.step(gate=gate)
    ref.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ours.step(gate=gate)
    for k in range(1, 7):
        feed(k)
        open_ = k % 2 == 0
        gate.fill_(1.0 if open_ else 0.0)
        graph.replay()
        if open_:
            ref.step()
    torch.cuda.synchronize()
    assert float(ours.state[next(a.parameters())]['step']) == 4
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.detach().cpu(), pb.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_gpu_one_launch_zero_grads_and_conv_shadows(dev):
    """One update launch per step (the schedule worked out in-kernel, the last
    block storing the counter), gradients cleared after use (also behind a
    closed gate), and the bf16 conv-weight shadow plus its data-gradient
    transpose kept equal to cast + conv_weights_t of the new weights --
    eager and replayed from a graph."""
    def conv_model(device='cpu'):
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Conv2d(4, 64, 4, 2, 1), torch.nn.BatchNorm2d(64),
                                   torch.nn.Conv2d(64, 32, 4, 2, 1, bias=False), torch.nn.Conv2d(32, 8, 4, 2, 1)).to(device)

    a, b = conv_model(dev), conv_model()
    a = a.to(memory_format=torch.channels_last)
    ours = ops.FusedAdam(a.parameters(), lr=1e-2, betas=(0.8, 0.95), one_launch=True)
    ref = ops.FusedAdam(b.parameters(), lr=1e-2, betas=(0.8, 0.95))
    conv = [m.weight for m in a if isinstance(m, torch.nn.Conv2d) and tuple(m.kernel_size) == (4, 4)]
    ours.enable_conv_shadows(conv)
    ours.set_zero_grads(True)
    grads = [torch.zeros_like(p) for p in a.parameters()]
    for p, g in zip(a.parameters(), grads):
        p.grad = g
    gate = torch.ones(1, device=dev)

    def feed(k):
        _grads(b, k)
        for g, q in zip(grads, b.parameters()):
            g.copy_(q.grad)

    before = (ops.KERNEL_CALLS.get('adam_update', 0), ops.KERNEL_CALLS.get('adam_schedule', 0))
    feed(0)
    ours.step(gate=gate)
    ref.step()
    assert ops.KERNEL_CALLS['adam_update'] == before[0] + 1
    assert ops.KERNEL_CALLS.get('adam_schedule', 0) == before[1]          # no schedule launch
    assert all(int(torch.count_nonzero(g)) == 0 for g in grads)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ours.step(gate=gate)
    steps = 1
    for k in range(1, 8):
        feed(k)
        open_ = k % 3 != 0
        gate.fill_(1.0 if open_ else 0.0)
        graph.replay()
        if open_:
            ref.step()
            steps += 1
        torch.cuda.synchronize()
        assert all(int(torch.count_nonzero(g)) == 0 for g in grads), k    # consumed, also when gated
    assert float(ours.state[next(a.parameters())]['step']) == steps
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.detach().cpu(), pb.detach(), rtol=1e-5, atol=1e-6)
    transposed = 0
    for w in conv:
        w16 = w.detach().to(torch.bfloat16)
        assert torch.equal(ours.shadow(w), w16)
        if 'shadow_t' in ours.state[w]:      # Cout, Cin multiples of 32
            transposed += 1
            assert torch.equal(ours.shadow_t(w), ops.conv_weights_t([w16])[0])
    assert transposed == 1


@pytest.mark.gpu
def test_gpu_discriminator_step_with_optimizer_shadows(dev):
    """The bench's disc step with the conv weights read from FusedAdam's
    shadows (no cast / transpose launches) and persistent gradient buckets
    cleared by the update (no fill) trains like the cast-every-step path."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
          for _ in range(4)]
    nets = []
    for shadow in (False, True):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        if shadow:
            m.use_optimizer_shadows(opt)
        step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                            buckets=shadow)
        casts = ops.KERNEL_CALLS.get('multi_cast', 0)
        for x in xs:
            step(x)
        torch.cuda.synchronize()
        assert step.state == 'graph'
        if shadow:
            assert ops.KERNEL_CALLS.get('multi_cast', 0) == casts    # no per-step weight casts captured
            assert step.grads is not None
        nets.append(m)
    lr = 2e-4
    for pa, pb in zip(nets[0].parameters(), nets[1].parameters()):
        d = (pb - pa).detach().abs()
        assert float(d.mean()) < 0.15 * lr and float((d > 0.5 * lr).float().mean()) < 0.03


@pytest.mark.gpu
def test_gpu_one_launch_schedule_ahead_follows_lr_changes(dev):
    """One-launch form: the schedule worked out ahead (by the previous
    update's last block) stays right across lr and gradient-scale changes and
    closed gates -- identical to the two-launch form step by step."""
    torch.manual_seed(3)
    ps = [torch.randn(n, device=dev) for n in (1000, 4096, 7)]
    runs = []
    for one in (True, False):
        params = [torch.nn.Parameter(p.clone()) for p in ps]
        opt = ops.FusedAdam(params, lr=1e-2, betas=(0.9, 0.99), one_launch=one)
        gate = torch.ones(1, device=dev)
        g = torch.Generator(device=dev).manual_seed(7)
        for k in range(9):
            for p in params:
                p.grad = torch.randn(p.shape, device=dev, generator=g)
            if k == 3:
                opt.set_lr(3e-3)
            if k == 5:
                opt.set_grad_scale(0.5)
            if k == 6:
                opt.param_groups[0]['lr'] = 5e-3          # edited through param_groups
            gate.fill_(0.0 if k == 4 else 1.0)
            opt.step(gate=gate)
        torch.cuda.synchronize()
        runs.append([p.detach().clone() for p in params] + [opt._group_state(opt.param_groups[0])['step'].clone()])
    for x, y in zip(*runs):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_schedule_attached_to_backward_reduce(monkeypatch):
    """CapturedStep hands FusedAdam's schedule to the backward's last weight-
    gradient slice-reduce launch (FusedAdam.attach_schedule): no schedule
    launch, and the weights and step counter are bit-identical to the
    schedule kernel's -- eager and captured.  A model whose backward has no
    such launch (an MLP) falls back to the schedule kernel."""
    from blendtorch import ops
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    import blendtorch.ops.adam as adam_mod
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.rand(4, 3, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
          for _ in range(4)]
    outs = []
    for attach in (True, False):
        monkeypatch.setattr(adam_mod, '_ATTACH', attach)
        torch.manual_seed(8)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        st = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, warmup=1)
        before = (ops.KERNEL_CALLS.get('adam_schedule', 0), ops.KERNEL_CALLS.get('adam_schedule_attached', 0))
        for x in xs:
            st(x)
        torch.cuda.synchronize()
        assert st.state == 'graph'
        sched = ops.KERNEL_CALLS.get('adam_schedule', 0) - before[0]
        att = ops.KERNEL_CALLS.get('adam_schedule_attached', 0) - before[1]
        assert (att > 0 and sched == 0) if attach else (att == 0 and sched > 0)
        steps = float(opt._group_state(opt.param_groups[0])['step'])
        outs.append(([p.detach().clone() for p in m.parameters()], steps))
    (pa, sa), (pb, sb) = outs
    assert sa == sb and sa >= 1
    # (the weight gradients' slice groups add with float atomics: the runs differ by
    # rounding, which early Adam steps scale to about +-lr -- nearly every weight agrees)
    lr = 2e-4
    for a, b in zip(pa, pb):
        d = (a - b).abs()
        assert float(d.mean()) < 0.1 * lr and float((d > 0.5 * lr).float().mean()) < 0.02
    monkeypatch.setattr(adam_mod, '_ATTACH', True)
    mlp = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1)).to(dev)
    opt = ops.FusedAdam(mlp.parameters(), lr=1e-3)
    st = CapturedStep(mlp, opt, lambda mm, x: mm(x).pow(2).mean(), allreduce=False, warmup=1)
    before = ops.KERNEL_CALLS.get('adam_schedule', 0)
    for _ in range(3):
        st(torch.randn(8, 16, device=dev))
    torch.cuda.synchronize()
    assert ops.KERNEL_CALLS.get('adam_schedule', 0) > before
    assert not ops.hip_ext().adam_schedule_taken()


@pytest.mark.gpu
def test_update_takes_backward_reduce(monkeypatch):
    """CapturedStep lets FusedAdam's update take the backward's last weight-
    gradient slice reduce (FusedAdam.attach_reduce): extra blocks of the update
    launch sum the deferred slices, update that weight and write its gradient.
    Weights and moments agree with the plain path's (its own reduce launch),
    and no claim outlives the step."""
    from blendtorch import ops
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    import blendtorch.ops.adam as adam_mod
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.rand(4, 3, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
          for _ in range(4)]
    outs = []
    for fuse in (True, False):
        monkeypatch.setattr(adam_mod, '_FUSE_REDUCE', fuse)
        torch.manual_seed(8)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        st = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, warmup=1)
        before = ops.KERNEL_CALLS.get('adam_fused_reduce', 0)
        for x in xs:
            st(x)
        torch.cuda.synchronize()
        assert st.state == 'graph'
        n = ops.KERNEL_CALLS.get('adam_fused_reduce', 0) - before
        assert (n > 0) if fuse else (n == 0)
        assert ops._REDUCE_CLAIM is None
        ps = list(m.parameters())
        outs.append(([p.detach().clone() for p in ps], [opt.state[p]['exp_avg'].clone() for p in ps]))
    (pa, ma), (pb, mb) = outs
    lr = 2e-4
    for a, b in zip(pa, pb):   # (slice groups of some layers add with float atomics: rounding)
        d = (a - b).abs()
        assert float(d.mean()) < 0.1 * lr and float((d > 0.5 * lr).float().mean()) < 0.02
    for a, b in zip(ma, mb):   # (the same rounding, through four steps)
        assert float((a - b).abs().mean()) <= 0.05 * float(b.abs().mean()) + 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize('zero', [False, True])
def test_fused_reduce_update_matches_plain(zero):
    """One 4x4 weight gradient (32 -> 64 channels) whose ordered slice reduce
    is handed to FusedAdam (AdamParams::fr) against the same reduce launched on
    its own and the plain update: identical gradient bits (or zeros under
    set_zero_grads) and the same weights and moments."""
    from blendtorch import ops
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(2, 32, 64, 96, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(2, 64, 32, 48, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w0 = (0.05 * torch.randn(64, 32, 4, 4, device=dev, generator=g)).contiguous(memory_format=cl)
    res = []
    for fuse in (True, False):
        w = torch.nn.Parameter(w0.clone())
        out = torch.zeros_like(w)
        w.grad = out
        w._bt_grad_sink = out
        opt = ops.FusedAdam([w], lr=1e-3, weight_decay=0.01)
        opt.set_zero_grads(zero)
        before = ops.KERNEL_CALLS.get('adam_fused_reduce', 0)
        for _ in range(2):
            if fuse:
                ops._REDUCE_CLAIM = {'params': {id(w)}, 'got': None}
            ops.conv_wgrad(x, dy, out, param=w)
            if fuse:
                assert ops._REDUCE_CLAIM['got'] is not None
            opt.step()
            ops._REDUCE_CLAIM = None
        torch.cuda.synchronize()
        assert (ops.KERNEL_CALLS.get('adam_fused_reduce', 0) - before == 2) == fuse
        st = opt.state[w]
        res.append((w.detach().clone(), st['exp_avg'].clone(), st['exp_avg_sq'].clone(), out.clone()))
    (wa, ma, va, ga), (wb, mb, vb, gb) = res
    assert torch.equal(ga, gb)
    if zero:
        assert not ga.any()
    for a, b in ((wa, wb), (ma, mb), (va, vb)):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-9)
