"""Consumer-step ops added in round 2: the one-launch multi-tensor bf16 cast,
the autocast-free bf16 discriminator forward built on it, and the BN
counter folded into the finalize kernel."""
import pytest
import torch

from blendtorch import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    ops.hip_ext()
    return torch.device('cuda', 0)


def test_cast_bf16_matches_torch(dev):
    g = torch.Generator(device=dev).manual_seed(0)
    ws = [torch.randn(s, device=dev, generator=g) * 3 for s in [(32, 3, 4, 4), (7,), (1, 1, 1, 1), (5, 1023)]]
    ws[0] = ws[0].to(memory_format=torch.channels_last)
    ws[1][2] = float('nan')
    ws[1][3] = float('inf')
    for w in ws:
        w.requires_grad_(True)
    before = ops.KERNEL_CALLS.get('multi_cast', 0)
    outs = ops.cast_bf16(*ws)
    assert ops.KERNEL_CALLS['multi_cast'] == before + 1          # one launch for all four
    for w, o in zip(ws, outs):
        ref = w.detach().to(torch.bfloat16)
        assert o.dtype == torch.bfloat16 and o.stride() == ref.stride()
        assert torch.equal(o.isnan(), ref.isnan())
        assert torch.equal(torch.nan_to_num(o.float()), torch.nan_to_num(ref.float()))
    grads = [torch.randn(o.shape, device=dev, generator=g).to(torch.bfloat16) for o in outs]
    torch.autograd.backward(outs, grads)
    assert ops.KERNEL_CALLS['multi_cast'] == before + 2          # ... and one back
    for w, gr in zip(ws, grads):
        assert w.grad.dtype == torch.float32 and torch.equal(w.grad, gr.float())


def test_discriminator_forward_bf16_equals_autocast(dev):
    from blendtorch.models import Discriminator
    torch.manual_seed(0)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 240, 320, 3, device=dev).to(torch.bfloat16).permute(0, 3, 1, 2)
    with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
        ya = a(x)
    yb = b.forward_bf16(x, mfma=False)
    torch.testing.assert_close(yb.float(), ya.float(), rtol=0, atol=0)
    ya.float().sum().backward()
    yb.float().sum().backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pb.grad, pa.grad, rtol=2e-2, atol=1e-3, msg=n)
    for ma, mb in zip(a.modules(), b.modules()):
        if isinstance(ma, ops.BatchNormLeakyReLU2d):
            assert int(ma.num_batches_tracked) == int(mb.num_batches_tracked) == 1   # counted on the device
            torch.testing.assert_close(mb.running_mean, ma.running_mean, rtol=1e-4, atol=1e-6)


def _split_vs_single(dev, make, loss_fn, xs, lr):
    from blendtorch.parallel.step import CapturedStep
    torch.manual_seed(0)
    nets = [make() for _ in range(2)]
    nets[1].load_state_dict(nets[0].state_dict())
    steps = [CapturedStep(n, ops.FusedAdam(n.parameters(), lr=lr), loss_fn, allreduce=False, warmup=2, split=s)
             for n, s in zip(nets, (False, True))]
    hits = []
    for x in xs:
        steps[0](x)
        steps[1](x, mid=lambda: hits.append(1))
    torch.cuda.synchronize()
    assert steps[1].state == 'graph' and steps[1].graph_bwd is not None and len(hits) == len(xs)
    return list(zip(nets[0].parameters(), nets[1].parameters()))


def test_split_graph_step_equals_single_graph(dev):
    """CapturedStep(split=True): forward and backward+update as two graphs in
    one pool replay to the same weights as the one-graph step (an MLP: GEMMs
    and elementwise kernels sum in a fixed order, so bit-exact)."""
    def make():
        return torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.GELU(), torch.nn.Linear(128, 8)).to(dev)

    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.randn(32, 64, device=dev, generator=g) for _ in range(5)]
    for pa, pb in _split_vs_single(dev, make, lambda m, x: m(x).pow(2).mean(), xs, 1e-2):
        torch.testing.assert_close(pb, pa, rtol=0, atol=0)


def test_split_graph_discriminator_step(dev):
    """The bench consumer step split in two graphs trains like the one-graph
    step.  MIOpen's weight-gradient kernels sum with atomics, so the two runs
    differ by rounding; early Adam steps move each weight by about +-lr, so
    the check is that nearly every weight agrees far below lr."""
    from blendtorch.models import Discriminator
    lr = 2e-4
    crit = torch.nn.BCELoss()

    def make():
        return Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)

    def loss_fn(m, x):
        out = m.forward_bf16(x).float()
        return crit(out, torch.ones_like(out))

    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.rand(4, 3, 96, 128, device=dev, generator=g).to(torch.bfloat16)
          .contiguous(memory_format=torch.channels_last) for _ in range(4)]
    for pa, pb in _split_vs_single(dev, make, loss_fn, xs, lr):
        d = (pb - pa).detach().abs()
        assert float(d.mean()) < 0.1 * lr and float((d > 0.5 * lr).float().mean()) < 0.02


@pytest.mark.parametrize('target', ['ones', 'mixed'])
@pytest.mark.parametrize('wlayout', ['contiguous', 'channels_last'])
def test_disc_head_bce_matches_fp32_reference(dev, target, wlayout):
    import torch.nn.functional as F
    g = torch.Generator(device=dev).manual_seed(11)
    z = (0.5 * torch.randn(8, 256, 30, 40, device=dev, generator=g)).to(torch.bfloat16)
    z = z.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = 0.02 * torch.randn(1, 256, 4, 4, device=dev, generator=g)
    if wlayout == 'channels_last':
        w = w.contiguous(memory_format=torch.channels_last)
    w.requires_grad_(True)
    y = torch.ones(8, device=dev) if target == 'ones' else torch.tensor([1., 0., 1., 1., 0., 0., 1., 0.], device=dev)
    before = ops.KERNEL_CALLS.get('head_forward', 0)
    loss, logits = ops.disc_head_bce(z, w, 1.0 if target == 'ones' else y)
    loss.backward()
    assert ops.KERNEL_CALLS['head_forward'] == before + 1
    zr = z.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    out = torch.sigmoid(F.conv2d(F.adaptive_avg_pool2d(zr, 4), wr)).view(-1)
    ref = F.binary_cross_entropy(out, y)
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.sigmoid(logits), out.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-4, atol=1e-7)
    assert z.grad.dtype == torch.bfloat16 and z.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(z.grad.float(), zr.grad, rtol=2 ** -7, atol=1e-3 * float(zr.grad.abs().max()))


@pytest.mark.parametrize('N,H,W', [(4, 240, 320), (3, 96, 128)])
def test_head_fwd_lean_kernel_matches_round4_kernel(dev, N, H, W):
    """The BN-applying head forward's round-trip-lean kernel (all window loads
    and the accumulator read up front, combined tickets) gives bit-identical
    losses, running statistics and gradients to round 4's head_fwd_kernel, and
    leaves the accumulators cleared (two steps: the second reuses them).
    96 x 128: a 6 x 8 head input, 4-pixel windows -- fewer than the lanes per
    pixel group, whose padding loads must stay inside the window."""
    from blendtorch.models import Discriminator
    ext = ops.hip_ext()
    runs = []
    try:
        for fast in (1, 0):
            ext.head_set_fast(fast)
            torch.manual_seed(0)
            m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
            m.lazy_head_bn = True
            g = torch.Generator(device=dev).manual_seed(4)
            out = []
            for _ in range(2):
                x = torch.rand(N, 3, H, W, device=dev, generator=g).to(torch.bfloat16)
                x = x.contiguous(memory_format=torch.channels_last)
                m.zero_grad(set_to_none=True)
                loss = m.bce_loss_bf16(x, 1.0)
                loss.backward()
                out.append(loss.detach().clone())
            rings = 0
            for mod in m.modules():   # every accumulator cleared by the kernels that folded it
                ring = mod.__dict__.get('_bt_acc_ring') if isinstance(mod, ops.BatchNormLeakyReLU2d) else None
                for acc in (ring[0] if ring else []):
                    assert int(torch.count_nonzero(acc.fwd)) == 0 and int(torch.count_nonzero(acc.bwd)) == 0
                rings += ring is not None
            assert rings >= 3            # (an RGB first layer takes the apply pass, not an accumulator)
            runs.append((out, [b.clone() for b in m.buffers()], [p.grad.clone() for p in m.parameters()]))
    finally:
        ext.head_set_fast(-1)
    (la, ba, ga), (lb, bb, gb) = runs
    assert all(torch.equal(x, y) for x, y in zip(la, lb)), (la, lb)
    assert all(torch.equal(x, y) for x, y in zip(ba, bb))
    for x, y in zip(ga, gb):   # (the weight-gradient reduce adds with fp32 atomics: order varies)
        assert float((x - y).abs().max()) <= 1e-2 * float(y.abs().max())


def test_discriminator_bce_loss_bf16(dev):
    """The fused-head loss of the whole discriminator equals the unfused
    bf16 forward + BCELoss, and trains the same parameters."""
    from blendtorch.models import Discriminator
    torch.manual_seed(0)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 120, 160, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    la = a.bce_loss_bf16(x, 1.0)
    out = b.forward_bf16(x).float()
    lb = torch.nn.functional.binary_cross_entropy(out, torch.ones_like(out))
    torch.testing.assert_close(la, lb, rtol=2e-2, atol=1e-4)   # the head pools/dots in fp32, the library in bf16
    la.backward()
    lb.backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        ga, gb = pa.grad.flatten().double(), pb.grad.flatten().double()
        assert float(ga @ gb / (ga.norm() * gb.norm())) > 0.98, n


def test_lazy_bn_applies_match_apply_pass(dev):
    """Every BatchNorm+LeakyReLU forward apply moved into its consumer
    (ops.BnActLazy: the next convolution's operand staging, or the fused
    head's pooling for the last one) and every backward apply into the
    producing convolution's weight gradient (ops.BnBwdFold) -- no apply
    launch either way -- gives the SAME loss and running statistics as the
    apply passes, and the same gradients up to the weight-gradient reduce's
    atomic order: the kernels compute the same bf16 values from the same
    folded statistics."""
    from blendtorch.models import Discriminator
    torch.manual_seed(0)
    nets = []
    for lazy in (True, False):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
        m.lazy_head_bn = m.lazy_conv_bn = m.defer_bn_bwd = lazy
        nets.append(m)
    g = torch.Generator(device=dev).manual_seed(2)
    before = ops.KERNEL_CALLS.get('bn_forward_lazy', 0)
    before_bwd = ops.KERNEL_CALLS.get('bn_backward_deferred_fold', 0)
    for _ in range(2):   # the second step re-uses the accumulators the first step's consumers cleared
        # (even sides down to the last convolution's input: every BN applies lazily)
        # RGBA frames: the first layer runs on the MFMA path, so its BN is lazy too
        x = torch.rand(4, 4, 128, 160, device=dev, generator=g).to(torch.bfloat16)
        x = x.contiguous(memory_format=torch.channels_last)
        losses = []
        for m in nets:
            m.zero_grad(set_to_none=True)
            loss = m.bce_loss_bf16(x, 1.0)
            loss.backward()
            losses.append(loss.detach())
        assert torch.equal(losses[0], losses[1])
        for (n, ba), bb in zip(nets[0].named_buffers(), nets[1].buffers()):
            assert torch.equal(ba, bb), n
        for mod in nets[0].modules():   # every accumulator cleared by the kernels that folded it
            if isinstance(mod, ops.BatchNormLeakyReLU2d):
                for acc in mod.__dict__['_bt_acc_ring'][0]:
                    assert int(torch.count_nonzero(acc.fwd)) == 0 and int(torch.count_nonzero(acc.bwd)) == 0
        # (with BT_WGRAD_ORDERED=0 the weight gradients' slice groups add with fp32 atomics,
        # whose order varies between runs: the tolerance covers that mode too)
        for (n, pa), pb in zip(nets[0].named_parameters(), nets[1].parameters()):
            tol = 1e-2 * float(pb.grad.abs().max())
            assert float((pa.grad - pb.grad).abs().max()) <= tol, (n, float((pa.grad - pb.grad).abs().max()), tol)
    assert ops.KERNEL_CALLS['bn_forward_lazy'] == before + 2 * 4   # all 4 BNs, 2 steps
    # and every BN backward ran in the producing convolution's weight gradient
    assert ops.KERNEL_CALLS['bn_backward_deferred_fold'] == before_bwd + 2 * 4


def _disc_steps(dev, buckets, graph, xs, grad_scale=None):
    from blendtorch.models import Discriminator
    from blendtorch.parallel import GradBuckets
    from blendtorch.parallel.step import CapturedStep
    torch.manual_seed(0)
    m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    opt = ops.FusedAdam(m.parameters(), lr=2e-4)
    gb = GradBuckets(m.parameters()) if buckets else None
    step = CapturedStep(m, opt, lambda mod, x: mod.bce_loss_bf16(x, 1.0), allreduce=False, warmup=2, graph=graph)
    step.grads = gb                 # buckets without a process group: zero_() per step, no collective
    ptrs = [p.grad.data_ptr() for p in m.parameters()] if gb is not None else None
    for x in xs:
        step(x)
    torch.cuda.synchronize()
    if gb is not None:
        assert [p.grad.data_ptr() for p in m.parameters()] == ptrs     # gradients never left the buckets
    return m, step


@pytest.mark.parametrize('graph', [False, True])
def test_bucketed_grads_written_in_place_train_identically(dev, graph):
    """The fused backward kernels (MFMA weight gradient, BN, head) write each
    parameter's gradient straight into its GradBuckets view: training matches
    ordinary per-step gradient tensors, eager and graphed.  (Not bit-exact:
    the weight-gradient slice reduce adds slice groups with float atomics, so
    two runs differ by rounding; early Adam steps move each weight by ~lr,
    so nearly every weight must agree far below lr.)"""
    g = torch.Generator(device=dev).manual_seed(7)
    xs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16)
          .contiguous(memory_format=torch.channels_last) for _ in range(4)]
    a, _ = _disc_steps(dev, False, graph, xs)
    before = ops.KERNEL_CALLS.get('conv_wgrad', 0)
    b, sb = _disc_steps(dev, True, graph, xs)
    assert ops.KERNEL_CALLS['conv_wgrad'] > before
    assert sb.state == ('graph' if graph else 'eager')
    lr = 2e-4
    for pa, pb in zip(a.parameters(), b.parameters()):
        d = (pb - pa).detach().abs()
        assert float(d.mean()) < 0.1 * lr and float((d > 0.5 * lr).float().mean()) < 0.02


def test_rccl_direct_one_rank_process_group(dev, tmp_path):
    """A 1-rank RCCL process group in a child process: DeviceComm calls RCCL
    on the compute stream (native), passes its start-up self-check, and the
    graphed DP step with its in-graph bucket all-reduce trains like the same
    step without a process group (not bit-identically: the weight-gradient
    slice reduce and the BatchNorm statistics add with float atomics, so the
    runs differ by rounding; lr = 2e-4 per Adam step)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    script = Path(__file__).with_name('rccl_worker.py')
    out = tmp_path / 'res.json'
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', RANK='0', WORLD_SIZE='1', LOCAL_RANK='0')
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    env['MASTER_PORT'] = str(s.getsockname()[1])
    s.close()
    r = subprocess.run([sys.executable, str(script), str(out)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(out.read_text())
    assert res['native'] and res['selfcheck']['native']
    assert res['collectives'] == 1 and res['state'] == 'graph'
    assert res['max_abs_diff'] < 1e-3 and res['mean_abs_diff'] < 2e-5 and res['frac_above_half_lr'] < 0.02
    assert res['allreduce_avg_ok'] and res['broadcast_ok'] and res['p2p_self_ok']
    # two buckets, the last layers' all-reduced ahead of the first layers' weight
    # gradients: captured (the last recorded step is the capture), issued after
    # 2 of the 4 weight-gradient launches, trains like the one-bucket step
    ov = res['overlap']
    assert ov['collectives'] == 2 and ov['state'] == 'graph', ov
    (b0, n0), (b1, n1) = ov['order'][-2:]
    assert (b0, b1) == (0, 1) and n1 - n0 == 2, ov['order']
    assert ov['max_abs_diff'] < 1e-3


def test_densityopt_step_captures_and_replays(dev):
    """The whole densityopt iteration (gated D step on the bf16 MFMA
    discriminator, gated S step, baseline, resampling) captures into one HIP
    graph and replays; the decisions stay device tensors (0/1) and the
    parameter samples stay finite and positive (LogNormal)."""
    from blendtorch.models import Discriminator, ProbModel
    from blendtorch.models.densityopt import DensityOptStep
    B = 64
    torch.manual_seed(0)
    netD = Discriminator().to(dev).to(memory_format=torch.channels_last)
    pm = ProbModel([1.2, 3.0], [0.4, 0.4]).to(dev)
    g = torch.Generator(device=dev).manual_seed(2)

    def batch():
        return (torch.rand(B, 64, 64, 4, device=dev, generator=g) * 2 - 1).to(torch.bfloat16).permute(0, 3, 1, 2)

    step = DensityOptStep(netD, pm, batch().clone(), B, graph=True, warmup=2)
    step.start()
    before = ops.KERNEL_CALLS.get('conv_fwd', 0)
    for i in range(6):
        step(batch(), torch.randperm(B))
    torch.cuda.synchronize()
    assert step.graph is not None and ops.KERNEL_CALLS['conv_fwd'] > before
    assert float(step.gate_d) in (0.0, 1.0) and float(step.gate_s) in (0.0, 1.0)
    assert bool(torch.isfinite(step.samples).all()) and bool((step.samples > 0).all())
    assert bool(torch.isfinite(step.params_out).all())


def test_densityopt_step_prefetch_matches_inline(dev):
    """DensityOptStep.prefetch(): the real-batch half replayed from its own
    graph ahead of the sim batch trains exactly like the inline iteration
    (warm-up, capture and replays; same inputs, same seeds)."""
    from blendtorch.models import Discriminator, ProbModel
    from blendtorch.models.densityopt import DensityOptStep
    B = 64
    outs = []
    for pre in (False, True):
        torch.manual_seed(0)
        netD = Discriminator().to(dev).to(memory_format=torch.channels_last)
        pm = ProbModel([1.2, 3.0], [0.4, 0.4]).to(dev)
        g = torch.Generator(device=dev).manual_seed(3)

        def batch():
            return (torch.rand(B, 64, 64, 4, device=dev, generator=g) * 2 - 1).to(torch.bfloat16).permute(0, 3, 1, 2)

        step = DensityOptStep(netD, pm, batch().clone(), B, graph=True, warmup=2)
        torch.manual_seed(1)
        step.start()
        sids = torch.Generator().manual_seed(4)
        hist = []
        for i in range(7):
            sim = batch()
            if pre:
                step.prefetch()
            step(sim, torch.randperm(B, generator=sids))
            hist.append(step.params_out.clone())
        torch.cuda.synchronize()
        assert step.graph is not None and step.graph_real is not None
        outs.append((torch.stack(hist), [p.detach().clone() for p in netD.parameters()]))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-6)
    for a, b in zip(outs[0][1], outs[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_captured_step_static_inputs_read_in_place(dev):
    """CapturedStep(static_inputs=N): one graph per input tensor, reading it
    in place (no copy into a static buffer) -- trains like the copy path over
    alternating inputs, and an input past N falls back to the copy."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(5)
    bufs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
            for _ in range(3)]
    nets, losses = [], []
    for static in (0, 2):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                            static_inputs=static)
        ls = []
        for k in range(7):
            ls.append(float(step(bufs[k % 3])))
        torch.cuda.synchronize()
        assert step.state == 'graph'
        if static:                                     # the third tensor took the copy path
            assert len(step._by_input) == 3 and 'copy' in step._by_input
        nets.append(m)
        losses.append(ls)
    torch.testing.assert_close(torch.tensor(losses[0]), torch.tensor(losses[1]), rtol=2e-3, atol=1e-4)
    lr = 2e-4
    for pa, pb in zip(nets[0].parameters(), nets[1].parameters()):
        d = (pb - pa).detach().abs()
        assert float(d.mean()) < 0.15 * lr


def _seven_steps(dev, bufs, fused_u8=False):
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    torch.manual_seed(0)
    m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    opt = ops.FusedAdam(m.parameters(), lr=2e-4)
    m.use_optimizer_shadows(opt)
    dec = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    if fused_u8:
        fn = lambda mm, x: mm.bce_loss_bf16(x.permute(0, 3, 1, 2), 1.0, decode=dec)   # noqa: E731
    else:
        fn = lambda mm, x: mm.bce_loss_bf16(x, 1.0)   # noqa: E731
    step = CapturedStep(m, opt, fn, allreduce=False, graph=True, static_inputs=2)
    ls = [step(bufs[k % 3]).clone() for k in range(7)]
    torch.cuda.synchronize()
    assert step.state == 'graph', step.error
    return torch.stack(ls), [p.detach().clone() for p in m.parameters()], \
        [b.detach().clone() for b in m.buffers()]


@pytest.mark.parametrize('fused_u8', [False, True], ids=['bf16', 'u8_fused'])
def test_training_step_is_bit_deterministic(dev, fused_u8):
    """the same 7 graphed steps twice in one process give
    bit-identical losses, weights and BN buffers.  The r5b12 miss (loss rel
    3.2e-3 over 7 steps) came from the weight-gradient slice reduce adding
    its 8-slice groups with fp32 atomics in arrival order; Adam turns the
    last-bit differences of near-zero gradients into lr-sized steps.  The
    slice reduce is now ordered (wgrad_reduce_ordered: fixed per-lane order,
    fixed xor-shuffle tree, plain stores).  The remaining atomics are the
    fp64 BatchNorm / head sums: fp32 values added in fp64 round to the same
    fp32 result in any order unless a sum lands within ~1e-16 of an fp32
    rounding boundary (odds ~1e-9 per value)."""
    g = torch.Generator(device=dev).manual_seed(9)
    cl = torch.channels_last
    if fused_u8:
        bufs = [torch.randint(0, 256, (4, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g)
                for _ in range(3)]
    else:
        bufs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
                for _ in range(3)]
    la, pa, ba = _seven_steps(dev, bufs, fused_u8)
    lb, pb, bb = _seven_steps(dev, bufs, fused_u8)
    assert torch.equal(la, lb), (la - lb).abs().max()
    for i, (x, y) in enumerate(zip(pa, pb)):
        assert torch.equal(x, y), (i, float((x - y).abs().max()))
    for i, (x, y) in enumerate(zip(ba, bb)):
        assert torch.equal(x, y), (i, float((x.double() - y.double()).abs().max()))


def test_captured_step_pair_steps_train_like_single_steps(dev):
    """CapturedStep(pair_steps=True): consecutive steps run in pairs from one
    graph per pair of input tensors; a held step runs when the next arrives or
    at flush().  Same training as one graph per step (7 steps: three pairs,
    then a flushed single)."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(7)
    bufs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
            for _ in range(4)]
    keep = [b.clone() for b in bufs]
    nets = []
    for pair in (False, True):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                            static_inputs=4, pair_steps=pair)
        held = 0
        for k in range(7):
            held += step(bufs[k % 4]) is None
        step.flush()
        torch.cuda.synchronize()
        assert step.state == 'graph' and step.error is None
        if pair:
            # step 0 captures the single graph; steps 1-6 pair up (1, 2), (3, 0), (1, 2)
            assert held == 3 and len(step._groups) == 2 and not step._held
        nets.append(m)
    for b, k in zip(bufs, keep):
        assert torch.equal(b, k)                            # inputs read in place, never written
    lr = 2e-4
    for pa, pb in zip(nets[0].parameters(), nets[1].parameters()):
        d = (pb - pa).detach().abs()
        assert float(d.mean()) < 0.15 * lr


def test_captured_step_group_of_four_steps_trains_like_single_steps(dev):
    """group_steps=4: steps 1-4 run from one graph, steps 5-6 stay held
    until flush() runs them one by one."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(11)
    bufs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
            for _ in range(4)]
    nets = []
    for n in (1, 4):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                            static_inputs=4, group_steps=n, reuse_distance=4)   # bufs are never rewritten
        held = sum(step(bufs[k % 4]) is None for k in range(7))
        if n == 4:
            assert held == 5 and len(step._groups) == 1 and len(step._held) == 2
        step.flush()
        torch.cuda.synchronize()
        assert step.state == 'graph' and step.error is None and not step._held
        nets.append(m)
    lr = 2e-4
    for pa, pb in zip(nets[0].parameters(), nets[1].parameters()):
        assert float((pb - pa).detach().abs().mean()) < 0.15 * lr


def test_captured_step_group_keeps_every_loss_and_guards_held_inputs(dev):
    """group_steps=2: last_losses() holds both steps' losses of a pair replay,
    equal to single steps' losses; an input rewritten in place while held
    (``x.copy_(batch); step(x)``) raises instead of training twice on the
    later data; group_steps above the reuse distance is refused; a pending
    held step runs before state_dict()."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(5)
    bufs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
            for _ in range(2)]
    per_step = {}
    for n in (1, 2):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                            static_inputs=4, group_steps=n)
        got = []
        for k in range(5):
            out = step(bufs[k % 2])
            if out is not None:
                got.extend(float(v) for v in step.last_losses())
        assert step.flush() is None           # 5 steps: capture + two pairs, nothing held
        per_step[n] = got
    assert len(per_step[1]) == len(per_step[2]) == 5, per_step
    torch.testing.assert_close(torch.tensor(per_step[2]), torch.tensor(per_step[1]), rtol=2e-3, atol=1e-4)
    # in-place rewrite of a held input
    torch.manual_seed(0)
    m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    opt = ops.FusedAdam(m.parameters(), lr=2e-4)
    step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                        static_inputs=4, group_steps=2)
    x = bufs[0].clone()
    step(x)                                   # capture + first step
    assert step(x) is None                    # held
    x.copy_(bufs[1])
    with pytest.raises(RuntimeError, match='modified in place'):
        step(x)
    # a held step runs before the checkpoint
    assert step(bufs[0]) is None and step._held
    m.state_dict()
    assert not step._held and len(step.last_losses()) == 1
    with pytest.raises(ValueError, match='reuse distance'):
        CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, static_inputs=4, group_steps=3)


def test_captured_step_never_replays_for_another_layout(dev):
    """A cache hit on the data pointer alone must not replay a graph: a view
    of a captured buffer with another shape (``x[:2]``: same data pointer;
    ``x[2:]``: same storage) runs an eager step -- visible as host-side op calls, which a replay makes
    none of -- and the captured input is never written."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(9)
    buf = torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    keep = buf.clone()
    for static in (0, 2):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        step = CapturedStep(m, opt, lambda mm, x: mm.bce_loss_bf16(x, 1.0), allreduce=False, graph=True,
                            static_inputs=static)
        step(buf)
        step(buf)
        torch.cuda.synchronize()
        assert step.state == 'graph'
        calls = ops.KERNEL_CALLS.get('conv_fwd', 0)
        step(buf)                                           # replay: no host-side op calls
        assert ops.KERNEL_CALLS.get('conv_fwd', 0) == calls
        for x in (buf[:2], buf[2:]):      # same pointer / same storage, other shape
            loss = step(x)
            torch.cuda.synchronize()
            assert ops.KERNEL_CALLS.get('conv_fwd', 0) > calls, 'replayed a graph for another layout'
            calls = ops.KERNEL_CALLS.get('conv_fwd', 0)
            assert bool(torch.isfinite(loss))
        assert torch.equal(buf, keep)                       # the caller's tensor was never written


@pytest.mark.parametrize('N,H,W', [(4, 240, 320), (3, 96, 128)])
def test_head_applies_bn_backward(dev, monkeypatch, N, H, W):
    """The fused head works out the last BN's backward sums in its forward
    (factored through dlogit) and applies that BN's backward itself, so the
    BN's input gradient leaves the head backward and no BN apply launch runs
    (BT_HEAD_BN_BWD): the same loss, and gradients equal to the accumulator
    path's within the rounding of their differently ordered sums."""
    from blendtorch.models import Discriminator
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(12)
    x = torch.rand(N, 3, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    runs = []
    for on in (True, False):
        monkeypatch.setattr(ops, '_HEAD_BN_BWD', on)
        torch.manual_seed(4)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
        m.lazy_head_bn = True
        before = (ops.KERNEL_CALLS.get('bn_backward_by_head', 0), ops.KERNEL_CALLS.get('bn_backward_acc', 0))
        for _ in range(2):   # (the second step reuses the zeroed scratch and accumulators)
            m.zero_grad(set_to_none=True)
            loss = m.bce_loss_bf16(x, 1.0)
            loss.backward()
        torch.cuda.synchronize()
        by_head = ops.KERNEL_CALLS.get('bn_backward_by_head', 0) - before[0]
        assert by_head == (2 if on else 0)
        runs.append((loss.detach().clone(), [p.grad.clone() for p in m.parameters()],
                     [b.clone() for b in m.buffers()]))
    (la, ga, ba), (lb, gb, bb) = runs
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-6)
    for x_, y_ in zip(ba, bb):
        torch.testing.assert_close(x_, y_, rtol=1e-5, atol=1e-6)
    for (n, _), x_, y_ in zip(Discriminator(nc=3, ndf=32, adaptive=True).named_parameters(), ga, gb):
        torch.testing.assert_close(x_, y_, rtol=2e-2, atol=2e-2 * float(y_.abs().max()), msg=n)
    assert int(torch.count_nonzero(ops._head_bn_scratch(dev, N, 256))) == 0   # cleared by the kernel


def _dopt_state(dev, B, N, seed=7):
    from blendtorch.models import ProbModel
    g = torch.Generator(device=dev).manual_seed(seed)
    pm = ProbModel([1.2, 3.0], [0.4, 0.3]).to(dev)
    st = {k: torch.zeros(n, device=dev) for k, n in
          (('stats', 2), ('gate_d', 1), ('gate_s', 1), ('b', 1), ('first', 1), ('params_out', 4), ('red', 5),
           ('adam', 9))}
    st['samples'] = torch.exp(torch.randn(2, N, device=dev, generator=g) * 0.3 + 1.0)
    st['counter'] = torch.zeros(1, dtype=torch.int32, device=dev)
    st['logit_s'] = torch.randn(B, device=dev, generator=g) * 2
    st['logit_real'] = torch.randn(B, device=dev, generator=g) + 1
    st['logit_sim'] = torch.randn(B, device=dev, generator=g) - 1
    st['sid'] = torch.randperm(N, device=dev, generator=g)[:B].to(torch.int64)
    return pm, st


def _dopt_kp(pm, st, B, N, rank=0, world=1, seed=11):
    return dict(samples=st['samples'].data_ptr(), mean=pm.m1m2_mean.data_ptr(), log_std=pm.m1m2_log_std.data_ptr(),
                exp_avg=st['adam'][0:4].data_ptr(), exp_avg_sq=st['adam'][4:8].data_ptr(),
                adam_step=st['adam'][8:9].data_ptr(), lr=5e-2, b1=0.7, b2=0.999, eps=1e-8, b=st['b'].data_ptr(),
                first=st['first'].data_ptr(), gate_s=st['gate_s'].data_ptr(), gate_d=st['gate_d'].data_ptr(),
                stats=st['stats'].data_ptr(), alpha=0.9, threshold=0.7, params_out=st['params_out'].data_ptr(),
                red=st['red'].data_ptr(), counter=st['counter'].data_ptr(), seed=seed, B=B, N=N, rank=rank,
                world=world, logit_s=st['logit_s'].data_ptr(), sid=st['sid'].data_ptr(),
                logit_real=st['logit_real'].data_ptr(), logit_sim=st['logit_sim'].data_ptr())


def test_dopt_kernels_match_reference(dev):
    """the densityopt gate and S step as gfx950 kernels
    (csrc/gpu/dopt.hip) against PyTorch: the D statistics / gate, the
    per-rank means of the fused S step (models.densityopt.sstep_reference,
    itself pinned to ProbModel autograd on the CPU), the gated Adam update
    (FusedAdam's reference arithmetic), baseline / first-step bookkeeping,
    and the Philox resampling: LogNormal moments, bit-identical for the same
    key and counter, a new draw per iteration."""
    from blendtorch.models.densityopt import sstep_reference
    ext = ops.hip_ext()
    st_ = ops._stream(dev)
    B, N = 64, 4096
    pm, st = _dopt_state(dev, B, N)
    st['b'].fill_(0.6)
    st['first'].fill_(1.0)
    kp = _dopt_kp(pm, st, B, N)
    ext.dopt_gate(kp, 0, st_)
    torch.cuda.synchronize()
    dr, ds = torch.sigmoid(st['logit_real']).mean(), torch.sigmoid(st['logit_sim']).mean()
    torch.testing.assert_close(st['stats'], torch.stack([dr, ds]), rtol=1e-5, atol=1e-6)
    assert float(st['gate_d']) == float(dr - ds < 0.7)
    st['gate_d'].fill_(0.0)                      # separated: the first S step runs (gate_s 1)
    ref = sstep_reference(st['logit_s'], st['sid'], st['samples'], pm.m1m2_mean.detach().clone(),
                          pm.m1m2_log_std.detach().clone(), 0.6)
    ext.dopt_sstep(kp, 1, st_)                   # phase 1: the means only
    torch.cuda.synchronize()
    torch.testing.assert_close(st['red'], ref, rtol=2e-5, atol=2e-6)
    p0 = torch.cat([pm.m1m2_mean.detach(), pm.m1m2_log_std.detach()]).clone()
    old = st['samples'].clone()
    ext.dopt_sstep(kp, 0, st_)                   # the whole step
    torch.cuda.synchronize()
    assert float(st['gate_s']) == 1.0 and float(st['first']) == 0.0 and float(st['adam'][8]) == 1.0
    torch.testing.assert_close(st['b'], ref[0:1], rtol=2e-5, atol=2e-6)   # first step: b = err mean
    # Adam, step 1: m = 0.3 g, v = 0.001 g^2 -> p -= lr / 0.3 * m / (sqrt(v) / sqrt(0.001) + eps)
    g = ref[1:5]
    m, v = 0.3 * g, 0.001 * g * g
    want = p0 - (5e-2 / 0.3) * m / (v.sqrt() / (0.001 ** 0.5) + 1e-8)
    got = torch.cat([pm.m1m2_mean.detach(), pm.m1m2_log_std.detach()])
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st['params_out'], torch.cat([got[:2], got[2:].exp()]), rtol=1e-6, atol=1e-6)
    # the new samples: LogNormal(mu, s) moments over N draws, a fresh draw (counter advanced)
    assert int(st['counter']) == 1 and not torch.equal(st['samples'], old)
    ls = st['samples'].log()
    torch.testing.assert_close(ls.mean(1), got[:2], rtol=0, atol=4 * float(got[2:].exp().max()) / N ** 0.5)
    torch.testing.assert_close(ls.std(1), got[2:].exp(), rtol=0.05, atol=0)
    # the same key and counter draw the same samples (every rank of a data-parallel run)
    _, st2 = _dopt_state(dev, B, N)
    st2['counter'].fill_(0)
    kp2 = _dopt_kp(pm, st2, B, N)
    ext.dopt_sstep(kp2, 3, st_)                  # phase 3: samples only, at the parameters now
    ext.dopt_sstep(kp2, 3, st_)
    st3 = dict(st2, counter=torch.ones(1, dtype=torch.int32, device=dev), samples=torch.empty_like(st2['samples']))
    ext.dopt_sstep(_dopt_kp(pm, st3, B, N), 3, st_)
    torch.cuda.synchronize()
    assert torch.equal(st3['samples'], st2['samples'])    # counter 1 in both
    # a skipped S step (not first, gate_s from gate_d = 1 and first = 1 -> 0): nothing moves but the samples
    st['first'].fill_(1.0)
    st['gate_d'].fill_(1.0)
    before = (got.clone(), st['b'].clone(), st['adam'].clone())
    ext.dopt_sstep(kp, 0, st_)
    torch.cuda.synchronize()
    assert float(st['gate_s']) == 0.0
    assert torch.equal(torch.cat([pm.m1m2_mean.detach(), pm.m1m2_log_std.detach()]), before[0])
    assert torch.equal(st['b'], before[1]) and torch.equal(st['adam'], before[2])


def test_densityopt_fused_host_state_and_static_sims(dev):
    """The fused DensityOptStep: sim batches read in place from a fixed ring of
    buffers (one sim-half graph each, no copy), shape ids from host-mapped
    memory, results in host-mapped memory (host_state) equal to the device
    tensors, and the same run twice is bit-identical (fixed-order sums, Philox
    sampler keyed by the seed)."""
    from blendtorch.models import Discriminator, ProbModel
    from blendtorch.models.densityopt import DensityOptStep
    B = 64
    runs = []
    for _ in range(2):
        torch.manual_seed(0)
        netD = Discriminator().to(dev).to(memory_format=torch.channels_last)
        pm = ProbModel([1.2, 3.0], [0.4, 0.4]).to(dev)
        g = torch.Generator(device=dev).manual_seed(2)
        ring = [(torch.rand(B, 64, 64, 4, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) for _ in range(3)]
        step = DensityOptStep(netD, pm, ring[0].permute(0, 3, 1, 2).clone(), B, graph=True, warmup=2, seed=5)
        assert step.fused
        step.start()
        torch.cuda.synchronize()
        assert torch.equal(step.host_state()['samples'], step.samples[:, :B].cpu())
        sids = torch.Generator().manual_seed(4)
        hist = []
        adds0 = ops.KERNEL_CALLS.get('grad_dest_autograd_add', 0)
        for i in range(8):
            step(ring[i % 3].permute(0, 3, 1, 2), torch.randperm(B, generator=sids))
            torch.cuda.synchronize()
            hs = step.host_state()
            assert torch.equal(hs['samples'], step.samples[:, :B].cpu())
            assert torch.equal(hs['params'], step.params_out.cpu())
            assert torch.equal(hs['stats'], step.stats.cpu())
            assert float(hs['gate_d']) == float(step.gate_d) and float(hs['gate_s']) == float(step.gate_s)
            hist.append(hs['params'].clone())
        assert step.graph is not None and 'copy' not in step._sims and len(step._sims) == 3
        # every capture (the real half, one sim half per ring buffer) writes the bucket views:
        # no gradient of the D step goes through an autograd add
        assert ops.KERNEL_CALLS.get('grad_dest_autograd_add', 0) == adds0
        assert bool(torch.isfinite(step.samples).all()) and bool((step.samples > 0).all())
        runs.append((torch.stack(hist), [p.detach().clone() for p in netD.parameters()]))
    assert torch.equal(runs[0][0], runs[1][0])
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)


def test_second_gradient_sinks_match_autograd_accumulate(dev):
    """GradBuckets(second_sinks=True): two backward passes before one
    FusedAdam step (densityopt's real / sim halves).  The second pass writes
    its gradients into the second bucket views and the update kernel adds
    them -- no AccumulateGrad launches -- and the weights after the step are
    bit-identical to autograd adding the second gradients into .grad."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel import GradBuckets
    torch.manual_seed(3)
    g = torch.Generator(device=dev).manual_seed(4)
    xa = (torch.rand(16, 64, 64, 4, device=dev, generator=g) * 2 - 1).to(torch.bfloat16).permute(0, 3, 1, 2)
    xb = (torch.rand(16, 64, 64, 4, device=dev, generator=g) * 2 - 1).to(torch.bfloat16).permute(0, 3, 1, 2)
    nets, adds = [], []
    base = Discriminator().to(dev).to(memory_format=torch.channels_last)
    for second in (False, True):
        net = Discriminator().to(dev).to(memory_format=torch.channels_last)
        net.load_state_dict(base.state_dict())
        gb = GradBuckets(net.parameters(), second_sinks=second)
        opt = ops.FusedAdam(net.parameters(), lr=1e-3, betas=(0.5, 0.999))
        opt.set_zero_grads(True)
        adds0 = ops.KERNEL_CALLS.get('grad_dest_autograd_add', 0)
        for _ in range(3):
            gb.zero_()
            la, _ = net.bce_bf16(xa, 1.0)
            la.backward()
            lb, _ = net.bce_bf16(xb, 0.0)
            lb.backward()
            opt.step()
        torch.cuda.synchronize()
        nets.append(net)
        adds.append((sum(1 for p in net.parameters() if getattr(p, '_bt_grad_second', False)),
                     ops.KERNEL_CALLS.get('grad_dest_autograd_add', 0) - adds0))
    n = len(list(nets[1].parameters()))
    assert adds[0] == (0, 3 * n) and adds[1] == (n, 0), adds
    for (n, pa), pb in zip(nets[0].named_parameters(), nets[1].parameters()):
        assert torch.equal(pa, pb), n
