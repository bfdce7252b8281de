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
