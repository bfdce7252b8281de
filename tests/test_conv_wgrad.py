"""gfx950 MFMA weight gradient of the 4x4/s2/p1 convolution (csrc/gpu/conv.hip)
against the fp32 PyTorch reference (torch.nn.grad.conv2d_weight on the same
bf16 inputs), and the discriminator's backward with it."""
import pytest
import torch

from blendtorch import ops


def test_supported_is_false_off_gpu():
    x = torch.zeros(1, 32, 8, 8, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    assert not ops.conv_wgrad_supported(x, torch.zeros(64, 32, 4, 4))


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    ops.hip_ext()
    return torch.device('cuda', 0)


def _ref(x, dy, cout):
    return torch.nn.grad.conv2d_weight(x.float(), (cout, x.shape[1], 4, 4), dy.float(), stride=2, padding=1)


@pytest.fixture(params=['plain', 'pipe', 'wide', 'co128'])
def wgrad_pipe(request):
    """Register-staged weight gradient: plain, fragments read a step ahead of the MFMAs
    (pipe), 256-column tiles (wide; layers with Cin >= 16, plain dY), or 128-channel
    tiles (co128; layers with Cout % 128 == 0, plain dY)."""
    ops.hip_ext().conv_set_wgrad_pipe(1 if request.param == 'pipe' else 0)
    ops.hip_ext().conv_set_wgrad_wide(1 if request.param == 'wide' else 0)
    ops.hip_ext().conv_set_wgrad_co128(1 if request.param == 'co128' else 0)
    yield request.param
    ops.hip_ext().conv_set_wgrad_pipe(-1)
    ops.hip_ext().conv_set_wgrad_wide(-1)
    ops.hip_ext().conv_set_wgrad_co128(-1)


@pytest.fixture(params=[0, 2, 3], ids=lambda s: f'staging{s}')
def wgrad_staging(request):
    """Weight-gradient staging: register ring (0) or LDS-DMA stages of 64
    pixels (2, 3; layers with Wo >= 32 -- narrower ones take the register ring)."""
    ops.hip_ext().conv_set_wgrad_staging(request.param)
    yield request.param
    ops.hip_ext().conv_set_wgrad_staging(-1)


@pytest.mark.gpu
@pytest.mark.parametrize('N,Cin,H,W,Cout', [(2, 32, 30, 40, 64), (2, 64, 16, 20, 128), (1, 128, 8, 10, 256),
                                            (3, 32, 14, 18, 64), (8, 32, 240, 320, 64), (2, 64, 60, 80, 128),
                                            (1, 128, 60, 64, 256), (3, 32, 10, 66, 64)])
@pytest.mark.parametrize('layout', ['channels_last', 'contiguous'])
def test_wgrad_matches_fp32_reference(dev, N, Cin, H, W, Cout, layout, wgrad_staging, wgrad_pipe):
    g = torch.Generator(device=dev).manual_seed(N * Cin + H)
    cl = torch.channels_last
    x = torch.randn(N, Cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(N, Cout, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    out = torch.full((Cout, Cin, 4, 4), float('nan'), device=dev)
    if layout == 'channels_last':
        out = out.contiguous(memory_format=cl)
    before = ops.KERNEL_CALLS.get('conv_wgrad', 0)
    ops.conv_wgrad(x, dy, out)
    assert ops.KERNEL_CALLS['conv_wgrad'] == before + 1
    ref = _ref(x, dy, Cout)
    scale = float(ref.abs().max())
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-4 * scale)


@pytest.mark.gpu
@pytest.mark.parametrize('ordered', [1, 0], ids=['ordered', 'atomic'])
@pytest.mark.parametrize('N,Cin,H,W,Cout', [(8, 4, 480, 640, 32), (8, 32, 240, 320, 64), (8, 64, 120, 160, 128),
                                            (1, 128, 60, 64, 256), (3, 32, 10, 66, 64)])
def test_wgrad_slice_reduce_modes(dev, N, Cin, H, W, Cout, ordered):
    """Both slice reduces (ordered, the default: bit-identical run to run;
    atomic groups: BT_WGRAD_ORDERED=0) against the fp32 reference, over the
    disc step's slice counts (first layer: 512 slices, 32 lanes per element
    group), and the ordered one twice for bit-identity."""
    g = torch.Generator(device=dev).manual_seed(Cin + W)
    cl = torch.channels_last
    x = torch.randn(N, Cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(N, Cout, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    ops.hip_ext().conv_set_wgrad_ordered(ordered)
    try:
        outs = [ops.conv_wgrad(x, dy, torch.full((Cout, Cin, 4, 4), float('nan'), device=dev)) for _ in range(2)]
    finally:
        ops.hip_ext().conv_set_wgrad_ordered(-1)
    ref = _ref(x, dy, Cout)
    torch.testing.assert_close(outs[0], ref, rtol=1e-3, atol=1e-4 * float(ref.abs().max()))
    if ordered:
        assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
def test_wgrad_asymmetric_operands(dev, wgrad_staging, wgrad_pipe):
    """Structured (non-random) operands: a transposed or mis-swizzled tile
    cannot pass by symmetry."""
    cl = torch.channels_last
    N, Cin, H, W, Cout = 1, 32, 8, 64, 64
    x = torch.zeros(N, Cin, H, W, device=dev)
    x[0, :, :, :] = (torch.arange(Cin, device=dev).view(Cin, 1, 1) * 0.01 +
                     torch.arange(W, device=dev).view(1, 1, W) * 0.001)
    x[0, 5, 3, 7] = 1.0
    dy = torch.zeros(N, Cout, H // 2, W // 2, device=dev)
    dy[0, 17, 2, 4] = 1.0
    dy[0, 40, 1, 30] = -2.0
    x, dy = x.to(torch.bfloat16).contiguous(memory_format=cl), dy.to(torch.bfloat16).contiguous(memory_format=cl)
    out = ops.conv_wgrad(x, dy, torch.empty(Cout, Cin, 4, 4, device=dev))
    torch.testing.assert_close(out, _ref(x, dy, Cout), rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
def test_discriminator_backward_with_mfma_convs(dev):
    """The bf16 discriminator with the MFMA convs (forward + fp32 weight
    gradient) against the same stack on MIOpen, both measured against an fp32
    model with the same weights: ours must be at least as close to fp32."""
    from blendtorch.models import Discriminator
    torch.manual_seed(0)
    nets = [Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
            for _ in range(3)]
    for n in nets[1:]:
        n.load_state_dict(nets[0].state_dict())
    x = torch.rand(4, 3, 240, 320, device=dev).contiguous(memory_format=torch.channels_last)
    before = ops.KERNEL_CALLS.get('conv_wgrad', 0)
    def stats_bns():   # BN calls that took the convolution epilogue's sums (applied, or lazily by a consumer)
        return (ops.KERNEL_CALLS.get('bn_forward_from_stats', 0) + ops.KERNEL_CALLS.get('bn_forward_lazy', 0)
                + ops.KERNEL_CALLS.get('bn_forward_by_producer', 0))
    bn_before = stats_bns()
    nets[0].forward_bf16(x.to(torch.bfloat16), mfma=True).float().sum().backward()
    assert ops.KERNEL_CALLS['conv_wgrad'] == before + 3          # conv 2, 3 and 4 (conv 1 has Cin = 3)
    assert stats_bns() == bn_before + 3   # their BNs take the epilogue sums
    nets[1].forward_bf16(x.to(torch.bfloat16), mfma=False).float().sum().backward()
    nets[2](x).sum().backward()                                   # fp32 reference
    for (n, pa), pb, pr in zip(nets[0].named_parameters(), nets[1].parameters(), nets[2].parameters()):
        r = pr.grad.flatten().double()

        def cos(g):
            g = g.flatten().double()
            return float(g @ r / (g.norm() * r.norm()))
        ca, cb = cos(pa.grad), cos(pb.grad)
        print(n, f'cos(mfma, fp32)={ca:.6f} cos(miopen, fp32)={cb:.6f}')
        assert ca > 0.99 and ca >= cb - 2e-3, n
    for ma, mb in zip(nets[0].modules(), nets[1].modules()):
        if isinstance(ma, ops.BatchNormLeakyReLU2d):
            assert int(ma.num_batches_tracked) == int(mb.num_batches_tracked) == 1
            torch.testing.assert_close(ma.running_mean, mb.running_mean, rtol=2e-2, atol=1e-4)
            torch.testing.assert_close(ma.running_var, mb.running_var, rtol=2e-2, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize('N,Cin,H,W,Cout', [(2, 32, 30, 40, 64), (2, 64, 16, 20, 128), (1, 128, 8, 10, 256),
                                            (3, 32, 14, 18, 64), (8, 32, 240, 320, 64), (2, 8, 12, 16, 64),
                                            (2, 16, 20, 24, 32), (1, 64, 6, 10, 96)])
def test_forward_matches_fp32_reference_and_stats(dev, N, Cin, H, W, Cout):
    import torch.nn.functional as F
    g = torch.Generator(device=dev).manual_seed(N + Cin + W)
    cl = torch.channels_last
    x = torch.randn(N, Cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.1 * torch.randn(Cout, Cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    M = N * (H // 2) * (W // 2)
    rows = ops.conv_fwd_stats_rows(M, Cout)
    stats = torch.full((rows * 2 * Cout,), float('nan'), device=dev)
    y = ops.conv_fwd(x, w, stats)
    ref = F.conv2d(x.float(), w.float(), None, 2, 1)
    assert y.is_contiguous(memory_format=cl) and y.dtype == torch.bfloat16
    # fp32 accumulation, one bf16 rounding: within one bf16 ulp of the fp32 result
    torch.testing.assert_close(y.float(), ref, rtol=2 ** -7, atol=1e-3 * float(ref.abs().max()))
    st = stats.view(2, Cout, rows).sum(-1)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, Cout)
    torch.testing.assert_close(st[0], yf.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(st[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize('N,Cin,H,W,Cout', [(2, 64, 30, 40, 64), (2, 64, 16, 20, 128), (1, 128, 8, 10, 256),
                                            (3, 64, 14, 18, 32), (8, 64, 120, 160, 128), (2, 128, 12, 16, 16),
                                            (8, 32, 240, 320, 64), (2, 32, 10, 12, 64)])
def test_dgrad_matches_fp32_reference(dev, N, Cin, H, W, Cout):
    g = torch.Generator(device=dev).manual_seed(N * 7 + Cin + W)
    cl = torch.channels_last
    w = (0.1 * torch.randn(Cout, Cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(N, Cout, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    before = ops.KERNEL_CALLS.get('conv_dgrad', 0)
    dx = ops.conv_dgrad(dy, w, (N, Cin, H, W))
    assert ops.KERNEL_CALLS['conv_dgrad'] == before + 1
    ref = torch.nn.grad.conv2d_input((N, Cin, H, W), w.float(), dy.float(), stride=2, padding=1)
    assert dx.is_contiguous(memory_format=cl) and dx.dtype == torch.bfloat16
    torch.testing.assert_close(dx.float(), ref, rtol=2 ** -7, atol=1e-3 * float(ref.abs().max()))


@pytest.fixture(params=[1, 0], ids=['c4wave', 'c4block'])
def c4_staging(request):
    """First-layer weight gradient: wave-private (1, default) or block-shared (0) staging."""
    ops.hip_ext().conv_set_c4_wave_private(request.param)
    yield request.param
    ops.hip_ext().conv_set_c4_wave_private(-1)


@pytest.mark.gpu
@pytest.mark.parametrize('N,H,W', [(2, 30, 40), (8, 480, 640), (3, 14, 18)])
def test_first_layer_rgba_forward_and_wgrad(dev, N, H, W, c4_staging):
    """RGBA-decoded frames into an RGB first layer: the 4-channel MFMA paths
    ignore the alpha channel (weight 0) and produce the 3-channel gradient."""
    import torch.nn.functional as F
    g = torch.Generator(device=dev).manual_seed(H + W)
    cl = torch.channels_last
    x = torch.rand(N, 4, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.1 * torch.randn(32, 3, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    rows = ops.conv_fwd_stats_rows(N * (H // 2) * (W // 2), 32)
    stats = torch.empty(rows * 2 * 32, device=dev)
    y = ops.conv_fwd(x, w, stats)
    ref = F.conv2d(x[:, :3].float(), w.float(), None, 2, 1)
    torch.testing.assert_close(y.float(), ref, rtol=2 ** -7, atol=1e-3 * float(ref.abs().max()))
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 32)
    torch.testing.assert_close(stats.view(2, 32, rows).sum(-1)[0], yf.sum(0), rtol=1e-4, atol=1e-3)
    dy = torch.randn(N, 32, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    for layout in (torch.contiguous_format, cl):
        out = torch.full((32, 3, 4, 4), float('nan'), device=dev).contiguous(memory_format=layout)
        ops.conv_wgrad(x, dy, out)
        wref = torch.nn.grad.conv2d_weight(x[:, :3].float(), (32, 3, 4, 4), dy.float(), stride=2, padding=1)
        torch.testing.assert_close(out, wref, rtol=1e-3, atol=1e-4 * float(wref.abs().max()))


@pytest.mark.gpu
def test_discriminator_rgba_input_equals_rgb(dev):
    from blendtorch.models import Discriminator
    torch.manual_seed(0)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x4 = torch.rand(4, 4, 120, 160, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x3 = x4[:, :3].contiguous(memory_format=torch.channels_last)
    before = ops.KERNEL_CALLS.get('conv_wgrad', 0)
    la = a.bce_loss_bf16(x4, 1.0)
    la.backward()
    assert ops.KERNEL_CALLS['conv_wgrad'] == before + 4          # all four 4x4/s2 layers on the MFMA path
    lb = b.bce_loss_bf16(x3, 1.0)
    lb.backward()
    torch.testing.assert_close(la, lb, rtol=1e-2, atol=1e-4)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        ga, gb = pa.grad.flatten().double(), pb.grad.flatten().double()
        assert float(ga @ gb / (ga.norm() * gb.norm())) > 0.99, n


@pytest.mark.gpu
def test_bn_backward_sums_from_dgrad_epilogue(dev, monkeypatch):
    """A BN+LeakyReLU whose output feeds an MFMA conv takes its backward sums
    from that conv's data-gradient epilogue (BnLink): same gradients as the
    separate reduction pass, on the bench's RGBA-fed layer stack."""
    from blendtorch.models import Discriminator
    torch.manual_seed(3)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 4, 96, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    before = ops.KERNEL_CALLS.get('bn_backward_from_stats', 0)
    head0 = ops.KERNEL_CALLS.get('bn_backward_by_head', 0)
    a.bce_loss_bf16(x, 1.0).backward()
    # BN1..BN3 feed conv2..conv4, BN4 the fused head: all four take their sums from the consumer
    # (BN4's: worked out by the head forward, which then applies its backward -- BT_HEAD_BN_BWD)
    by_head = ops.KERNEL_CALLS.get('bn_backward_by_head', 0) - head0
    after = ops.KERNEL_CALLS.get('bn_backward_from_stats', 0)
    assert after - before + by_head == 4
    monkeypatch.setattr(ops.BnLink, 'ready', lambda self, dx: False)
    b.bce_loss_bf16(x, 1.0).backward()
    assert ops.KERNEL_CALLS.get('bn_backward_from_stats', 0) == after
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=2e-2, atol=2e-2 * float(pb.grad.abs().max()), msg=n)


@pytest.fixture
def tiles(request):
    ops.conv_set_tiles(*request.param)
    yield request.param
    ops.conv_set_tiles(0, 0, -1, 0)


@pytest.mark.gpu
@pytest.mark.parametrize('tiles', [(bm, bn, st, 0) for st in (0, 2, 3, 4) for bm in (64, 128) for bn in (32, 64, 128)]
                         + [(bm, bn, 2, cls) for cls in (1, 4) for bm in (64, 128) for bn in (32, 64)],
                         indirect=True, ids=lambda t: f'bm{t[0]}_bn{t[1]}_st{t[2]}_cls{t[3]}')
def test_tap_gemm_tile_variants(dev, tiles):
    """Every tile shape of the tap-gather GEMM (pixels x output channels),
    staging (register ring, 2 or 3 LDS-DMA stages) and data-gradient parity
    classes per block (1, 4; 0 = automatic) against the fp32 reference:
    forward with statistics, data gradient, and the data gradient with the
    BN-backward epilogue (Discriminator backward)."""
    import torch.nn.functional as F
    from blendtorch.models import Discriminator
    bm, bn = tiles[0], tiles[1]
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(bm + bn)
    for N, Cin, H, W, Cout in [(2, 64, 30, 40, 128), (1, 128, 8, 10, 256), (3, 32, 14, 18, 64)]:
        x = torch.randn(N, Cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
        w = (0.1 * torch.randn(Cout, Cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
        M = N * (H // 2) * (W // 2)
        rows = ops.conv_fwd_stats_rows(M, Cout)
        stats = torch.full((rows * 2 * Cout,), float('nan'), device=dev)
        y = ops.conv_fwd(x, w, stats)
        ref = F.conv2d(x.float(), w.float(), None, 2, 1)
        torch.testing.assert_close(y.float(), ref, rtol=2 ** -7, atol=1e-3 * float(ref.abs().max()))
        yf = y.float().permute(0, 2, 3, 1).reshape(-1, Cout)
        st = stats.view(2, Cout, rows).sum(-1)
        torch.testing.assert_close(st[0], yf.sum(0), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(st[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
        dy = torch.randn(N, Cout, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
        dx = ops.conv_dgrad(dy, w, (N, Cin, H, W))
        dref = torch.nn.grad.conv2d_input((N, Cin, H, W), w.float(), dy.float(), stride=2, padding=1)
        torch.testing.assert_close(dx.float(), dref, rtol=2 ** -7, atol=1e-3 * float(dref.abs().max()))
    torch.manual_seed(5)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    xin = torch.rand(4, 4, 96, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    a.bce_loss_bf16(xin, 1.0).backward()
    got = [p.grad.clone() for p in a.parameters()]
    ops.conv_set_tiles(0, 0, 0, 1)  # reference: default tiles, register staging, one class per block
    a.zero_grad(set_to_none=True)
    a.bce_loss_bf16(xin, 1.0).backward()
    for (n, p), g0 in zip(a.named_parameters(), got):
        torch.testing.assert_close(g0, p.grad, rtol=2e-2, atol=2e-2 * float(p.grad.abs().max()), msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize('side', [False, True])
def test_bn_accumulators_fold_and_clear(dev, monkeypatch, side):
    """Accumulator hand-off (BnAccumulator): the conv epilogues add BN sums
    into zeroed accumulators that the apply kernels fold and clear -- same
    loss, gradients and running statistics as the partial-row + finalize
    path, over several steps, and every accumulator is zero after each step.
    In line, the weight-gradient launches fold BN1..3's backward sums; with
    the weight gradients on the side stream the BN applies fold them."""
    from blendtorch.models import Discriminator
    monkeypatch.setattr(ops, '_SIDE_WGRAD', side)
    torch.manual_seed(7)
    cl = torch.channels_last
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    for m in (a, b):   # the apply kernels' path (the BN applies moved into their neighbours:
        m.lazy_head_bn = m.lazy_conv_bn = m.defer_bn_bwd = False   # test_lazy_bn_applies_match_apply_pass)
        m.conv_out_bn = False   # (or into their producers: test_conv_applies_its_output_bn)
    x = torch.rand(4, 4, 96, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    acc_supported = ops.bn_acc_supported
    for step in range(3):
        a.zero_grad(set_to_none=True)
        b.zero_grad(set_to_none=True)
        before = (ops.KERNEL_CALLS.get('bn_forward_acc', 0), ops.KERNEL_CALLS.get('bn_backward_acc', 0),
                  ops.KERNEL_CALLS.get('bn_backward_folded', 0), ops.KERNEL_CALLS.get('conv_dgrad_held', 0))
        la = a.bce_loss_bf16(x, 1.0)
        la.backward()
        held = ops.KERNEL_CALLS.get('conv_dgrad_held', 0) - before[3]   # data gradients sharing a launch
        # 4 BN layers forward; backward: BN1..3 from the dgrad epilogues, BN4 from the head's
        assert ops.KERNEL_CALLS['bn_forward_acc'] == before[0] + 4
        assert ops.KERNEL_CALLS['bn_backward_acc'] == before[1] + 4
        # BN1..3's sums are folded by the next conv's weight-gradient launch (in line), unless
        # that launch also runs the data gradient filling them (held: the apply folds them)
        assert ops.KERNEL_CALLS.get('bn_backward_folded', 0) == before[2] + (0 if side else 3 - held)
        monkeypatch.setattr(ops, 'bn_acc_supported', lambda C: False)
        lb = b.bce_loss_bf16(x, 1.0)
        lb.backward()
        monkeypatch.setattr(ops, 'bn_acc_supported', acc_supported)
        torch.testing.assert_close(la, lb, rtol=1e-3, atol=1e-4)
        for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
            torch.testing.assert_close(pa.grad, pb.grad, rtol=2e-2, atol=2e-2 * float(pb.grad.abs().max()), msg=n)
        for ma, mb in zip(a.modules(), b.modules()):
            if isinstance(ma, ops.BatchNormLeakyReLU2d):
                torch.testing.assert_close(ma.running_mean, mb.running_mean, rtol=1e-3, atol=1e-5)
                torch.testing.assert_close(ma.running_var, mb.running_var, rtol=1e-3, atol=1e-5)
                assert int(ma.num_batches_tracked) == int(mb.num_batches_tracked) == step + 1
                for acc in ma.__dict__['_bt_acc_ring'][0]:
                    assert int(torch.count_nonzero(acc.fwd)) == 0 and int(torch.count_nonzero(acc.bwd)) == 0


@pytest.mark.gpu
def test_wgrad_chain_defers_slice_reduces(dev):
    """With bucketed gradients the MFMA weight gradients hand their slice
    reduce to the next layer's launch (3 side reduces, one reduce launch in
    all): same gradients as the unchained per-layer reduces."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.grads import GradBuckets
    torch.manual_seed(11)
    cl = torch.channels_last
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 4, 96, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    gb = GradBuckets(a.parameters())
    gb.zero_()
    before = ops.KERNEL_CALLS.get('conv_wgrad_side_reduce', 0)
    a.bce_loss_bf16(x, 1.0).backward()
    assert ops.KERNEL_CALLS.get('conv_wgrad_side_reduce', 0) == before + 3
    b.bce_loss_bf16(x, 1.0).backward()                      # plain .grad tensors: no chaining
    assert ops.KERNEL_CALLS.get('conv_wgrad_side_reduce', 0) == before + 3
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()), msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize('rows', [1, 2, 4])
@pytest.mark.parametrize('bn', [False, True])
def test_first_layer_wgrad_from_decoded_patch(dev, rows, bn):
    """conv_wgrad_c4p_kernel (bands of output rows, the input decoded once into
    LDS, B fragments read from it): against fp32 PyTorch on the decoded frames
    and against the wave-private kernel, with and without the BN1 backward
    applied to dY while it is staged."""
    cl = torch.channels_last
    ext = ops.hip_ext()
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(11)
    N, H, W, C = 3, 96, 128, 32
    raw = torch.randint(0, 256, (N, H, W, 4), dtype=torch.uint8, device=dev, generator=g)
    xu8 = raw.permute(0, 3, 1, 2)
    xdec = ops.decode(raw, cfg).permute(0, 3, 1, 2)
    lut = ops.decode_lut_bf16(cfg, dev)
    dy = (torch.randn(N, C, H // 2, W // 2, device=dev, generator=g) * 0.1).to(torch.bfloat16).contiguous(memory_format=cl)
    bnd = None
    if bn:
        y = torch.randn(N, H // 2, W // 2, C, device=dev, generator=g).to(torch.bfloat16)
        mean = torch.randn(C, device=dev, generator=g) * 0.1
        invstd = torch.rand(C, device=dev, generator=g) + 0.5
        bw = torch.rand(C, device=dev, generator=g) + 0.5
        bb = torch.randn(C, device=dev, generator=g) * 0.1
        dws = torch.randn(C, device=dev, generator=g) * 10
        dbs = torch.randn(C, device=dev, generator=g) * 10
        bnd = (y, mean, invstd, bw, bb, dws, dbs, 0.2)
    try:
        ext.conv_set_c4p_rows(rows)
        assert ext.conv_c4p_rows(N, H, W, H // 2, W // 2, C) == rows
        got = ops.conv_wgrad(xu8, dy, torch.empty(C, 3, 4, 4, device=dev), lut=lut, bn_dy=bnd)
        ext.conv_set_c4p_rows(0)
        assert ext.conv_c4p_rows(N, H, W, H // 2, W // 2, C) == 0
        wave = ops.conv_wgrad(xu8, dy, torch.empty(C, 3, 4, 4, device=dev), lut=lut, bn_dy=bnd)
    finally:
        ext.conv_set_c4p_rows(-1)
    if bn:   # the BN backward's gx in fp32, rounded to bf16 as the kernels stage it
        yf = y.float().permute(0, 3, 1, 2)
        xh = (yf - mean.view(1, -1, 1, 1)) * invstd.view(1, -1, 1, 1)
        z = xh * bw.view(1, -1, 1, 1) + bb.view(1, -1, 1, 1)
        gz = torch.where(z > 0, dy.float(), dy.float() * 0.2)
        M = N * (H // 2) * (W // 2)
        gx = bw.view(1, -1, 1, 1) * invstd.view(1, -1, 1, 1) * (gz - dbs.view(1, -1, 1, 1) / M
                                                             - xh * dws.view(1, -1, 1, 1) / M)
        dyr = gx.to(torch.bfloat16).float()
    else:
        dyr = dy.float()
    ref = torch.nn.grad.conv2d_weight(xdec.float()[:, :3], (C, 3, 4, 4), dyr, stride=2, padding=1)
    torch.testing.assert_close(got, ref, rtol=1e-3, atol=2e-3 * float(ref.abs().max()))
    # the same bf16 operands summed in another order: equal to fp32 rounding
    torch.testing.assert_close(got, wave, rtol=1e-4, atol=1e-4 * float(wave.abs().max()))


@pytest.mark.gpu
def test_first_layer_reads_raw_u8_frames_through_decode_table(dev, c4_staging):
    """Decode fused into the first convolution: raw u8 RGBA frames through the
    bf16 decode table give bit-identical forward outputs and weight gradients
    to ops.decode -> bf16 NHWC -> the same layer; and the whole disc step
    (bce_loss_bf16(decode=)) matches the decode-first step."""
    from blendtorch.models import Discriminator
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(4)
    raw = torch.randint(0, 256, (3, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g)
    xu8 = raw.permute(0, 3, 1, 2)                         # [N, 4, H, W], NHWC bytes
    xdec = ops.decode(raw, cfg).permute(0, 3, 1, 2)       # bf16 NHWC as [N, 4, H, W]
    lut = ops.decode_lut_bf16(cfg, dev)
    w = (0.1 * torch.randn(32, 3, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    ya = ops.conv_fwd(xu8, w, lut=lut)
    yb = ops.conv_fwd(xdec, w)
    assert torch.equal(ya, yb)
    dy = torch.randn(3, 32, 48, 64, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    oa = ops.conv_wgrad(xu8, dy, torch.empty(32, 3, 4, 4, device=dev), lut=lut)
    ob = ops.conv_wgrad(xdec, dy, torch.empty(32, 3, 4, 4, device=dev))
    # slice groups add with float atomics: equal up to the adds' order
    torch.testing.assert_close(oa, ob, rtol=1e-4, atol=1e-4 * float(ob.abs().max()))
    torch.manual_seed(2)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    la = a.bce_loss_bf16(xu8, 1.0, decode=cfg)
    lb = b.bce_loss_bf16(xdec, 1.0)
    # (the two first layers sum the BN statistics' fp32 partials over different pixel groups --
    # and the u8 one applies its BN itself, test_first_layer_applies_its_bn: mean / invstd may
    # differ in the last float bit, which flips some bf16 roundings downstream)
    torch.testing.assert_close(la, lb, rtol=2e-3, atol=1e-5)
    la.backward()
    lb.backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        ga, gb = pa.grad.flatten().double(), pb.grad.flatten().double()
        assert float(ga @ gb / (ga.norm() * gb.norm())) > 0.999, n


@pytest.mark.gpu
def test_wgrad_chain_with_frozen_first_layer(dev):
    """A frozen first layer (no weight gradient, no input gradient: no
    backward node) must not strand the reduces handed down the chain: the
    chain closes at the first layer that does take a weight gradient."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.grads import GradBuckets
    torch.manual_seed(12)
    cl = torch.channels_last
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        m.features[0].weight.requires_grad_(False)
    x = torch.rand(4, 4, 96, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    gb = GradBuckets([p for p in a.parameters() if p.requires_grad])
    gb.zero_()
    a.bce_loss_bf16(x, 1.0).backward()
    b.bce_loss_bf16(x, 1.0).backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        if pa.requires_grad:
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()),
                                       msg=n)


@pytest.mark.gpu
def test_first_bn_backward_deferred_into_first_wgrad(dev, c4_staging):
    """With raw u8 frames the first BN's backward apply runs inside the first
    convolution's weight-gradient kernel (ops.BnDeferred): its dY operand is
    gx computed from the BN input and output gradient while staging, with the
    same formula and bf16 rounding as bn_bwd_apply.  Every gradient matches
    the step with the separate apply launch (the slice reduce adds with float
    atomics: equal up to the order of those adds), and the apply launch is
    gone."""
    from blendtorch.models import Discriminator
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(21)
    xu8 = torch.randint(0, 256, (4, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g).permute(0, 3, 1, 2)
    torch.manual_seed(3)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    a.defer_bn_bwd = False                      # only the first BN hands its backward on
    b.defer_first_bn = b.defer_bn_bwd = False   # none
    d0 = ops.KERNEL_CALLS.get('bn_backward_deferred_fold', 0)
    w0 = ops.KERNEL_CALLS.get('conv_wgrad_bn_dy', 0)
    la = a.bce_loss_bf16(xu8, 1.0, decode=cfg)
    la.backward()
    assert ops.KERNEL_CALLS.get('bn_backward_deferred_fold', 0) == d0 + 1
    assert ops.KERNEL_CALLS.get('conv_wgrad_bn_dy', 0) == w0 + 1
    lb = b.bce_loss_bf16(xu8, 1.0, decode=cfg)
    lb.backward()
    assert ops.KERNEL_CALLS.get('bn_backward_deferred_fold', 0) == d0 + 1      # b took the apply launch
    # the same forward; its BN sums are fp64 atomics whose arrival order may differ run to run:
    # equal up to an ulp of the fp32 loss
    torch.testing.assert_close(la, lb, rtol=2.4e-7, atol=1e-30)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()), msg=n)
    # a frozen first layer never takes the hand-off: the other gradients are unchanged
    a.zero_grad(set_to_none=True)
    b.zero_grad(set_to_none=True)
    for m in (a, b):
        m.features[0].weight.requires_grad_(False)
    a.bce_loss_bf16(xu8, 1.0, decode=cfg).backward()
    b.bce_loss_bf16(xu8, 1.0, decode=cfg).backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        if pa.requires_grad:
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()),
                                       msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,decoded', [((4, 96, 128), False), ((4, 96, 128), True), ((8, 480, 640), False),
                                           ((3, 100, 136), False), ((3, 100, 136), True)])
def test_first_layer_applies_its_bn(dev, monkeypatch, shape, decoded):
    """The u8 first layer applies the first BatchNorm+LeakyReLU itself, after
    a grid barrier on its statistics (ops.BnProduced): no apply launch; its
    activation is exactly the apply kernel's on the same z with the kernel's
    own mean / invstd; those match the apply path's to float rounding (10
    tiles' fp32 partial sums per block instead of 4: the last bit may
    differ); the steps train alike; no barrier wait gave up."""
    from blendtorch.models import Discriminator
    N, H, W = shape
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    if not ops.conv1_bn_apply_fits(N, H // 2, W // 2, 32, dev):
        pytest.skip('grid larger than the resident blocks')
    g = torch.Generator(device=dev).manual_seed(22)
    xu8 = torch.randint(0, 256, (N, H, W, 4), dtype=torch.uint8, device=dev, generator=g).permute(0, 3, 1, 2)
    t0 = ops.conv_grid_barrier_timeouts()
    # the kernel alone: y = the apply kernel of (z, its mean / invstd), bit for bit
    lut = ops.decode_lut_bf16(cfg, dev)
    w16 = (0.1 * torch.randn(32, 3, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    bn = ops.BatchNormLeakyReLU2d(32).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.2, 0.2, generator=g)
    acc = ops.BnAccumulator(32, dev)
    early = bn.produced_by_conv(dev)
    xd = torch.empty((N, 4, H, W), dtype=torch.bfloat16, device=dev, memory_format=cl) if decoded else None
    z = ops.conv_fwd(xu8, w16, acc.fwd, acc.R, lut=lut, act_out=xd, out_bn=early)
    assert early.y is not None and early.z is z
    zs = z.permute(0, 2, 3, 1)
    ref = torch.empty_like(zs)
    ops.hip_ext().bn_fwd_apply(zs.data_ptr(), ref.data_ptr(), zs.numel() // 32, 32, ops.OUT_DTYPES['bfloat16'],
                               early.mean.data_ptr(), early.invstd.data_ptr(), early.w.data_ptr(), early.b.data_ptr(),
                               0.2, ops._stream(dev))
    assert torch.equal(early.y.permute(0, 2, 3, 1), ref)
    zf = z.float().permute(0, 2, 3, 1).reshape(-1, 32)
    torch.testing.assert_close(early.mean, zf.mean(0), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(early.invstd, zf.var(0, unbiased=False).add(1e-5).rsqrt(), rtol=1e-4, atol=0)
    assert int(bn.num_batches_tracked) == 1
    assert int(torch.count_nonzero(acc.fwd)) == 0          # released for the next producer
    # the model: the first BN without its apply launch, trained like the apply path
    torch.manual_seed(4)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    a.conv1_bn, b.conv1_bn = True, False
    a.conv_out_bn = b.conv_out_bn = False   # (test_conv_applies_its_output_bn)
    monkeypatch.setattr(ops, '_C4_DECODED', decoded)   # (the forward also writes the decoded frames)
    for step in range(2):   # the accumulator and the barrier word are reused
        a.zero_grad(set_to_none=True)
        b.zero_grad(set_to_none=True)
        c0 = (ops.KERNEL_CALLS.get('conv_fwd_bn_apply', 0), ops.KERNEL_CALLS.get('bn_forward_by_producer', 0))
        la = a.bce_loss_bf16(xu8, 1.0, decode=cfg)
        assert ops.KERNEL_CALLS.get('conv_fwd_bn_apply', 0) == c0[0] + 1
        assert ops.KERNEL_CALLS.get('bn_forward_by_producer', 0) == c0[1] + 1
        lb = b.bce_loss_bf16(xu8, 1.0, decode=cfg)
        assert ops.KERNEL_CALLS.get('bn_forward_by_producer', 0) == c0[1] + 1   # b applied BN1 in its own launch
        la.backward()
        lb.backward()
        torch.cuda.synchronize()
        assert ops.conv_grid_barrier_timeouts() == t0
        torch.testing.assert_close(la, lb, rtol=2e-3, atol=1e-5)
        bn_a, bn_b = a.features[1], b.features[1]
        torch.testing.assert_close(bn_a.running_mean, bn_b.running_mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(bn_a.running_var, bn_b.running_var, rtol=1e-5, atol=1e-6)
        assert int(bn_a.num_batches_tracked) == int(bn_b.num_batches_tracked) == step + 1
        for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
            ga, gb = pa.grad.flatten().double(), pb.grad.flatten().double()
            assert float(ga @ gb / (ga.norm() * gb.norm())) > 0.999, n


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(4, 128, 160), (8, 480, 640), (2, 72, 200)])
def test_conv_applies_its_output_bn(dev, shape):
    """The MFMA forward of the deeper layers applies the BatchNorm+LeakyReLU
    of its output itself when its whole grid fits on the chip (grid barrier,
    ops.BnProduced): the same loss, running statistics and
    num_batches_tracked bit for bit as the apply launches, gradients equal up
    to the weight-gradient reduce's atomic order, over two steps."""
    from blendtorch.models import Discriminator
    N, H, W = shape
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(23)
    x = torch.rand(N, 4, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    torch.manual_seed(5)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    a.conv_out_bn, b.conv_out_bn = True, False
    # conv2 and conv3 (conv4's BN is applied by the fused head)
    fits = [ops.conv_out_bn_fits(N, H // 2 ** (k + 1), W // 2 ** (k + 1), 32 * 2 ** (k - 1), 32 * 2 ** k, dev)
            for k in (1, 2)]
    if not any(fits):
        pytest.skip('no grid small enough')
    t0 = ops.conv_grid_barrier_timeouts()
    for step in range(2):
        a.zero_grad(set_to_none=True)
        b.zero_grad(set_to_none=True)
        c0 = ops.KERNEL_CALLS.get('conv_fwd_bn_apply', 0), ops.KERNEL_CALLS.get('bn_forward_by_producer', 0)
        la = a.bce_loss_bf16(x, 1.0)
        assert ops.KERNEL_CALLS.get('conv_fwd_bn_apply', 0) == c0[0] + sum(fits)
        assert ops.KERNEL_CALLS.get('bn_forward_by_producer', 0) == c0[1] + sum(fits)
        lb = b.bce_loss_bf16(x, 1.0)
        assert ops.KERNEL_CALLS.get('conv_fwd_bn_apply', 0) == c0[0] + sum(fits)
        la.backward()
        lb.backward()
        torch.cuda.synchronize()
        assert ops.conv_grid_barrier_timeouts() == t0
        ops.check_grid_barrier()
        # the BN sums are fp64 atomics whose arrival order differs between the two paths (and
        # from run to run): equal up to 1 float ulp once rounded to the fp32 buffers / loss
        ulp = dict(rtol=1.2e-7, atol=1e-30)
        torch.testing.assert_close(la, lb, rtol=1e-6, atol=1e-30)   # (ulps of the stats, propagated)
        for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
            if ba.is_floating_point():
                torch.testing.assert_close(ba, bb, **ulp, msg=n)
            else:
                torch.testing.assert_close(ba, bb, rtol=0, atol=0, msg=n)
        # the same backward inputs bit for bit: the gradients differ only by the float atomics'
        # order of the weight-gradient reduces (small layers: a few large cancelling partials)
        for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
            ga, gb = pa.grad.flatten().double(), pb.grad.flatten().double()
            assert float(ga @ gb / (ga.norm() * gb.norm())) > 0.9999, n


@pytest.mark.gpu
@pytest.mark.parametrize('u8', [True, False])
@pytest.mark.parametrize('cout,wc', [(32, 3), (64, 4)])
@pytest.mark.parametrize('tiles,rows', [(4, 2), (1, 4), (3, 4)])
def test_first_layer_patch_forward(dev, u8, cout, wc, tiles, rows):
    """The first layer's patch kernel (input decoded once into LDS, rows x 64
    output tiles, several tiles per block, BN sums into a BnAccumulator)
    against the im2col tap-GEMM path: bit-identical outputs (the same MFMA
    dot products with the operands swapped), the same channel sums (fp64
    atomics over other partials), both equal to the fp32 reference.  644
    columns: a ragged last column tile; 482 rows: a ragged last row tile."""
    import torch.nn.functional as F
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(cout + wc)
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    raw = torch.randint(0, 256, (3, 482, 644, 4), dtype=torch.uint8, device=dev, generator=g)
    if u8:
        x, lut = raw.permute(0, 3, 1, 2), ops.decode_lut_bf16(cfg, dev)
        xdec = ops.decode(raw, cfg).permute(0, 3, 1, 2)
    else:
        x = xdec = ops.decode(raw, cfg).permute(0, 3, 1, 2)
        lut = None
    w = (0.1 * torch.randn(cout, wc, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    outs = []
    try:
        for t in (tiles, -1):
            ops.hip_ext().conv_set_conv1_tiles(t, rows)
            acc = ops.BnAccumulator(cout, dev)
            y = ops.conv_fwd(x, w, acc.fwd, acc.R, lut=lut)
            s = acc.fwd[:acc.R * 2 * cout].view(acc.R, 2, cout).sum(0)
            outs.append((y, s))
    finally:
        ops.hip_ext().conv_set_conv1_tiles(0, 0)
    assert torch.equal(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-6, atol=1e-3)
    wref = w.float() if wc == 4 else torch.cat([w.float(), torch.zeros(cout, 1, 4, 4, device=dev)], 1)
    ref = F.conv2d(xdec.float(), wref, None, 2, 1)
    torch.testing.assert_close(outs[0][0].float(), ref, rtol=2 ** -7, atol=1e-3 * float(ref.abs().max()))
    yf = outs[0][0].float().permute(0, 2, 3, 1).reshape(-1, cout).double()
    torch.testing.assert_close(outs[0][1][0], yf.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(outs[0][1][1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(outs[0][1][1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)


def _fill_acc(acc, x):
    """A BnAccumulator's forward replicas as a producer leaves them: replica 0
    holds the fp64 channel sums and sums of squares of x, the rest zero."""
    C = x.shape[1]
    xf = x.permute(0, 2, 3, 1).reshape(-1, C).double()
    acc.fwd.zero_()
    v = acc.fwd[:acc.R * 2 * C].view(acc.R, 2, C)
    v[0, 0] = xf.sum(0)
    v[0, 1] = (xf * xf).sum(0)


@pytest.mark.gpu
@pytest.mark.parametrize('cin,cout,hw', [(32, 64, (48, 64)), (64, 128, (32, 40)), (128, 256, (16, 24))])
def test_forward_applies_input_bn(dev, cin, cout, hw):
    """A convolution that applies the BatchNorm+LeakyReLU producing its input
    in its own operand staging (ops.BnActLazy: the BN call skips its apply)
    against the apply pass + plain convolution: bit-identical output, output
    statistics, activation side output (act_out: every input element, from
    the centre taps), BN mean / invstd and running statistics; the
    accumulator cleared for the next producer either way.  cin 128: a
    thread's chunk alternates between two channel sets."""
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(cin)
    H, W = hw
    x = (torch.randn(2, cin, H, W, device=dev, generator=g) * 0.7 + 0.2).to(torch.bfloat16).contiguous(memory_format=cl)
    w16 = (0.05 * torch.randn(cout, cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    bns = []
    for _ in range(2):
        bn = ops.BatchNormLeakyReLU2d(cin).to(dev)
        with torch.no_grad():
            bn.weight.copy_(1 + 0.1 * torch.randn(cin, device=dev, generator=torch.Generator(device=dev).manual_seed(1)))
            bn.bias.copy_(0.1 * torch.randn(cin, device=dev, generator=torch.Generator(device=dev).manual_seed(2)))
        bns.append(bn)
    # reference: apply pass, then the convolution
    acc_in, acc_out = ops.BnAccumulator(cin, dev), ops.BnAccumulator(cout, dev)
    _fill_acc(acc_in, x)
    with torch.no_grad():
        a = bns[0].forward_from_stats(x, acc_in)
        y_ref = ops.conv_fwd(a.contiguous(memory_format=cl), w16, acc_out.fwd, acc_out.R)
    s_ref = acc_out.fwd.clone()
    assert float(acc_in.fwd.abs().sum()) == 0.0
    # the convolution applies the BN
    acc_in2, acc_out2 = ops.BnAccumulator(cin, dev), ops.BnAccumulator(cout, dev)
    _fill_acc(acc_in2, x)
    lazy = ops.BnActLazy()
    before = ops.KERNEL_CALLS.get('conv_fwd_act', 0)
    with torch.no_grad():
        xo = bns[1].forward_from_stats(x, acc_in2, lazy=lazy)
        assert xo.data_ptr() == x.data_ptr()   # the BN's input, no apply launch
        xa = torch.empty_like(x, memory_format=cl)
        y = ops.conv_fwd(xo, w16, acc_out2.fwd, acc_out2.R, act=lazy, act_out=xa)
    torch.cuda.synchronize()
    assert ops.KERNEL_CALLS['conv_fwd_act'] == before + 1
    assert float(acc_in2.fwd.abs().sum()) == 0.0          # cleared by the last block
    assert torch.equal(xa, a)                               # the activation, every element
    assert torch.equal(y, y_ref)
    # (the reference forward may be the patch GEMM, whose blocks add into other replicas: compare the
    # per-channel sums over the replicas)
    R2 = acc_out2.R
    torch.testing.assert_close(acc_out2.fwd[:R2 * 2 * cout].view(R2, -1).sum(0),
                               s_ref[:R2 * 2 * cout].view(R2, -1).sum(0), rtol=1e-6, atol=1e-3)
    for ba, bb in zip(bns[0].buffers(), bns[1].buffers()):
        assert torch.equal(ba, bb)


@pytest.mark.gpu
@pytest.mark.parametrize('cin,cout,hw', [(32, 64, (64, 80)), (128, 256, (32, 40)), (4, 32, (96, 128))])
def test_wgrad_applies_bn_backward_folded(dev, cin, cout, hw, wgrad_pipe):
    """The weight gradient that applies the following BatchNorm+LeakyReLU's
    backward to its staged dY (ops.BnBwdFold): it folds the BN's backward
    accumulator itself (dw / db equal to the fp64 sums rounded once), its gx
    side output is bit-identical to the apply kernel's (bn_bwd_apply: the same
    BnBwdCoef arithmetic), the weight gradient equals the one computed from
    that gx, and the accumulator is left cleared.  cin 4: the first layer's
    wave-private kernel (no data gradient, no gx output)."""
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(cin + cout)
    H, W = hw
    N, Ho, Wo = 2, H // 2, W // 2
    x = torch.randn(N, cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    y = (torch.randn(N, Ho, Wo, cout, device=dev, generator=g) * 0.8 + 0.1).to(torch.bfloat16)   # BN input, NHWC
    gy = (torch.randn(N, cout, Ho, Wo, device=dev, generator=g) * 1e-2).to(torch.bfloat16).contiguous(memory_format=cl)
    yf = y.float().reshape(-1, cout)
    mean = yf.mean(0)
    invstd = torch.rsqrt(yf.var(0, unbiased=False) + 1e-5)
    w = 1 + 0.1 * torch.randn(cout, device=dev, generator=g)
    b = 0.1 * torch.randn(cout, device=dev, generator=g)
    slope = 0.2
    acc = ops.BnAccumulator(cout, dev)
    # the backward sums as the consumer leaves them (any values do: both paths read them)
    xh = (yf - mean) * invstd
    gz = torch.where(xh * w + b > 0, 1.0, slope) * gy.permute(0, 2, 3, 1).reshape(-1, cout).float()
    acc.bwd.zero_()
    v = acc.bwd[:acc.R * 2 * cout].view(acc.R, 2, cout)
    v[0, 0] = gz.double().sum(0)
    v[0, 1] = (gz.double() * xh.double()).sum(0)
    db_ref = v[0, 0].float().clone()
    dw_ref = v[0, 1].float().clone()
    # reference: the apply kernel, then the weight gradient of its output
    gx_ref = torch.empty_like(y)
    ops.hip_ext().bn_bwd_apply(y.data_ptr(), gy.data_ptr(), gx_ref.data_ptr(), N * Ho * Wo, cout,
                               ops.OUT_DTYPES['bfloat16'], mean.data_ptr(), invstd.data_ptr(), w.data_ptr(),
                               b.data_ptr(), dw_ref.data_ptr(), db_ref.data_ptr(), slope,
                               ops._stream(dev))
    gx_ref = gx_ref.permute(0, 3, 1, 2)
    wout = 3 if cin == 4 else cin
    out_ref = torch.zeros(cout, wout, 4, 4, device=dev)
    xin = x if cin != 4 else x
    ops.conv_wgrad(xin, gx_ref.contiguous(memory_format=cl), out_ref)
    # the weight gradient folds and applies
    dw, db = torch.empty(cout, device=dev), torch.empty(cout, device=dev)
    pend = ops.BnBwdFold(y, mean, invstd, w, b, slope, acc, dw, db, ())
    if cin != 4:
        pend.gx_out = torch.empty_like(gy, memory_format=cl)
    out = torch.zeros(cout, wout, 4, 4, device=dev)
    before = ops.KERNEL_CALLS.get('conv_wgrad_bn_dy_fold', 0)
    ops.conv_wgrad(xin, gy, out, bn_dy=pend)
    torch.cuda.synchronize()
    assert ops.KERNEL_CALLS['conv_wgrad_bn_dy_fold'] == before + 1
    assert torch.equal(dw, dw_ref) and torch.equal(db, db_ref)
    assert float(acc.bwd.abs().sum()) == 0.0
    if cin != 4:
        assert torch.equal(pend.gx_out, gx_ref)
    torch.testing.assert_close(out, out_ref, rtol=1e-5, atol=1e-5 * float(out_ref.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(2, 64, 80), (3, 50, 72)])
@pytest.mark.parametrize('with_bn', [False, True])
def test_dgrad_patch_matches_tap_gemm(dev, shape, with_bn):
    """The 32-channel layer's data gradient from a dY patch (all four parity
    classes per block, weights as the MFMA A operand) against the tap-GEMM
    path: bit-identical dx (the same K-step order), the same BN-backward sums
    (fp64 adds in another grouping), both equal to the fp32 reference.  50 x
    72: ragged class-grid tiles (25 x 36 against 4 x 32)."""
    import torch.nn.functional as F
    cl = torch.channels_last
    N, H, W = shape
    g = torch.Generator(device=dev).manual_seed(H + W)
    dy = torch.randn(N, 64, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.05 * torch.randn(64, 32, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    outs = []
    for patch in (1, 0):
        ops.hip_ext().conv_set_dgrad_patch(patch)
        try:
            link = None
            if with_bn:
                link = ops.BnLink()
                x = torch.randn(N, H, W, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
                link.x = x.to(torch.bfloat16)
                link.mean = torch.full((32,), 0.1, device=dev)
                link.invstd = torch.full((32,), 1.3, device=dev)
                link.w = torch.linspace(0.5, 1.5, 32, device=dev)
                link.b = torch.linspace(-0.2, 0.2, 32, device=dev)
                link.slope = 0.2
                link.acc = ops.BnAccumulator(32, dev)
            dx = ops.conv_dgrad(dy, w, (N, 32, H, W), bn=link)
            sums = link.acc.bwd[:link.acc.R * 64].view(link.acc.R, 2, 32).sum(0) if with_bn else None
            outs.append((dx, sums))
        finally:
            ops.hip_ext().conv_set_dgrad_patch(-1)
    assert torch.equal(outs[0][0], outs[1][0])
    if with_bn:   # (fp32 per-block partials over other pixel groupings, then fp64 adds)
        torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-5 * float(outs[1][1].abs().max()))
    ref = F.conv_transpose2d(dy.float(), w.float(), None, 2, 1)
    torch.testing.assert_close(outs[0][0].float(), ref, rtol=2 ** -7, atol=1e-3 * float(ref.abs().max()))


@pytest.mark.gpu
def test_first_layer_decoded_side_output(dev, monkeypatch):
    """The first layer's patch forward also writes the decoded frames
    (act_out) and the weight gradient reads those bf16 frames instead of
    decoding the u8 frames again: the decoded tensor equals ops.decode's,
    and the step gives the same loss and gradients (up to the weight
    reduce's atomic order) as decoding in the weight gradient."""
    from blendtorch.models import Discriminator
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(9)
    raw = torch.randint(0, 256, (4, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g)
    xu8 = raw.permute(0, 3, 1, 2)
    lut = ops.decode_lut_bf16(cfg, dev)
    w16 = (0.1 * torch.randn(32, 3, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    xd = torch.full(xu8.shape, float('nan'), dtype=torch.bfloat16, device=dev).contiguous(memory_format=cl)
    acc = ops.BnAccumulator(32, dev)
    ops.conv_fwd(xu8, w16, acc.fwd, acc.R, lut=lut, act_out=xd)
    assert torch.equal(xd, ops.decode(raw, cfg).permute(0, 3, 1, 2))
    torch.manual_seed(3)
    nets = [Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl) for _ in range(2)]
    nets[1].load_state_dict(nets[0].state_dict())
    losses = []
    for m, dec in zip(nets, (True, False)):
        monkeypatch.setattr(ops, '_C4_DECODED', dec)
        loss = m.bce_loss_bf16(xu8, 1.0, decode=cfg)
        loss.backward()
        losses.append(loss.detach())
    assert torch.equal(losses[0], losses[1])
    for (n, pa), pb in zip(nets[0].named_parameters(), nets[1].parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()), msg=n)


@pytest.mark.gpu
def test_side_stream_weight_gradients(dev):
    """Weight gradients on the side stream (ops.set_side_wgrad(True), forked
    before each data gradient and joined after the chain's last launch) give
    the gradients of the in-line order -- eager, and in the bench's captured
    step (FusedAdam bucket views, so the deferred-reduce chain rides on the
    side stream) where the weights after three steps agree far below lr."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(21)
    xs = [torch.randint(0, 256, (4, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g) for _ in range(3)]
    torch.manual_seed(5)
    nets = [Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl) for _ in range(4)]
    for m in nets[1:]:
        m.load_state_dict(nets[0].state_dict())
    prev = ops.set_side_wgrad(True)
    try:
        for m, side in zip(nets[:2], (True, False)):   # eager
            ops.set_side_wgrad(side)
            m.bce_loss_bf16(xs[0].permute(0, 3, 1, 2), 1.0, decode=cfg).backward()
        torch.cuda.synchronize()
        for (n, pa), pb in zip(nets[0].named_parameters(), nets[1].parameters()):
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()),
                                       msg=n)
        lr = 2e-4
        steps = []
        for m, side in zip(nets[2:], (True, False)):   # captured (the setting is read while capturing)
            ops.set_side_wgrad(side)
            st = CapturedStep(m, ops.FusedAdam(m.parameters(), lr=lr),
                              lambda mm, x: mm.bce_loss_bf16(x.permute(0, 3, 1, 2), 1.0, decode=cfg),
                              allreduce=False, warmup=1)
            for x in xs:
                st(x)
            steps.append(st)
        torch.cuda.synchronize()
        assert all(st.state == 'graph' for st in steps)
    finally:
        ops.set_side_wgrad(prev)
    for pa, pb in zip(nets[2].parameters(), nets[3].parameters()):
        d = (pa - pb).detach().abs()
        assert float(d.mean()) < 0.1 * lr and float((d > 0.5 * lr).float().mean()) < 0.02


@pytest.mark.gpu
def test_fused_data_and_weight_gradient_launch(dev):
    """ops.set_fuse_dw(True): a tap-GEMM layer's data gradient is held and
    launched with its weight gradient in one kernel (dgrad_wgrad_kernel) --
    two such layers per disc backward -- and the step's gradients, BN
    statistics and (captured, FusedAdam) weights match the two-launch order."""
    from blendtorch.models import Discriminator
    from blendtorch.parallel.step import CapturedStep
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(31)
    xs = [torch.randint(0, 256, (4, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g) for _ in range(3)]
    torch.manual_seed(6)
    nets = [Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl) for _ in range(4)]
    for m in nets[1:]:
        m.load_state_dict(nets[0].state_dict())
    prev = ops.set_fuse_dw(True)
    try:
        for m, fuse in zip(nets[:2], (True, False)):   # eager
            ops.set_fuse_dw(fuse)
            before = ops.KERNEL_CALLS.get('conv_dgrad_held', 0)
            m.bce_loss_bf16(xs[0].permute(0, 3, 1, 2), 1.0, decode=cfg).backward()
            # conv3, conv4 (tap GEMM) and conv2 (patch data gradient, unless BT_FUSE_PATCH=0)
            assert ops.KERNEL_CALLS.get('conv_dgrad_held', 0) - before in ((3, 2) if fuse else (0,))
        torch.cuda.synchronize()
        assert not ops.hip_ext().conv_dgrad_held()
        for (n, pa), pb in zip(nets[0].named_parameters(), nets[1].parameters()):
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-6 + 1e-4 * float(pb.grad.abs().max()),
                                       msg=n)
        for ba, bb in zip(nets[0].buffers(), nets[1].buffers()):
            torch.testing.assert_close(ba, bb, rtol=1e-5, atol=1e-6)
        lr = 2e-4
        steps = []
        for m, fuse in zip(nets[2:], (True, False)):   # captured (the setting is read while capturing)
            ops.set_fuse_dw(fuse)
            st = CapturedStep(m, ops.FusedAdam(m.parameters(), lr=lr),
                              lambda mm, x: mm.bce_loss_bf16(x.permute(0, 3, 1, 2), 1.0, decode=cfg),
                              allreduce=False, warmup=1)
            for x in xs:
                st(x)
            steps.append(st)
        torch.cuda.synchronize()
        assert all(st.state == 'graph' for st in steps)
    finally:
        ops.set_fuse_dw(prev)
    for pa, pb in zip(nets[2].parameters(), nets[3].parameters()):
        d = (pa - pb).detach().abs()
        assert float(d.mean()) < 0.1 * lr and float((d > 0.5 * lr).float().mean()) < 0.02


@pytest.mark.gpu
@pytest.mark.parametrize('co128', [0, 1, 2], ids=['co64', 'co128', 'co128_dbn128'])
@pytest.mark.parametrize('cin,cout,hw', [(64, 128, (60, 80)), (128, 256, (30, 40)), (64, 128, (12, 18)),
                                         (128, 256, (14, 22))])
def test_dgrad_wgrad_kernel_matches_separate_launches(dev, cin, cout, hw, co128):
    """One layer, direct ops: conv_dgrad held + conv_wgrad (one launch) give
    the bit-identical data gradient and the same weight gradient as the two
    launches (odd shapes: partial tiles and runs of 8 padded with exiting
    blocks)."""
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(cin + cout + hw[0])
    H, W = hw
    x = torch.randn(8, cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(8, cout, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.05 * torch.randn(cout, cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    ext = ops.hip_ext()
    ext.conv_set_wgrad_co128(1 if co128 else 0)
    ext.conv_set_dgrad_bn128(1 if co128 == 2 else 0)
    outs = []
    for fuse in (False, True):
        if fuse:
            ext.conv_dgrad_hold(1)
        try:
            dx = ops.conv_dgrad(dy, w, tuple(x.shape))
        finally:
            ext.conv_dgrad_hold(0)
        assert bool(ext.conv_dgrad_held()) == fuse
        gw = ops.conv_wgrad(x, dy, torch.empty(cout, cin, 4, 4, device=dev))
        assert not ext.conv_dgrad_held()
        torch.cuda.synchronize()
        outs.append((dx, gw))
    ext.conv_set_wgrad_co128(-1)
    ext.conv_set_dgrad_bn128(-1)
    assert torch.equal(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-5, atol=1e-5 * float(outs[0][1].abs().max()))
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 4, 4), dy.float(), stride=2, padding=1)
    torch.testing.assert_close(outs[1][1], ref, rtol=1e-3, atol=1e-3 * float(ref.abs().max()))


@pytest.mark.gpu
def test_grid_barrier_failure_raises(dev):
    """a grid barrier that gives up must not train on
    incomplete BN statistics silently.  The kernel raises a host-mapped flag;
    ops.check_grid_barrier and every CapturedStep call raise on it."""
    from blendtorch.parallel.step import CapturedStep
    ops._grid_barrier_armed()                 # maps the flag (as the first BN-applying launch does)
    assert ops.GRID_BARRIER_USED
    assert ops.hip_ext().conv_grid_barrier_failed() == 0
    ops.check_grid_barrier()
    net = torch.nn.Linear(4, 1).to(dev)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    step = CapturedStep(net, opt, lambda m, x: m(x).square().mean(), allreduce=False, graph=False)
    step(torch.ones(2, 4, device=dev))
    ops.clear_grid_barrier(_simulate_failure=True)
    try:
        with pytest.raises(ops.GridBarrierError, match='grid barrier timed out'):
            step(torch.ones(2, 4, device=dev))
        with pytest.raises(ops.GridBarrierError):
            ops.check_grid_barrier()
    finally:
        ops.clear_grid_barrier()
    ops.check_grid_barrier()
    step(torch.ones(2, 4, device=dev))


@pytest.mark.gpu
@pytest.mark.parametrize('N,H,W', [(8, 240, 320), (2, 30, 40), (3, 10, 66), (1, 18, 130)])
def test_fwd_patch_gemm_matches_tap_gemm(dev, N, H, W):
    """The 32 -> 64 forward's persistent patch GEMM (conv_fwd_patch_kernel)
    against the tap GEMM: the same tap order, so the bf16 output is bit for
    bit the same; the accumulator's BN sums agree to fp32 rounding (summed in
    another order), and both match an fp32 conv2d.  Shapes with partial
    tiles (rows and columns) included."""
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(H + W)
    x = torch.randn(N, 32, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.1 * torch.randn(64, 32, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    ext = ops.hip_ext()
    out = {}
    for on in (1, 0):
        acc = ops.BnAccumulator(64, dev)
        ext.conv_set_fwd_patch(on)
        try:
            y = ops.conv_fwd(x, w, acc.fwd, acc.R)
            y2 = ops.conv_fwd(x, w)                     # no statistics
        finally:
            ext.conv_set_fwd_patch(-1)
        torch.cuda.synchronize()
        s = acc.fwd[:acc.R * 128].view(acc.R, 2, 64).sum(0)
        out[on] = (y, y2, s)
    assert torch.equal(out[1][0], out[0][0])
    assert torch.equal(out[1][1], out[0][0])
    torch.testing.assert_close(out[1][2], out[0][2], rtol=1e-5, atol=1e-3)
    ref = torch.nn.functional.conv2d(x.float(), w.float(), stride=2, padding=1)
    torch.testing.assert_close(out[1][0].float(), ref, rtol=2e-2, atol=2e-2)
    yf = out[1][0].float().permute(0, 2, 3, 1).reshape(-1, 64).double()
    torch.testing.assert_close(out[1][2][0], yf.sum(0), rtol=1e-5, atol=1e-2)
    torch.testing.assert_close(out[1][2][1], (yf * yf).sum(0), rtol=1e-5, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize('wide', [0, 1], ids=['w128', 'w256'])
@pytest.mark.parametrize('hw', [(240, 320), (30, 46)])
def test_patch_dgrad_with_wide_wgrad_one_launch(dev, hw, wide):
    """The 32-channel layer's patch data gradient held and launched together
    with its weight gradient (dpatch_wgrad_kernel), with 128- or 256-column
    weight-gradient tiles (conv_wgrad_wide_body): the data gradient is
    bit-identical to its own launch, the weight gradient matches fp32 PyTorch."""
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(hw[0] + wide)
    H, W = hw
    cin, cout = 32, 64
    x = torch.randn(8, cin, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(8, cout, H // 2, W // 2, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.05 * torch.randn(cout, cin, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    ext = ops.hip_ext()
    ext.conv_set_wgrad_wide(wide)
    try:
        alone = ops.conv_dgrad(dy, w, tuple(x.shape))
        ext.conv_dgrad_hold(1)
        try:
            dx = ops.conv_dgrad(dy, w, tuple(x.shape))
        finally:
            ext.conv_dgrad_hold(0)
        assert ext.conv_dgrad_held()
        gw = ops.conv_wgrad(x, dy, torch.empty(cout, cin, 4, 4, device=dev))
        assert not ext.conv_dgrad_held()
        torch.cuda.synchronize()
    finally:
        ext.conv_set_wgrad_wide(-1)
    assert torch.equal(dx, alone)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 4, 4), dy.float(), stride=2, padding=1)
    torch.testing.assert_close(gw, ref, rtol=1e-3, atol=1e-3 * float(ref.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize('N,C,H,W,CO', [(8, 64, 120, 160, 128), (8, 128, 60, 80, 256), (2, 64, 30, 46, 128),
                                        (1, 128, 18, 130, 256)])
def test_fwd_split_k_matches_fp32(dev, N, C, H, W, CO):
    """The split-K forward (tap_gemm_body SPLIT = 2: two blocks per 128-channel
    tile, one K half each, the first to finish parks its accumulators for the
    second): matches fp32 conv2d and the unsplit forward to bf16 rounding, its
    BN sums match the output's, and repeated runs (eager and graph replays --
    the tickets reset themselves) are bit-identical: a + b is the same bits
    whichever half finishes first."""
    cl = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(C + H)
    x = torch.randn(N, C, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (0.05 * torch.randn(CO, C, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
    ext = ops.hip_ext()
    ref = torch.nn.functional.conv2d(x.float(), w.float(), stride=2, padding=1)
    y0 = ops.conv_fwd(x, w)
    ext.conv_set_fwd_split(1)
    try:
        n0 = ext.conv_fwd_split_launches()
        acc = ops.BnAccumulator(CO, dev)
        y1 = ops.conv_fwd(x, w, acc.fwd, acc.R)
        y2 = ops.conv_fwd(x, w)
        assert ext.conv_fwd_split_launches() == n0 + 2
        stream = torch.cuda.Stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            ops.conv_fwd(x, w)             # (the capture stream's scratch, allocated eagerly)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                yg = ops.conv_fwd(x, w)
        torch.cuda.current_stream(dev).wait_stream(stream)
        outs = []
        for _ in range(3):
            graph.replay()
            outs.append(yg.clone())
    finally:
        ext.conv_set_fwd_split(-1)
    torch.cuda.synchronize()
    assert ext.conv_fwd_split_launches() == n0 + 4
    assert torch.equal(y1, y2)
    for o in outs:
        assert torch.equal(o, y1)
    torch.testing.assert_close(y1.float(), ref, rtol=2e-2, atol=2e-2)
    # against the unsplit forward: the same products, summed as two halves (bf16 rounding apart)
    assert (y1.float() - y0.float()).abs().max() <= 2 ** -6 * y0.float().abs().max()
    s = acc.fwd[:acc.R * 2 * CO].view(acc.R, 2, CO).sum(0)
    yf = y1.float().permute(0, 2, 3, 1).reshape(-1, CO).double()
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-4, atol=5e-2)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-4, atol=5e-2)
