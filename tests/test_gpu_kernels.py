"""Numerics of the gfx950 kernels against plain-PyTorch fp32 references."""
import numpy as np
import pytest
import torch

from blendtorch import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    assert torch.cuda.is_available(), 'GPU tests need a HIP device'
    ops.hip_ext()  # must load: no silent fallback
    return torch.device('cuda', 0)


def _imgs(B, H, W, C, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (B, H, W, C), dtype=torch.uint8, generator=g).to(dev)


@pytest.mark.parametrize('C,channels', [(4, 'rgb'), (4, 'rgba'), (3, 'rgb'), (3, 'bgr'), (4, 'bgra')])
@pytest.mark.parametrize('dtype', ['float32', 'bfloat16', 'float16'])
@pytest.mark.parametrize('layout', ['nchw', 'nhwc'])
def test_decode_matches_reference(dev, C, channels, dtype, layout):
    x = _imgs(3, 48, 64, C, dev)
    cfg = ops.DecodeConfig.densityopt(channels=channels, gamma=2.2, dtype=dtype, layout=layout)
    out = ops.decode(x, cfg)
    ref = ops.reference_decode(x.cpu(), cfg)
    torch.cuda.synchronize()
    assert out.shape == ref.shape and out.dtype == ref.dtype
    assert torch.equal(out.cpu(), ref), (out.cpu().float() - ref.float()).abs().max()


@pytest.mark.parametrize('W', [640, 30, 17])
def test_decode_unit_flip_shapes(dev, W):
    x = _imgs(2, 7, W, 4, dev, seed=1)
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2, flip=True)
    out = ops.decode(x, cfg)
    ref = ops.reference_decode(x.cpu(), cfg)
    assert torch.equal(out.cpu(), ref)


def test_decode_per_image_flip_and_u8(dev):
    x = _imgs(4, 16, 32, 4, dev, seed=2)
    cfg = ops.DecodeConfig(channels='rgba', gamma=2.2, dtype='uint8')
    flip = [1, 0, 0, 1]
    out = ops.decode(x, cfg, flip=flip)
    ref = ops.reference_decode(x.cpu(), cfg, flip=flip)
    assert torch.equal(out.cpu(), ref)
    # gamma LUT bit-exact with the numpy formula of btb/offscreen.py:105-112
    np_ref = np.uint8(255.0 * (x.cpu().numpy()[..., :3].astype(np.float32) / 255) ** (1 / 2.2))
    xf = x.cpu().numpy()
    xf[[0, 3]] = xf[[0, 3], ::-1]
    np_ref = np.uint8(255.0 * (xf[..., :3].astype(np.float32) / 255) ** (1 / 2.2))
    assert np.array_equal(out.cpu().numpy()[:, :3].transpose(0, 2, 3, 1), np_ref)


def test_decode_large_batch_vector_path(dev):
    x = _imgs(8, 480, 640, 4, dev, seed=3)
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    out = ops.decode(x, cfg)
    ref = ops.reference_decode(x, cfg)  # on-device torch reference
    assert torch.equal(out, ref)


@pytest.mark.parametrize('gamma', [None, 2.2])
def test_color4x4_mfma(dev, gamma):
    x = _imgs(2, 16, 96, 4, dev, seed=4)
    rng = np.random.default_rng(0)
    M = rng.normal(size=(4, 4)).astype(np.float32)
    b = rng.normal(size=4).astype(np.float32)
    out = ops.color4x4(x, M, b, gamma=gamma)
    ref = ops.reference_color4x4(x.cpu(), M, b, gamma=gamma)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-3)


def test_color4x4_identity_layout_probe(dev):
    """Asymmetric check of the MFMA operand map: a permutation matrix must
    route input channel k to output channel perm[k] exactly."""
    x = _imgs(1, 4, 64, 4, dev, seed=5)
    perm = [2, 0, 3, 1]
    M = np.zeros((4, 4), np.float32)
    for k, c in enumerate(perm):
        M[c, k] = 1.0
    out = ops.color4x4(x, M, [0, 0, 0, 0])
    xs = x.cpu().float()
    for k, c in enumerate(perm):
        assert torch.equal(out[0, c].cpu(), xs[0, :, :, k]), (k, c)


def test_color4x4_per_image_matrices(dev):
    """One transform per image ([B, 4, 4] + [B, 4]): every image equals the
    fp32 reference with its own matrix."""
    x = _imgs(5, 32, 64, 4, dev, seed=8)
    rng = np.random.default_rng(5)
    M = rng.uniform(-1, 1, size=(5, 4, 4)).astype(np.float32)
    b = rng.normal(size=(5, 4)).astype(np.float32)
    out = ops.color4x4(x, M, b, gamma=2.2)
    ref = ops.reference_color4x4(x.cpu(), M, b, gamma=2.2)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-3)
    for k in range(5):   # and each image alone through the one-matrix path
        one = ops.color4x4(x[k:k + 1], M[k], b[k], gamma=2.2)
        torch.testing.assert_close(out[k:k + 1], one, rtol=1e-5, atol=1e-3)


def test_color4x4_jitter_built_in_kernel(dev):
    """Colour jitter: the kernel builds each image's transform from its 4
    factors; it must equal reference_color4x4 with ops.color_jitter_matrix
    per image (atol 1e-3 on 0..255 values), identity factors included."""
    x = _imgs(6, 48, 64, 4, dev, seed=9)
    f = np.array([[1, 1, 1, 0], [1.3, 0.7, 1.4, 0.1], [0.6, 1.2, 0.5, -0.2], [1.0, 1.0, 0.0, 0.0],
                  [0.9, 1.4, 1.2, 0.5], [1.1, 0.9, 0.8, -0.05]], np.float32)
    out = ops.color4x4(x, jitter=f, gamma=2.2, pivot=127.5)
    mb = [ops.color_jitter_matrix(r, 127.5) for r in f]
    ref = ops.reference_color4x4(x.cpu(), np.stack([m for m, _ in mb]), np.stack([b for _, b in mb]), gamma=2.2)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-4, atol=1e-3)
    ident = ops.reference_color4x4(x[:1].cpu(), np.eye(4), [0] * 4, gamma=2.2)
    torch.testing.assert_close(out[:1].cpu(), ident, rtol=0, atol=1e-3)


@pytest.mark.parametrize('flip', [False, True])
def test_color4x4_full_frame(dev, flip):
    x = _imgs(3, 480, 640, 4, dev, seed=6)
    M = np.random.default_rng(2).uniform(-1, 1, size=(4, 4)).astype(np.float32)
    out = ops.color4x4(x, M, [0.5, -0.5, 0, 1], gamma=2.2, flip=flip)
    ref = ops.reference_color4x4(x, M, [0.5, -0.5, 0, 1], gamma=2.2, flip=flip)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-3)


def test_project_matches_reference(dev):
    rng = np.random.default_rng(1)
    pts = rng.normal(size=(1000, 3)).astype(np.float32)
    V = np.eye(4, dtype=np.float32)
    V[2, 3] = -7.0
    f = 50 / 36 * 2
    P = np.array([[f, 0, 0, 0], [0, f * 640 / 480, 0, 0], [0, 0, -1.2, -2.2], [0, 0, -1, 0]], np.float32)
    px, d = ops.project(torch.from_numpy(pts).to(dev), P @ V, V, 640, 480)
    rpx, rd = ops.reference_project(pts, (P @ V).astype(np.float64), V.astype(np.float64), 640, 480)
    torch.testing.assert_close(px.cpu().double(), rpx, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(d.cpu().double(), rd, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize('shape,out', [((8, 256, 30, 40), 4), ((2, 5, 7, 5), (3, 2)), ((1, 3, 3, 2), (5, 4)),
                                       ((2, 64, 16, 16), 4)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('channels_last', [True, False])
def test_adaptive_avg_pool_nhwc(dev, shape, out, dtype, channels_last):
    g = torch.Generator().manual_seed(3)
    x32 = torch.randn(shape, generator=g)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    x = x32.to(dev, dtype).to(memory_format=fmt).requires_grad_(True)
    y = ops.adaptive_avg_pool_nhwc(x, out)
    gy32 = torch.randn(y.shape, generator=g)
    y.backward(gy32.to(dev, dtype))
    xr = x32.to(dtype).float().requires_grad_(True)          # same (rounded) inputs, fp32 math
    yr = ops.reference_adaptive_avg_pool(xr, out)
    yr.backward(gy32.to(dtype).float())
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert y.shape == yr.shape and y.dtype == dtype
    assert torch.allclose(y.detach().float().cpu(), yr.detach(), atol=tol, rtol=tol)
    assert torch.allclose(x.grad.float().cpu(), xr.grad, atol=tol, rtol=tol)


def test_discriminator_pool_runs_hip_kernel(dev):
    from blendtorch.models import Discriminator
    net = Discriminator(adaptive=True).to(dev).to(memory_format=torch.channels_last)
    pool = [m for m in net.modules() if type(m).__name__ == 'AdaptiveAvgPool2d'][0]
    assert type(pool) is ops.AdaptiveAvgPool2d
    x = torch.rand(2, 3, 96, 128, device=dev).to(memory_format=torch.channels_last)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = net(x)
    out.float().sum().backward()
    assert out.shape == (2,) and torch.isfinite(out.float()).all()
    assert all(torch.isfinite(p.grad).all() for p in net.parameters())


@pytest.mark.parametrize('shape', [(8, 32, 60, 80), (4, 256, 15, 20), (3, 64, 7, 9), (2, 128, 1, 1),
                                   (8, 64, 120, 160), (2, 512, 6, 10)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('channels_last', [True, False])
def test_batch_norm_leaky_relu(dev, shape, dtype, channels_last):
    g = torch.Generator().manual_seed(5)
    C = shape[1]
    x32 = torch.randn(shape, generator=g) * 1.5 + 0.3
    w32 = torch.rand(C, generator=g) + 0.5
    b32 = torch.randn(C, generator=g) * 0.1
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    x = x32.to(dev, dtype).to(memory_format=fmt).requires_grad_(True)
    w = w32.to(dev).requires_grad_(True)
    b = b32.to(dev).requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    y = ops.batch_norm_leaky_relu(x, w, b, rm, rv, 1e-5, 0.1, 0.2)
    gy32 = torch.randn(y.shape, generator=g)
    y.backward(gy32.to(dev, dtype))

    xr = x32.to(dtype).float().requires_grad_(True)
    wr, br = w32.clone().requires_grad_(True), b32.clone().requires_grad_(True)
    rmr, rvr = torch.zeros(C), torch.ones(C)
    yr = ops.reference_batch_norm_leaky_relu(xr, wr, br, rmr, rvr, 1e-5, 0.1, 0.2)
    yr.backward(gy32.to(dtype).float())
    torch.cuda.synchronize()
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    assert y.shape == yr.shape and y.dtype == dtype
    assert torch.allclose(y.detach().float().cpu(), yr.detach(), atol=tol, rtol=tol)
    assert torch.allclose(rm.cpu(), rmr, atol=1e-4, rtol=1e-4)
    assert torch.allclose(rv.cpu(), rvr, atol=1e-4, rtol=1e-4)
    gtol = 1e-3 if dtype == torch.float32 else 5e-2
    # elements at the LeakyReLU kink (pre-activation ~ 0) may take either
    # slope: bf16 inputs repeat the same grid values thousands of times, so one
    # value whose z rounds across 0 flips them all.  Compare the data gradient
    # away from the kink (the flips still enter dw/db sums, within tolerance).
    with torch.no_grad():
        z = torch.nn.functional.batch_norm(xr.detach(), None, None, wr.detach(), br.detach(), training=True, eps=1e-5)
    away = z.abs() > 1e-2
    assert torch.allclose(x.grad.float().cpu()[away], xr.grad[away], atol=gtol, rtol=gtol)
    assert torch.allclose(w.grad.cpu(), wr.grad, atol=gtol * C, rtol=gtol)
    assert torch.allclose(b.grad.cpu(), br.grad, atol=gtol * C, rtol=gtol)


def test_discriminator_fused_matches_unfused(dev):
    from blendtorch.models import Discriminator
    torch.manual_seed(0)
    a = Discriminator(adaptive=True).to(dev).to(memory_format=torch.channels_last)
    b = Discriminator(adaptive=True, fused=False).to(dev).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 96, 128, device=dev).to(memory_format=torch.channels_last)
    ya, yb = a(x), b(x)
    ya.sum().backward()
    yb.sum().backward()
    torch.cuda.synchronize()
    assert torch.allclose(ya, yb, atol=1e-4, rtol=1e-4)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa.grad, pb.grad, atol=1e-3, rtol=1e-2), n
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert torch.allclose(ba.float(), bb.float(), atol=1e-4, rtol=1e-4), n


@pytest.mark.parametrize('copies', ['16', '32'])
def test_decode_forced_arithmetic_transform_bit_exact(monkeypatch, copies):
    """BLENDTORCH_DECODE_XFORM=1: the verified arithmetic value transform with
    a lane-private gamma table (no LDS bank conflicts) is bit-exact with the
    fp32 reference for gamma, normalisation (reciprocal + fma correction) and
    raw configs, in the stream decode, the gather decode and the replay sample."""
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    monkeypatch.setenv('BLENDTORCH_DECODE_XFORM', '1')
    monkeypatch.setenv('BLENDTORCH_GAMMA_COPIES', copies)
    monkeypatch.setattr(ops, '_lut_cache', {})
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.randint(0, 256, (6, 48, 64, 4), dtype=torch.uint8, device=dev, generator=g)
    cfgs = [ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
            ops.DecodeConfig.unit(channels='rgba', gamma=1.8, dtype='bfloat16', layout='nhwc'),
            ops.DecodeConfig(channels='bgr', mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), scale=1 / 255),
            ops.DecodeConfig.raw(channels='rgb')]
    for cfg in cfgs:
        assert ops.build_table(cfg)[ops.XF_HEADER] == 1.0
        ref = ops.reference_decode(x.cpu(), cfg)
        assert torch.equal(ops.decode(x, cfg).cpu(), ref), cfg
        idx = torch.tensor([5, 0, 3], device=dev)
        assert torch.equal(ops.decode_gather(x, idx, cfg).cpu(), ref[idx.cpu()]), cfg
        out, got_idx, _ = ops.replay_sample(x, 6, 4, cfg, seed=3, counter=11)
        assert torch.equal(out.cpu(), ref[got_idx.cpu()]), cfg
    y = ops.color4x4(x, np.eye(4), gamma=2.2)
    torch.testing.assert_close(y.cpu(), ops.reference_color4x4(x.cpu(), np.eye(4), [0] * 4, gamma=2.2),
                               rtol=0, atol=0)
