"""Diagnostic: the u8 first layer with its BN applied in-kernel (conv_fwd
out_bn=, grid barrier) against the same layer + the BN apply launch, on the
same frames: z, mean / invstd and the activation compared element by
element.  Prints one JSON line per shape."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402

from blendtorch import ops  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    ext = ops.hip_ext()
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    lut = ops.decode_lut_bf16(cfg, dev)
    cl = torch.channels_last
    for N, H, W in [(4, 96, 128), (3, 100, 136), (8, 480, 640)]:
        g = torch.Generator(device=dev).manual_seed(1)
        xu8 = torch.randint(0, 256, (N, H, W, 4), dtype=torch.uint8, device=dev, generator=g).permute(0, 3, 1, 2)
        w16 = (0.1 * torch.randn(32, 3, 4, 4, device=dev, generator=g)).to(torch.bfloat16).contiguous(memory_format=cl)
        bn = ops.BatchNormLeakyReLU2d(32).to(dev)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5, generator=g)
            bn.bias.uniform_(-0.2, 0.2, generator=g)
        acc1 = ops.BnAccumulator(32, dev)
        early = bn.produced_by_conv(dev)
        t0 = ops.conv_grid_barrier_timeouts()
        z1 = ops.conv_fwd(xu8, w16, acc1.fwd, acc1.R, lut=lut, out_bn=early)
        torch.cuda.synchronize()
        applied = early.y is not None
        y1 = early.y.permute(0, 2, 3, 1).contiguous() if applied else None
        m1, s1 = early.mean.clone(), early.invstd.clone()
        acc2 = ops.BnAccumulator(32, dev)
        z2 = ops.conv_fwd(xu8, w16, acc2.fwd, acc2.R, lut=lut)
        zs = z2.permute(0, 2, 3, 1).contiguous()
        y2 = torch.empty_like(zs)
        m2 = torch.empty(32, device=dev)
        s2 = torch.empty(32, device=dev)
        M = zs.numel() // 32
        w = bn.weight.detach().float().contiguous()
        b = bn.bias.detach().float().contiguous()
        ext.bn_forward_acc(zs.data_ptr(), y2.data_ptr(), M, 32, ops.OUT_DTYPES['bfloat16'], acc2.fwd.data_ptr(),
                           acc2.R, 1e-5, 0.1, m2.data_ptr(), s2.data_ptr(), 0, 0, w.data_ptr(), b.data_ptr(), 0.2,
                           ops._stream(dev), 0)
        torch.cuda.synchronize()
        res = {'shape': [N, H, W], 'applied': applied, 'timeouts': ops.conv_grid_barrier_timeouts() - t0,
               'z_equal': bool(torch.equal(z1, z2)),
               'mean_maxdiff': float((m1 - m2).abs().max()), 'invstd_maxdiff': float((s1 - s2).abs().max()),
               'acc1_zero': int(torch.count_nonzero(acc1.fwd)) == 0, 'acc2_zero': int(torch.count_nonzero(acc2.fwd)) == 0}
        if applied:
            d = (y1.float() - y2.float()).abs()
            res['y_equal'] = bool(torch.equal(y1, y2))
            res['y_maxdiff'] = float(d.max())
            res['y_ndiff'] = int((d > 0).sum())
            if res['y_ndiff']:
                idx = torch.nonzero(d.reshape(-1, 32) > 0)
                res['diff_channels'] = sorted(set(int(c) for c in idx[:, 1].tolist()))[:32]
                pix = idx[:, 0]
                res['diff_pixels_first'] = pix[:8].tolist()
                res['diff_pixels_count'] = int(pix.unique().numel())
                res['y1_zero_frac'] = float((y1 == 0).float().mean())
        print(json.dumps(res), flush=True)


if __name__ == '__main__' and len(sys.argv) == 1:
    main()


def model_diag():
    """The disc forward with the first BN in the conv kernel against the apply
    launch: every BN call's output and the loss."""
    from blendtorch.models import Discriminator
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    cfg = ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc')
    g = torch.Generator(device=dev).manual_seed(4)
    xu8 = torch.randint(0, 256, (3, 96, 128, 4), dtype=torch.uint8, device=dev, generator=g).permute(0, 3, 1, 2)
    torch.manual_seed(2)
    a = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=cl)
    b.load_state_dict(a.state_dict())
    a.conv1_bn, b.conv1_bn = True, False
    a.conv_out_bn = b.conv_out_bn = False
    rec = []
    orig = ops._bn_apply_unchecked

    def wrap(x, *args):
        y = orig(x, *args)
        rec.append((x.detach().clone(), y.detach().clone()))
        return y
    ops._bn_apply_unchecked = wrap
    la = a.bce_loss_bf16(xu8, 1.0, decode=cfg)
    ra, rec[:] = list(rec), []
    lb = b.bce_loss_bf16(xu8, 1.0, decode=cfg)
    rb = list(rec)
    ops._bn_apply_unchecked = orig
    out = {'la': float(la), 'lb': float(lb), 'calls': [len(ra), len(rb)]}
    for k, ((xa, ya), (xb, yb)) in enumerate(zip(ra, rb)):
        out[f'bn{k + 1}'] = {'x_equal': bool(torch.equal(xa, xb)), 'y_equal': bool(torch.equal(ya, yb)),
                             'y_maxdiff': float((ya.float() - yb.float()).abs().max()),
                             'shape_a': list(ya.shape), 'stride_a': list(ya.stride()),
                             'shape_b': list(yb.shape), 'stride_b': list(yb.stride())}
    print(json.dumps(out), flush=True)


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'model':
    model_diag()
