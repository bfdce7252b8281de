"""Consumer models used by the examples and the benchmark (random init).

* :class:`Discriminator` -- the DCGAN image discriminator of the densityopt
  example (reference: examples/densityopt/densityopt.py:139-190): 4x
  [conv4x4/s2 -> BN -> LeakyReLU(0.2)] then conv4x4 -> sigmoid, ndf=32, for
  64x64 inputs.  ``adaptive=True`` inserts a global pooling head so the same
  stack scores 640x480 Cube frames (used by ``bench.py --consumer disc``).
* :class:`ProbModel` -- LogNormal simulation-parameter model trained with the
  score-function gradient (densityopt.py:30-93).
* :class:`CartpolePolicy` -- the P-controller of examples/control/cartpole.py
  as a batched GPU module.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.distributions as D


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _weights_init(m):
    name = m.__class__.__name__
    if 'Conv' in name:
        nn.init.normal_(m.weight, 0.0, 0.02)
    elif 'BatchNorm' in name:
        nn.init.normal_(m.weight, 1.0, 0.02)
        nn.init.zeros_(m.bias)


def _env_flag(name, default):
    v = os.environ.get(name)
    return default if v is None or v == '' else v not in ('0', 'false', 'False', 'off')


class Discriminator(nn.Module):
    """DCGAN discriminator: N x nc x H x W -> N probabilities."""

    # bf16 path with raw u8 frames (decode fused into the first conv): the first
    # BN's backward apply runs inside the first conv's weight-gradient kernel
    # (ops.BnDeferred); False keeps the separate apply launch (A/B, tests)
    defer_first_bn = True
    # Where the BatchNorm+LeakyReLU applies run (profiles/r4/bn_placement.md has the per-kernel A/B):
    # the last BN's forward apply in the fused head's pooling (ops.BnActLazy): -6.4 us per step
    lazy_head_bn = _env_flag('BT_LAZY_HEAD_BN', True)
    # the other forward applies in the next MFMA convolution's operand staging: measured +15 us
    # per step (each such convolution doubles; its per-k-step rewrite of the staged tile sits
    # between the stage's arrival and the barrier of latency-bound k-loops), so off by default
    lazy_conv_bn = _env_flag('BT_LAZY_CONV_BN', False)
    # every backward apply in the producing convolution's weight gradient (in-kernel fold, gx side
    # output): measured +9 us per step against the apply launches, so off by default (the first
    # layer, which has no data gradient, always takes its BN's backward: defer_first_bn)
    defer_bn_bwd = _env_flag('BT_DEFER_BN_BWD', False)
    # the first BN's forward apply in the u8 first layer's own kernel, after a grid barrier on its
    # statistics (ops.BnProduced): no apply launch, no second read of the layer's output.  Measured
    # slower (conv1 24.7 + 11.6 us -> 60.3 us: the barrier's tail and the 2-waves-per-SIMD launch,
    # profiles/r5/b14), so off by default
    conv1_bn = _env_flag('BT_CONV1_BN', False)
    # the same for the other layers whose forward grid fits on the chip at once (ops.conv_out_bn_fits),
    # except the last BN, which the fused head applies (lazy_head_bn: no activation written at all);
    # conv3 20.2 + 9.3 -> 46.0 us (profiles/r5/b14), off by default
    conv_out_bn = _env_flag('BT_CONV_OUT_BN', False)

    def __init__(self, nc=3, ndf=32, adaptive=False, fused=True):
        super().__init__()
        from .. import ops
        layers = []
        cin = nc
        for i, mult in enumerate((1, 2, 4, 8)):
            if fused:
                # BN + LeakyReLU as one gfx950 op on GPU training steps (7 MIOpen/PyTorch
                # kernels -> 3 forward + 3 backward); the Identity keeps the module
                # indices, so state dicts match the unfused stack
                norm_act = [ops.BatchNormLeakyReLU2d(ndf * mult, slope=0.2), nn.Identity()]
            else:
                norm_act = [nn.BatchNorm2d(ndf * mult), nn.LeakyReLU(0.2, inplace=True)]
            layers += [nn.Conv2d(cin, ndf * mult, 4, 2, 1, bias=False)] + norm_act
            cin = ndf * mult
        if adaptive:
            # gfx950 NHWC pooling kernels on the GPU (PyTorch's NHWC adaptive pool
            # took ~100 us of a 1.2 ms training step, profiles/consumer_step.md)
            layers += [ops.AdaptiveAvgPool2d(4)]
        layers += [nn.Conv2d(cin, 1, 4, 1, 0, bias=False), nn.Sigmoid()]
        self.features = nn.Sequential(*layers)
        self.apply(_weights_init)

    def forward(self, x):
        return self.features(x).view(-1, 1).squeeze(1)

    def use_optimizer_shadows(self, opt):
        """Read the bf16 conv weights (and their data-gradient transposes)
        from ``opt``'s shadows (``ops.FusedAdam.enable_conv_shadows``: the
        update kernel rewrites them) instead of casting and transposing the
        fp32 weights in two launches every step.  Only the 4x4 / stride-2
        layers (the MFMA path, whose weight gradient goes to the fp32 weight
        directly) use them.  ``opt=None`` switches back."""
        self._shadow_opt = None
        if opt is not None:
            ws = [m.weight for m in self.features if isinstance(m, nn.Conv2d) and m.stride == (2, 2)
                  and tuple(m.kernel_size) == (4, 4)]
            # the first layer's input is the batch: no data gradient, no transpose
            opt.enable_conv_shadows(ws, transpose=[i > 0 for i in range(len(ws))])
            self._shadow_opt = opt

    def forward_bf16(self, x, mfma=True):
        """bf16 forward without autocast.  ``x`` may carry a 4th (alpha)
        channel that the first convolution ignores (RGBA-decoded frames feed
        its MFMA kernel directly; ``mfma`` only).  ONE kernel casts every conv weight
        to bf16 (and one casts their gradients back to fp32 in backward)
        instead of a cast per layer each way; numerically the same as
        ``autocast(bfloat16)`` over :meth:`forward` (RNE weight casts, bf16
        activations).  ``x``: bf16 on the GPU.

        ``mfma``: the 4x4/s2 layers whose channels fit (Cin % 32, Cout % 64:
        all but the first) run on the gfx950 MFMA conv kernels
        (``ops.conv4x4s2``): forward, and the weight gradient in fp32 instead
        of MIOpen's bf16 path (zero-fill + atomic GEMM + cast per layer).
        ``mfma=False`` is bit-identical to autocast over :meth:`forward`."""
        return self._run_bf16(x, list(self.features), mfma).view(-1, 1).squeeze(1)

    def bce_loss_bf16(self, x, target=1.0, mfma=True, decode=None):
        """Mean binary cross-entropy of :meth:`forward_bf16`'s output against
        ``target`` (scalar or [N]), with the head (pool -> 4x4 conv -> sigmoid
        -> BCE) fused into ``ops.disc_head_bce`` (2 launches forward, 2
        backward, instead of ~20 library kernels; fp32 weight and gradient).
        Falls back to :meth:`forward_bf16` + ``BCELoss`` off that shape.
        ``decode`` (an RGBA ``ops.DecodeConfig``): ``x`` is the RAW u8 RGBA
        frames ([N, 4, H, W] channels-last, i.e. NHWC bytes) and the first
        convolution decodes them inside its MFMA kernels' loads -- the same
        values as ``ops.decode`` to bf16 NHWC, without the decode pass and its
        bf16 copy of the batch.  Returns the loss."""
        return self.bce_bf16(x, target, mfma, probs=False, decode=decode)[0]

    def bce_bf16(self, x, target=1.0, mfma=True, probs=True, decode=None):
        """``(mean BCE loss, per-sample probabilities)`` of the bf16 forward
        (``probs=False``: the fused head's logits are not turned into
        probabilities -- one kernel fewer when only the loss is used;
        ``probs='logits'``: the fused head's fp32 logits instead, for a
        consumer that applies the sigmoid itself).

        The fused head applies to the adaptive stack (pool -> conv -> sigmoid)
        and to the plain DCGAN stack whose last conv consumes the whole
        feature map (densityopt's 64x64 model: 4x4 features, 4x4 kernel --
        the head kernel's pooling is then the identity)."""
        import torch.nn.functional as F
        from .. import ops
        layers = list(self.features)
        head = body = pool = None
        adaptive = (len(layers) >= 3 and isinstance(layers[-3], ops.AdaptiveAvgPool2d)
                    and isinstance(layers[-2], nn.Conv2d) and isinstance(layers[-1], nn.Sigmoid)
                    and tuple(layers[-2].kernel_size) == _pair(layers[-3].output_size))
        if adaptive:
            head, body, pool = layers[-2], layers[:-3], _pair(layers[-3].output_size)
        elif len(layers) >= 2 and isinstance(layers[-2], nn.Conv2d) and isinstance(layers[-1], nn.Sigmoid):
            head, body, pool = layers[-2], layers[:-2], tuple(layers[-2].kernel_size)
        ok = (head is not None and x.is_cuda and head.out_channels == 1 and head.bias is None
              and head.stride == (1, 1) and head.padding == (0, 0) and head.groups == 1
              and head.in_channels % 8 == 0)
        lut = None
        if decode is not None:
            if not (ok and mfma and x.dtype == torch.uint8):
                raise ValueError('bce_bf16(decode=): raw u8 RGBA frames on the fused-head MFMA path only')
            lut = ops.decode_lut_bf16(decode, x.device)
        if ok:
            # adaptive stack: the last BN's apply runs in the head's pooling (BnActLazy)
            z, link, lazy = self._run_bf16(x, body, mfma, want_link=True, lut=lut, want_lazy=True,
                                           lazy_tail=adaptive and self.lazy_head_bn)
            if adaptive or tuple(z.shape[2:]) == pool:
                if not z.is_contiguous(memory_format=torch.channels_last):
                    if lazy is not None:
                        raise RuntimeError('bce_bf16: the lazily applied BN input is not channels-last')
                    z, link = z.contiguous(memory_format=torch.channels_last), None
                loss, logits = ops.disc_head_bce(z, head.weight, target, pool, bn_link=link, act=lazy)
                if probs == 'logits':
                    return loss, logits
                return loss, (torch.sigmoid(logits) if probs else None)
            out = self._run_bf16(z, layers[len(body):], mfma)
        else:
            out = self._run_bf16(x, layers, mfma)
        out = out.reshape(-1).float()
        tgt = target if isinstance(target, torch.Tensor) else torch.full_like(out, float(target))
        return F.binary_cross_entropy(out, tgt), out

    @staticmethod
    def _conv_applies_bn(x, layers, j, mfma):
        """True when layers[j] is an MFMA convolution that can apply the
        BatchNorm+LeakyReLU producing its input ``x`` in its own operand
        staging (ops.BnActLazy): the accumulator-statistics path (a fused BN
        follows it) on a bf16 input of 8-128 channels."""
        from .. import ops
        if not mfma or j >= len(layers) or not isinstance(layers[j], nn.Conv2d):
            return False
        m = layers[j]
        nxt = layers[j + 1] if j + 1 < len(layers) else None
        cin = m.in_channels
        # even input sides: the centre taps that write the activation cover every input row / column
        return (x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and m.stride == (2, 2) and m.padding == (1, 1) and m.bias is None and m.groups == 1
                and m.dilation == (1, 1) and tuple(m.kernel_size) == (4, 4) and ops.conv_wgrad_supported(x, m.weight)
                and 8 <= cin <= 128 and cin & (cin - 1) == 0 and m.out_channels % 32 == 0
                and isinstance(nxt, ops.BatchNormLeakyReLU2d) and ops.bn_acc_supported(m.out_channels)
                and nxt.fused_with_stats(x.new_empty((1, m.out_channels, 1, 1), dtype=torch.bfloat16)))

    def _run_bf16(self, x, layers, mfma, want_link=False, lut=None, lazy_tail=False, want_lazy=False):
        import torch.nn.functional as F
        from .. import ops
        convs = [m for m in layers if isinstance(m, nn.Conv2d)]
        shadows = self.__dict__.get('_shadow_opt') if (mfma and x.is_cuda) else None
        # with optimizer shadows only the layers off the MFMA path are cast (usually none)
        w16s = ops.cast_bf16(*[c.weight for c in convs]) if shadows is None else None
        weights = iter(w16s) if w16s is not None else None
        # data-gradient operands of the MFMA layers that need one (not the first:
        # its input is the batch), transposed in one launch per step
        wts = {}
        if shadows is None and mfma and torch.is_grad_enabled() and x.is_cuda:
            need = [k for k, c in enumerate(convs) if k > 0 and c.in_channels % 32 == 0 and c.stride == (2, 2)
                    and tuple(c.kernel_size) == (4, 4) and c.out_channels % 32 == 0]
            if need:
                wts = dict(zip(need, ops.conv_weights_t([w16s[k] for k in need])))
        ci = -1
        stats = link = defer = lazy = act_next = early = None
        # the MFMA weight gradients of one backward hand their slice reduce to the
        # next one (ops.WgradChain): the first such layer's runs last and closes it
        wchain = ops.WgradChain() if (mfma and torch.is_grad_enabled() and x.is_cuda) else None
        first_mfma = True
        for i, m in enumerate(layers):
            if isinstance(m, nn.Conv2d):
                ci += 1
                on_mfma = (mfma and m.stride == (2, 2) and m.padding == (1, 1) and m.bias is None
                           and m.groups == 1 and m.dilation == (1, 1) and ops.conv_wgrad_supported(x, m.weight))
                if shadows is None:
                    w16 = next(weights)
                elif on_mfma and 'shadow' in shadows.state.get(m.weight, {}):
                    w16 = shadows.shadow(m.weight)
                    if ci > 0 and torch.is_grad_enabled():
                        wts[ci] = shadows.shadow_t(m.weight)
                else:
                    w16 = ops.cast_bf16(m.weight)[0]
                if on_mfma:
                    nxt = layers[i + 1] if i + 1 < len(layers) else None
                    fuse = (isinstance(nxt, ops.BatchNormLeakyReLU2d) and ops.conv_fwd_supported(x, w16)
                            and nxt.fused_with_stats(x.new_empty((1, m.out_channels, 1, 1), dtype=torch.bfloat16)))
                    # the BN that produced x: this conv's data gradient does its backward reduction
                    bl, link = link, None
                    # the chain closes at the first MFMA layer whose weight takes a gradient:
                    # its backward node exists whatever the input, so the deferred reduces
                    # handed down to it always run (frozen layers flush, see ops.conv4x4s2)
                    closes = first_mfma and m.weight.requires_grad
                    wk = dict(wt=wts.get(ci), bn_link=bl, wchain=wchain, wlast=closes)
                    if act_next is not None:   # x is the previous BN's input: apply it in the staging
                        wk['act'], act_next = act_next, None
                    if ci == 0 and lut is not None:
                        wk['lut'] = lut    # raw u8 frames: decoded in this layer's kernels
                    if (fuse and torch.is_grad_enabled() and ops.bn_acc_supported(m.out_channels)
                            and (self.defer_bn_bwd or (ci == 0 and lut is not None and self.defer_first_bn))):
                        # the following BN's backward apply runs inside this layer's
                        # weight-gradient kernel (ops.BnDeferred / BnBwdFold): it folds the
                        # BN's backward sums, applies the BN backward to the staged dY and
                        # writes the BN's input gradient for this layer's data gradient
                        defer = wk['bn_out'] = ops.BnDeferred()
                    if closes:
                        first_mfma = False
                    if fuse and ops.bn_acc_supported(m.out_channels) and not self.lazy_conv_bn:
                        # the BN applied in this layer's kernel when its grid fits (ops.BnProduced) --
                        # not the BN the caller's consumer applies (lazy_tail)
                        j2 = i + 2
                        while j2 < len(layers) and isinstance(layers[j2], nn.Identity):
                            j2 += 1
                        first = ci == 0 and lut is not None
                        if (self.conv1_bn if first else self.conv_out_bn) and not (lazy_tail and j2 == len(layers)):
                            early = wk['bn_early'] = nxt.produced_by_conv(x.device)
                    if fuse and ops.bn_acc_supported(m.out_channels):
                        # BN statistics come out of the conv kernel's epilogue, added into
                        # the BN call's zeroed accumulator (its apply kernel folds them)
                        stats = nxt.accumulator(x.device)
                        x = ops.conv4x4s2(x, m.weight, w16, with_stats=stats, **wk)
                    elif fuse:   # per-tile partial rows + a finalize launch
                        x, stats = ops.conv4x4s2(x, m.weight, w16, with_stats=True, **wk)
                    else:
                        x = ops.conv4x4s2(x, m.weight, w16, **wk)
                else:
                    if ci == 0 and lut is not None:
                        raise ValueError('raw u8 frames need the MFMA first layer')
                    if act_next is not None:
                        raise RuntimeError('_run_bf16: a lazily applied BN feeds a layer off the MFMA path')
                    link = None
                    x = F.conv2d(x, w16, None, m.stride, m.padding, m.dilation, m.groups)
            elif stats is not None and isinstance(m, ops.BatchNormLeakyReLU2d):
                link = ops.BnLink() if torch.is_grad_enabled() else None
                acc_bf16 = isinstance(stats, ops.BnAccumulator) and x.dtype == torch.bfloat16
                j = i + 1   # the consumer: the next layer that is not an Identity
                while j < len(layers) and isinstance(layers[j], nn.Identity):
                    j += 1
                if lazy_tail and j == len(layers) and acc_bf16:
                    lazy = ops.BnActLazy()   # the caller's consumer applies this BN
                elif acc_bf16 and self.lazy_conv_bn and self._conv_applies_bn(x, layers, j, mfma):
                    lazy = act_next = ops.BnActLazy()   # the next convolution applies this BN
                if early is not None and early.y is not None:
                    lazy, act_next = early, None   # the first convolution applied this BN (ops.BnProduced)
                x = m.forward_from_stats(x, stats, link, defer, lazy)
                if lazy is act_next or lazy is early:
                    lazy = None
                stats = defer = early = None
            else:
                if not isinstance(m, nn.Identity):
                    link = None
                x = m(x)
        # want_link: also the BnLink of a BN whose output is returned (its consumer
        # -- the fused head -- can then do that BN's backward reduction), and with
        # want_lazy the BnActLazy of that BN when lazy_tail let it skip its apply
        # (None: x is the BN's output, not its input)
        if want_lazy:
            return x, link, lazy
        return (x, link) if want_link else x


class ProbModel(nn.Module):
    """Independent LogNormal distributions over the supershape frequencies
    (m1, m2) (densityopt.py:30-93).

    ``m1m2_mean`` is the LogNormal ``loc`` (mean of log m) and
    ``m1m2_log_std`` the log of its scale, both optimised with the
    score-function (REINFORCE) gradient
    ``grad E[f(x)] = E[(f(x) - b) grad log p(x)]``.
    """

    def __init__(self, m1m2_mean, m1m2_std):
        super().__init__()
        self.m1m2_mean = nn.Parameter(torch.as_tensor(m1m2_mean).float(), requires_grad=True)
        self.m1m2_log_std = nn.Parameter(torch.log(torch.as_tensor(m1m2_std).float()), requires_grad=True)

    @property
    def dists(self):
        # built on the fly so autograd sees fresh graphs every step; no argument
        # validation: its checks read device values back (a host sync per call,
        # and not capturable in a HIP graph)
        return (D.LogNormal(self.m1m2_mean[0], torch.exp(self.m1m2_log_std[0]), validate_args=False),
                D.LogNormal(self.m1m2_mean[1], torch.exp(self.m1m2_log_std[1]), validate_args=False))

    def sample(self, n):
        """``n`` draws of (m1, m2): ``exp(mean + std * eps)``, eps ~ N(0, 1) --
        the LogNormal's sample written out (torch.normal with tensor
        arguments checks ``std >= 0`` on the host, which is a device sync and
        cannot be captured in a HIP graph)."""
        with torch.no_grad():
            eps = torch.randn(2, n, device=self.m1m2_mean.device)
            m = torch.exp(self.m1m2_mean.detach()[:, None] + torch.exp(self.m1m2_log_std.detach())[:, None] * eps)
        return {'m1': m[0], 'm2': m[1]}

    def log_prob(self, samples):
        m1, m2 = self.dists
        return m1.log_prob(samples['m1']) + m2.log_prob(samples['m2'])

    def readable_params(self):
        return torch.cat([self.m1m2_mean.detach(), torch.exp(self.m1m2_log_std).detach()])

    @staticmethod
    def to_supershape(samples):
        """(N, 2, 6) supershape params: rows (m, a=1, b=1, n1=n2=n3=3), m from the samples."""
        n = samples['m1'].shape[0]
        params = samples['m1'].new_tensor([[0, 1, 1, 3, 3, 3], [0, 1, 1, 3, 3, 3]]).float().view(1, 2, 6).repeat(n, 1, 1)
        params[:, 0, 0] = samples['m1'].detach()
        params[:, 1, 0] = samples['m2'].detach()
        return params


class CartpolePolicy(nn.Module):
    """Proportional controller ``a = kappa * (pole_x - cart_x)`` for a batch
    of observations ``(cart_x, pole_x, pole_angle)`` (examples/control/
    cartpole.py:17-36), evaluated on the GPU for many envs at once."""

    def __init__(self, kappa=30.0):
        super().__init__()
        self.register_buffer('kappa', torch.tensor(float(kappa)))

    def forward(self, obs):
        return self.kappa * (obs[..., 1] - obs[..., 0])
