"""Hand-written gfx950 kernels for the image path, with fp32 PyTorch references.

The reference does all of this with numpy on the CPU, per item, inside
DataLoader workers:

* vertical flip to the upper-left origin   -- ``btb/offscreen.py:95-96``
* gamma "linear->sRGB" ``u8(255*(x/255)**(1/g))``, alpha untouched
                                           -- ``btb/offscreen.py:105-112``,
                                              ``examples/datagen/generate.py:10-14``
* RGBA -> RGB channel select               -- ``btb/offscreen.py:57-62``
* normalize ``(x-127.5)/127.5`` + HWC->CHW -- ``examples/densityopt/densityopt.py:117-119``
* batch collate                            -- torch ``default_collate``

Here they are one fused HIP kernel over a whole batch (:func:`decode`), plus
a per-pixel 4x4 colour transform on the MFMA units (:func:`color4x4`) and
batched pinhole projection (:func:`project`, ``btb/camera.py:84-162``).

Every kernel has a plain-PyTorch fp32 reference (``reference_*``) used by the
numerics tests.  On a machine with a GPU the HIP extension MUST load:
:func:`hip_ext` raises instead of silently falling back.
"""
from __future__ import annotations

import dataclasses
import importlib
import os
from typing import Optional, Sequence

import numpy as np

__all__ = [
    'DecodeConfig', 'ColorJitter', 'color_jitter_matrix', 'jitter_factors', 'hip_ext', 'hip_available', 'gamma_lut', 'build_lut', 'build_table', 'decode', 'decode_gather',
    'color4x4',
    'project', 'adaptive_avg_pool_nhwc', 'AdaptiveAvgPool2d', 'batch_norm_leaky_relu', 'BatchNormLeakyReLU2d',
    'reference_decode', 'reference_color4x4', 'reference_project', 'reference_gamma',
]

OUT_DTYPES = {'float32': 0, 'bfloat16': 1, 'float16': 2, 'uint8': 3}
LAYOUTS = {'nchw': 0, 'nhwc': 1}

_hip = None
_hip_error = None


def hip_ext():
    """Return the loaded ``blendtorch._hip`` extension (gfx950 kernels).

    Importing torch first makes the extension bind to the HIP runtime torch
    already loaded (same ``libamdhip64.so.7`` soname).
    """
    global _hip, _hip_error
    if _hip is not None:
        return _hip
    import torch  # noqa: F401  (load torch's HIP runtime first)
    try:
        _hip = importlib.import_module('blendtorch._hip')
    except ImportError as e:  # pragma: no cover - depends on build state
        _hip_error = e
        raise ImportError(
            'blendtorch HIP extension is not built; run `python -m blendtorch._build` '
            f'(hipcc --offload-arch=gfx950): {e}') from e
    return _hip


def hip_available():
    """True when a GPU is visible AND the HIP extension loads."""
    import torch
    if not torch.cuda.is_available():
        return False
    hip_ext()
    return True


# ---------------------------------------------------------------------------
# LUT construction (host, numpy float32 -- bit-exact with the references)
# ---------------------------------------------------------------------------
def gamma_lut(gamma: Optional[float]) -> np.ndarray:
    """uint8[256] table of the reference's gamma correction.

    Same float32 expression as ``OffScreenRenderer._color_correct``
    (``btb/offscreen.py:105-112``): ``np.uint8(255.0 * (x/255)**(1/g))``,
    i.e. truncation, pure power law (not piecewise sRGB).
    """
    x = np.arange(256, dtype=np.float32)
    if not gamma:
        return x.astype(np.uint8)
    rgb = x / 255
    return np.uint8(255.0 * rgb ** (1 / gamma))


@dataclasses.dataclass(frozen=True)
class ColorJitter:
    """Random photometric augmentation on the loader's MFMA colour kernel.

    Every image draws brightness, contrast and saturation factors uniformly
    from ``[max(0, 1 - r), 1 + r]`` and a hue shift from ``[-hue, hue]``
    (turns), from a seeded stream in arrival order; each batch reports the
    factors it was decoded with (``batch['color_jitter']``, [B, 4]).  The
    transform of one image is the affine map of :func:`color_jitter_matrix`
    applied to ``gamma(x) * scale``; ``pivot`` (default: mid-grey in output
    units, 127.5 * scale) is the contrast pivot.  The reference has no such
    stage: it generalises the per-image colour handling of
    ``btb/offscreen.py:105-112`` to augmentation at PCIe rate.
    """
    brightness: float = 0.0
    contrast: float = 0.0
    saturation: float = 0.0
    hue: float = 0.0
    seed: int = 0
    pivot: Optional[float] = None

    def __post_init__(self):
        for f in ('brightness', 'contrast', 'saturation'):
            if getattr(self, f) < 0:
                raise ValueError(f'ColorJitter.{f} must be >= 0')
        if not 0.0 <= self.hue <= 0.5:
            raise ValueError('ColorJitter.hue must be in [0, 0.5]')


def jitter_factors(seed: int, ranges, n: int) -> np.ndarray:
    """float32 [n, 4]: the colour-jitter factors the stream loader draws for
    its first ``n`` images (csrc/gpu/loader.cpp, splitmix64 in arrival
    order): brightness, contrast, saturation in ``[max(0, 1 - r), 1 + r]``,
    hue in ``[-r, r]`` turns, for ``ranges`` = (r_b, r_c, r_s, r_h)."""
    M64 = (1 << 64) - 1
    state = (int(seed) * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & M64
    out = np.zeros((n, 4), np.float32)
    for i in range(n):
        for k in range(4):
            state = (state + 0x9E3779B97F4A7C15) & M64
            z = state
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            z ^= z >> 31
            u = np.float32(z >> 40) * np.float32(1.0 / 16777216.0)
            r = np.float32(ranges[k])
            lo = max(np.float32(0.0), np.float32(1.0) - r) if k < 3 else -r
            hi = np.float32(1.0) + r if k < 3 else r
            out[i, k] = np.float32(lo) + (np.float32(hi) - np.float32(lo)) * u
    return out


_LUMA = np.array([0.213, 0.715, 0.072])


def color_jitter_matrix(factors, pivot=0.5):
    """(M [4, 4], bias [4]) float32 of the colour jitter ``factors`` =
    (brightness b, contrast c, saturation s, hue h in turns), as the loader's
    kernel builds it (csrc/gpu/kernels.hip ``color_row``):
    ``rgb' = b c (Hue(h) Sat(s)) rgb + (1 - c) pivot``, alpha unchanged, with
    ``Sat(s) = s I + (1 - s) 1 w^T`` and ``Hue`` the rotation about the grey
    axis (luminance ``w = (0.213, 0.715, 0.072)``).  Both keep grey grey."""
    b, c, s, h = (float(v) for v in factors)
    cs, sn = np.cos(2 * np.pi * h), np.sin(2 * np.pi * h)
    hue = np.array([
        [0.213 + cs * 0.787 - sn * 0.213, 0.715 - cs * 0.715 - sn * 0.715, 0.072 - cs * 0.072 + sn * 0.928],
        [0.213 - cs * 0.213 + sn * 0.143, 0.715 + cs * 0.285 + sn * 0.140, 0.072 - cs * 0.072 - sn * 0.283],
        [0.213 - cs * 0.213 - sn * 0.787, 0.715 - cs * 0.715 + sn * 0.715, 0.072 + cs * 0.928 + sn * 0.072]])
    sat = s * np.eye(3) + (1 - s) * np.outer(np.ones(3), _LUMA)
    M = np.eye(4)
    M[:3, :3] = b * c * (hue @ sat)
    bias = np.zeros(4)
    bias[:3] = (1 - c) * pivot
    return M.astype(np.float32), bias.astype(np.float32)


@dataclasses.dataclass(frozen=True)
class DecodeConfig:
    """What the fused decode kernel does to each u8 HWC image.

    channels: 'rgb' | 'rgba' | 'bgr' | 'gray' or an explicit input-channel map
        (output channel c reads input channel ``channels[c]``).
    gamma: gamma applied to the colour channels (alpha passes through), as the
        reference's ``_color_correct``; None = off.
    scale, mean, std: ``out = (g(x) * scale - mean[c]) / std[c]`` in fp32.
    dtype: 'float32' | 'bfloat16' | 'float16' | 'uint8' (uint8 only without
        normalisation).
    layout: 'nchw' (default, the densityopt item_transform) or 'nhwc'.
    flip: force a vertical flip of every image (GL lower-left -> upper-left).
        Producers that send lower-left frames with ``origin='lower-left'`` are
        flipped per image automatically by the stream loader.
    color_matrix / color_bias: optional 4x4 affine colour transform applied
        after gamma (RGBA input, fp32 NCHW output; runs on the MFMA units).
    color_matrices / color_biases: one such transform per batch position
        ([B, 4, 4] / [B, 4]; the loader's batch size must be B).
    color_jitter: a :class:`ColorJitter` -- a random transform per image,
        built inside the same kernel, applied to ``gamma(x) * scale``
        (channels 'rgb' or 'rgba', no mean/std).
    """
    channels: object = 'rgb'
    gamma: Optional[float] = None
    scale: float = 1.0
    mean: Optional[Sequence[float]] = None
    std: Optional[Sequence[float]] = None
    dtype: str = 'float32'
    layout: str = 'nchw'
    flip: bool = False
    color_matrix: Optional[Sequence[Sequence[float]]] = None
    color_bias: Optional[Sequence[float]] = None
    color_matrices: Optional[Sequence] = None
    color_biases: Optional[Sequence] = None
    color_jitter: Optional[ColorJitter] = None

    def __post_init__(self):
        # normalise sequences to tuples: configs are hashable cache keys
        if not isinstance(self.channels, str):
            object.__setattr__(self, 'channels', tuple(int(c) for c in self.channels))
        for f in ('mean', 'std', 'color_bias'):
            v = getattr(self, f)
            if v is not None:
                object.__setattr__(self, f, tuple(float(x) for x in v))
        if self.color_matrix is not None:
            object.__setattr__(self, 'color_matrix', tuple(tuple(float(x) for x in r) for r in self.color_matrix))
        if self.dtype not in OUT_DTYPES:
            raise ValueError(f'dtype must be one of {list(OUT_DTYPES)}')
        if self.layout not in LAYOUTS:
            raise ValueError(f'layout must be one of {list(LAYOUTS)}')
        if self.dtype == 'uint8' and (self.mean is not None or self.std is not None or self.scale != 1.0):
            raise ValueError('uint8 output cannot be normalised')
        if self.color_matrix is not None:
            m = np.asarray(self.color_matrix, dtype=np.float32)
            if m.shape != (4, 4):
                raise ValueError('color_matrix must be 4x4')
            if self.dtype != 'float32' or self.layout != 'nchw':
                raise ValueError('color_matrix produces float32 NCHW output')
        if self.color_matrices is not None:
            m = np.asarray(self.color_matrices, dtype=np.float32)
            if m.ndim != 3 or m.shape[1:] != (4, 4) or not 1 <= m.shape[0] <= 64:
                raise ValueError('color_matrices must be [B, 4, 4] with B <= 64')
            object.__setattr__(self, 'color_matrices', tuple(tuple(tuple(float(x) for x in r) for r in mm) for mm in m))
            bb = np.zeros((m.shape[0], 4), np.float32) if self.color_biases is None else \
                np.asarray(self.color_biases, np.float32)
            if bb.shape != (m.shape[0], 4):
                raise ValueError('color_biases must be [B, 4]')
            object.__setattr__(self, 'color_biases', tuple(tuple(float(x) for x in r) for r in bb))
        if self.color_jitter is not None:
            if not isinstance(self.color_jitter, ColorJitter):
                raise TypeError('color_jitter must be an ops.ColorJitter')
            if self.channels not in ('rgb', 'rgba') or self.mean is not None or self.std is not None:
                raise ValueError("color_jitter needs channels 'rgb' or 'rgba' and no mean/std")
        if sum(x is not None for x in (self.color_matrix, self.color_matrices, self.color_jitter)) > 1:
            raise ValueError('color_matrix, color_matrices and color_jitter are exclusive')
        if (self.color_matrices is not None or self.color_jitter is not None) and \
                (self.dtype != 'float32' or self.layout != 'nchw'):
            raise ValueError('per-image colour transforms produce float32 NCHW output')

    # -- presets -----------------------------------------------------------
    @classmethod
    def densityopt(cls, **kw):
        """``(x - 127.5) / 127.5`` + HWC->CHW (``densityopt.py:117-119``)."""
        return cls(mean=(127.5,) * 4, std=(127.5,) * 4, **kw)

    @classmethod
    def unit(cls, **kw):
        """x / 255 in [0, 1]."""
        return cls(scale=1.0 / 255.0, **kw)

    @classmethod
    def raw(cls, channels='rgba', **kw):
        """Bytes as they came: u8, channels-last, no gamma (identity table) --
        e.g. to fill a :class:`~blendtorch.btt.replay.DeviceReplayBuffer`."""
        return cls(channels=channels, dtype='uint8', layout='nhwc', **kw)

    @property
    def cmap(self):
        if isinstance(self.channels, str):
            return {'rgb': [0, 1, 2], 'rgba': [0, 1, 2, 3], 'bgr': [2, 1, 0], 'bgra': [2, 1, 0, 3],
                    'gray': [0], 'r': [0]}[self.channels]
        return list(self.channels)

    @property
    def colour_kernel(self):
        """Decoded by the MFMA colour kernel (RGBA input)."""
        return self.color_matrix is not None or self.color_matrices is not None or self.color_jitter is not None

    @property
    def cout(self):
        if self.color_jitter is not None:
            return len(self.cmap)
        return 4 if self.colour_kernel else len(self.cmap)

    @property
    def jitter_pivot(self):
        j = self.color_jitter
        return float(j.pivot) if j is not None and j.pivot is not None else 127.5 * float(self.scale)

    def out_shape(self, B, H, W):
        c = self.cout
        return (B, c, H, W) if self.layout == 'nchw' else (B, H, W, c)

    def torch_dtype(self):
        import torch
        return getattr(torch, self.dtype)


def build_lut(cfg: DecodeConfig) -> np.ndarray:
    """float32[4, 256]: value of output channel c for input byte v.

    Gamma applies to output channels fed by input channels 0..2 (colour), not
    to alpha (input channel 3), as in the reference.  For a colour matrix the
    table is indexed by INPUT channel (the MFMA kernel mixes channels after).
    """
    g = gamma_lut(cfg.gamma).astype(np.float32)
    ident = np.arange(256, dtype=np.float32)
    lut = np.zeros((4, 256), dtype=np.float32)
    if cfg.color_matrix is not None or cfg.color_matrices is not None:
        for k in range(4):
            lut[k] = g if k < 3 else ident
        return lut
    if cfg.color_jitter is not None:   # the jitter works on gamma(x) * scale (alpha: x * scale)
        for k in range(4):
            lut[k] = (g if k < 3 else ident) * np.float32(cfg.scale)
        return lut
    mean = np.asarray(cfg.mean if cfg.mean is not None else [0.0] * 4, dtype=np.float32)
    std = np.asarray(cfg.std if cfg.std is not None else [1.0] * 4, dtype=np.float32)
    scale = np.float32(cfg.scale)
    for c, ic in enumerate(cfg.cmap):
        x = g if ic < 3 else ident
        if cfg.mean is None and cfg.std is None and cfg.scale == 1.0:
            lut[c] = x
        else:
            lut[c] = (x * scale - mean[c]) / std[c]
    return lut


# value table handed to the kernels (csrc/gpu/kernels.h: lut): the fp32 table
# plus a per-channel arithmetic form the host has verified bit for bit
XF_HEADER, XF_GAMMA, TABLE_FLOATS = 1024, 1088, 1152


def _xform_channel(x, y, gam, normalize, scale, mean, std):
    """(op, a, b, d, r) reproducing float32 table ``y`` from inputs ``x``
    exactly, or None (csrc/codec/xform_fit.h: op 0 fma, 1 mul-sub, 3 mul-sub
    times the reciprocal with one fma correction, 2 division; each verified
    over all 256 inputs).  Without the native module: the forms numpy can
    emulate exactly (op 0 with b == 0, ops 1 and 2)."""
    f32 = np.float32
    try:
        from .. import _native
        return _native.xform_fit(np.ascontiguousarray(x, f32), np.ascontiguousarray(y, f32), float(scale),
                                 float(mean), float(std), bool(normalize))
    except ImportError:
        pass
    cands = []
    if not normalize:
        cands.append((0, f32(1.0), f32(0.0), f32(1.0)))
    else:
        if mean == 0.0 and std == 1.0:
            cands.append((0, f32(scale), f32(0.0), f32(1.0)))
        if std == 1.0:
            cands.append((1, f32(scale), f32(mean), f32(1.0)))
        cands.append((2, f32(scale), f32(mean), f32(std)))
    with np.errstate(all='ignore'):
        for op, a, b, d in cands:
            if op == 0:
                z = x * a            # b == 0: the fma is this product, rounded once
            elif op == 1:
                z = x * a - b
            else:
                z = (x * a - b) / d
            if np.array_equal(z.view(np.uint32), y.view(np.uint32)):
                return op, float(a), float(b), float(d), float(f32(1.0) / d)
    return None


def build_table(cfg: DecodeConfig) -> np.ndarray:
    """float32[TABLE_FLOATS]: :func:`build_lut` plus the header and u8 gamma
    table of the kernels' arithmetic path (see csrc/gpu/kernels.h).

    ``BLENDTORCH_DECODE_XFORM``: ``auto`` (default) uses the arithmetic path
    when it reads no LDS and needs no division (no gamma, ops 0/1), the fp32
    table otherwise; ``1`` always the arithmetic path (bank-conflict-free
    lane-private gamma copies, ``BLENDTORCH_GAMMA_COPIES`` 16/32); ``0``
    always the table.  Mode 0 also whenever a channel has no verified form."""
    lut = build_lut(cfg)
    out = np.zeros(TABLE_FLOATS, dtype=np.float32)
    out[:1024] = lut.reshape(-1)
    policy = os.environ.get('BLENDTORCH_DECODE_XFORM', 'auto')
    if policy == '0':
        return out                                  # fp32 table lookups
    g = gamma_lut(cfg.gamma)
    gf = g.astype(np.float32)
    ident = np.arange(256, dtype=np.float32)
    if cfg.colour_kernel:
        chans = [(k, k) for k in range(4)]          # indexed by input channel, no normalisation
        normalize = cfg.color_jitter is not None and cfg.scale != 1.0   # (jitter: gamma(x) * scale)
    else:
        chans = list(enumerate(cfg.cmap))
        normalize = not (cfg.mean is None and cfg.std is None and cfg.scale == 1.0)
    mean = list(cfg.mean) if cfg.mean is not None else [0.0] * 4
    std = list(cfg.std) if cfg.std is not None else [1.0] * 4
    hdr = np.zeros(26, dtype=np.float32)   # mode, gamma_used, gam[4], op[4], a[4], b[4], d[4], r[4]
    hdr[10:14] = 1.0
    hdr[18:26] = 1.0
    for c, ic in chans:
        gam = bool(cfg.gamma) and ic < 3
        x = gf if gam else ident
        form = _xform_channel(x, lut[c], gam, normalize, np.float32(cfg.scale), mean[c], std[c])
        if form is None:
            return out                              # mode 0: table lookups
        op, a, b, d, r = form
        hdr[2 + c], hdr[6 + c], hdr[10 + c], hdr[14 + c], hdr[18 + c], hdr[22 + c] = float(gam), op, a, b, d, r
        hdr[1] = max(hdr[1], float(gam))
    if policy == 'auto' and (hdr[1] or any(int(o) not in (0, 1) for o in hdr[6:6 + len(chans)])):
        # measured (profiles/r3/decode_ab.md): with a gamma table or a division
        # the arithmetic form costs ~35 % more VALU and 5-15 % more time than
        # the fp32 table, whose bank conflicts (2.2 extra cycles per ds_read on
        # uniform random pixels) are not what bounds the kernel; without
        # either it reads no LDS at all at the table's speed
        return out
    if hdr[1]:
        hdr[1] = float(int(os.environ.get('BLENDTORCH_GAMMA_COPIES', '32')))   # lane-private copies: 16 or 32
        if hdr[1] not in (16.0, 32.0):
            raise ValueError('BLENDTORCH_GAMMA_COPIES must be 16 or 32')
    hdr[0] = 1.0
    out[XF_HEADER:XF_HEADER + 26] = hdr
    out[XF_GAMMA:XF_GAMMA + 64] = np.frombuffer(g.astype(np.uint8).tobytes(), dtype=np.float32)
    return out


# ---------------------------------------------------------------------------
# references (plain PyTorch fp32)
# ---------------------------------------------------------------------------
def reference_gamma(images, gamma):
    """Torch port of the reference formula on a u8 tensor (alpha untouched)."""
    import torch
    rgb = images[..., :3].to(torch.float32) / 255
    rgb = (255.0 * rgb ** (1 / gamma)).to(torch.uint8)
    if images.shape[-1] == 4:
        return torch.cat([rgb, images[..., 3:4]], dim=-1)
    return rgb


def reference_decode(images, cfg: DecodeConfig, flip=None, jitter=None):
    """fp32 PyTorch reference of :func:`decode` (images: u8 [B,H,W,C]); for a
    ``color_jitter`` config, ``jitter`` holds the [B, 4] factors of the batch
    (``batch['color_jitter']``)."""
    import torch
    x = images
    if x.dim() == 3:
        x = x.unsqueeze(-1)
    if cfg.colour_kernel:
        if flip is not None:
            f = torch.as_tensor(flip, dtype=torch.bool, device=x.device)
            x = torch.where(f.view(-1, 1, 1, 1), torch.flip(x, dims=[1]), x)
        if cfg.color_matrix is not None:
            M, b = np.asarray(cfg.color_matrix, np.float32), np.asarray(cfg.color_bias or [0.0] * 4, np.float32)
        elif cfg.color_matrices is not None:
            M, b = np.asarray(cfg.color_matrices, np.float32), np.asarray(cfg.color_biases, np.float32)
        else:
            if jitter is None:
                raise ValueError('reference_decode: a color_jitter config needs the batch\'s jitter factors')
            mb = [color_jitter_matrix(f, cfg.jitter_pivot) for f in np.asarray(jitter, np.float64)]
            # the jitter works on gamma(x) * scale: fold the scale into the matrix columns
            M = np.stack([m for m, _ in mb]) * np.float32(cfg.scale)
            b = np.stack([bb for _, bb in mb])
        out = reference_color4x4(x, M, b, gamma=cfg.gamma, flip=cfg.flip)
        return out[:, :cfg.cout]
    if cfg.flip:
        x = torch.flip(x, dims=[1])
    if flip is not None:
        f = torch.as_tensor(flip, dtype=torch.bool, device=x.device)
        x = torch.where(f.view(-1, 1, 1, 1), torch.flip(x, dims=[1]), x)
    chans = []
    for c, ic in enumerate(cfg.cmap):
        v = x[..., ic]
        if cfg.gamma and ic < 3:
            v = (255.0 * (v.to(torch.float32) / 255) ** (1 / cfg.gamma)).to(torch.uint8)
        v = v.to(torch.float32)
        if not (cfg.mean is None and cfg.std is None and cfg.scale == 1.0):
            mean = (cfg.mean or [0.0] * 4)[c]
            std = (cfg.std or [1.0] * 4)[c]
            v = (v * torch.tensor(cfg.scale, dtype=torch.float32) - torch.tensor(mean, dtype=torch.float32)) \
                / torch.tensor(std, dtype=torch.float32)
        chans.append(v)
    out = torch.stack(chans, dim=1 if cfg.layout == 'nchw' else -1)
    return out.to(cfg.torch_dtype())


def reference_color4x4(images, M, bias, gamma=None, flip=False):
    """fp32 reference: ``M`` [4, 4] / ``bias`` [4], or one per image ([B, 4, 4] / [B, 4])."""
    import torch
    x = images
    if flip:
        x = torch.flip(x, dims=[1])
    if gamma:
        x = reference_gamma(x, gamma)
    x = x.to(torch.float32)
    M = torch.as_tensor(np.asarray(M, np.float32) if not isinstance(M, torch.Tensor) else M,
                        dtype=torch.float32, device=x.device)
    b = torch.as_tensor(np.asarray(bias, np.float32) if not isinstance(bias, torch.Tensor) else bias,
                        dtype=torch.float32, device=x.device)
    if M.dim() == 3:
        out = torch.einsum('bhwk,bck->bchw', x, M)
        return out + (b.view(-1, b.shape[-1], 1, 1) if b.dim() == 2 else b.view(1, -1, 1, 1))
    out = torch.einsum('bhwk,ck->bchw', x, M) + b.view(1, -1, 1, 1)
    return out


def reference_project(points, PV, V, W, H, upper_left=True):
    """btb.Camera.world_to_ndc + ndc_to_pixel (``camera.py:84-136``) in torch."""
    import torch
    p = torch.as_tensor(points, dtype=torch.float64)
    xyzw = torch.cat([p, torch.ones_like(p[:, :1])], dim=1)
    clip = xyzw @ torch.as_tensor(PV, dtype=torch.float64).T
    ndc = clip[:, :3] / clip[:, 3:4]
    xy = (ndc[:, :2] + 1) * 0.5
    if upper_left:
        xy[:, 1] = 1.0 - xy[:, 1]
    px = xy * torch.tensor([[W, H]], dtype=torch.float64)
    depth = -(xyzw @ torch.as_tensor(V, dtype=torch.float64).T)[:, 2]
    return px, depth


# ---------------------------------------------------------------------------
# HIP launchers
# ---------------------------------------------------------------------------
_lut_cache = {}


def device_lut(cfg: DecodeConfig, device):
    import torch
    key = (cfg, str(device))
    t = _lut_cache.get(key)
    if t is None:
        tab = build_table(cfg)
        t = torch.from_numpy(tab).to(device)
        _lut_cache[key] = t
        mode = int(tab[XF_HEADER])
        # table mode with the same 256 values for every output channel: the
        # replay kernel's conflict-free 32-copy table form takes it (table_only 2)
        uni = mode == 0 and all(np.array_equal(tab[:256], tab[256 * c:256 * (c + 1)]) for c in range(1, cfg.cout))
        _lut_cache[('mode',) + key] = mode
        _lut_cache[('uni',) + key] = uni
    return t


def table_only(cfg: DecodeConfig, device) -> int:
    """1 when ``device_lut(cfg, device)`` is in table mode (header mode 0):
    kernels may then take their table-only variant; 2 when besides every
    output channel has the same table."""
    device_lut(cfg, device)
    if _lut_cache[('mode', cfg, str(device))] != 0:
        return 0
    return 2 if _lut_cache[('uni', cfg, str(device))] else 1


def _stream(device):
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def decode(images, cfg: DecodeConfig = DecodeConfig(), flip=None, out=None):
    """Fused decode of a u8 [B,H,W,C] device tensor with the gfx950 kernel."""
    import torch
    ext = hip_ext()
    if images.dtype != torch.uint8 or not images.is_cuda:
        raise TypeError('decode expects a uint8 CUDA/HIP tensor')
    x = images.contiguous()
    if x.dim() == 3:
        x = x.unsqueeze(-1)
    B, H, W, C = x.shape
    if max(cfg.cmap) >= C:
        raise ValueError(f'channel map {cfg.cmap} needs more than {C} input channels')
    if cfg.color_matrix is not None:
        return color4x4(x, cfg.color_matrix, cfg.color_bias or [0.0] * 4, gamma=cfg.gamma, flip=cfg.flip)
    if cfg.color_matrices is not None:
        if B != len(cfg.color_matrices):
            raise ValueError(f'decode: {len(cfg.color_matrices)} colour matrices for {B} images')
        return color4x4(x, cfg.color_matrices, cfg.color_biases, gamma=cfg.gamma, flip=cfg.flip)
    if cfg.color_jitter is not None:
        raise ValueError('decode: colour jitter draws its factors in the stream loader; apply given factors with '
                         'color4x4(images, jitter=factors)')
    if out is None:
        out = torch.empty(cfg.out_shape(B, H, W), dtype=cfg.torch_dtype(), device=x.device)
    lut = device_lut(cfg, x.device)
    fl = 0
    if flip is not None:
        fl_t = torch.as_tensor(flip, dtype=torch.uint8, device=x.device).contiguous()
        if fl_t.numel() != B:
            raise ValueError('flip needs one flag per image')
        fl = fl_t.data_ptr()
    ext.decode(x.data_ptr(), 0, out.data_ptr(), lut.data_ptr(), fl, B, H, W, C, cfg.cout, cfg.cmap,
               int(cfg.flip), OUT_DTYPES[cfg.dtype], LAYOUTS[cfg.layout], _stream(x.device))
    return out


def decode_gather(store, index, cfg: DecodeConfig = DecodeConfig(), out=None):
    """Fused gather + decode: ``decode(store[index], cfg)`` without
    materialising the gathered u8 batch.  ``store`` is a u8 [N,H,W,C] device
    tensor (e.g. an HBM-resident frame store), ``index`` an int [B] device
    tensor.  The kernel reads image b at ``store + index[b] * H*W*C``."""
    import torch
    ext = hip_ext()
    if store.dtype != torch.uint8 or not store.is_cuda or not store.is_contiguous() or store.dim() != 4:
        raise TypeError('decode_gather expects a contiguous uint8 [N,H,W,C] CUDA/HIP tensor')
    if cfg.colour_kernel:
        raise ValueError('decode_gather: colour matrices are not supported; use color4x4 on store[index]')
    N, H, W, C = store.shape
    if max(cfg.cmap) >= C:
        raise ValueError(f'channel map {cfg.cmap} needs more than {C} input channels')
    idx = index.to(device=store.device, dtype=torch.int64)
    B = int(idx.numel())
    frame = H * W * C
    offsets = (idx * frame).contiguous()
    if out is None:
        out = torch.empty(cfg.out_shape(B, H, W), dtype=cfg.torch_dtype(), device=store.device)
    lut = device_lut(cfg, store.device)
    ext.decode(store.data_ptr(), offsets.data_ptr(), out.data_ptr(), lut.data_ptr(), 0, B, H, W, C, cfg.cout,
               cfg.cmap, int(cfg.flip), OUT_DTYPES[cfg.dtype], LAYOUTS[cfg.layout], _stream(store.device),
               frame % 16 == 0)
    return out


def philox_indices(seed: int, counter: int, B: int, count: int) -> np.ndarray:
    """The frame indices :func:`replay_sample` draws (numpy reference):
    Philox4x32-10 with key ``seed`` and counter ``(b, counter)`` for image b,
    first output word scaled to ``[0, count)`` as ``(word * count) >> 32``."""
    M0, M1, W0, W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), 0x9E3779B9, 0xBB67AE85
    mask = np.uint64(0xFFFFFFFF)
    c0 = np.arange(B, dtype=np.uint64)
    c1 = np.full(B, counter & 0xFFFFFFFF, np.uint64)
    c2 = np.full(B, (counter >> 32) & 0xFFFFFFFF, np.uint64)
    c3 = np.zeros(B, np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0, p1 = M0 * c0, M1 * c2          # < 2^64: exact in uint64
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return ((c0 * np.uint64(count)) >> np.uint64(32)).astype(np.int64)


def replay_sample(store, count: int, batch: int, cfg: DecodeConfig = DecodeConfig(), seed: int = 0, counter=None,
                  index=None, meta=None, out=None):
    """Fused replay sample on the gfx950 kernel: draw ``batch`` frame indices
    in ``[0, count)`` on the device (Philox, see :func:`philox_indices`) --
    or use ``index`` (int64 [batch]) -- decode those frames of ``store`` (u8
    [N,H,W,C] on the device) with ``cfg``, and gather row ``idx`` of every
    ``meta`` column (dict name -> device tensor [N, ...]), in ONE launch.

    ``counter``: an int (the Philox counter; the caller advances it by
    ``batch``), or a device int64 tensor holding it -- then a one-lane kernel
    behind the sample advances it, so a captured HIP graph draws fresh
    indices on every replay.  Returns ``(images, index, meta_out)``."""
    import torch
    ext = hip_ext()
    if store.dtype != torch.uint8 or not store.is_cuda or store.dim() != 4 or not store.is_contiguous():
        raise TypeError('replay_sample expects a contiguous uint8 [N,H,W,C] device tensor')
    if cfg.colour_kernel:
        raise ValueError('replay_sample does not apply colour matrices (use gather + color4x4)')
    N, H, W, C = store.shape
    if max(cfg.cmap) >= C:
        raise ValueError(f'channel map {cfg.cmap} needs more than {C} input channels')
    dev = store.device
    if out is None:
        out = torch.empty(cfg.out_shape(batch, H, W), dtype=cfg.torch_dtype(), device=dev)
    idx_out = torch.empty(batch, dtype=torch.int64, device=dev)
    idx_in, ctr_ptr, ctr_value = 0, 0, 0
    if index is not None:
        index = index.to(dev, torch.int64).contiguous()
        if index.numel() != batch:
            raise ValueError('index needs one entry per image')
        idx_in = index.data_ptr()
    elif isinstance(counter, torch.Tensor):
        if counter.dtype != torch.int64 or counter.numel() < 1 or counter.device != dev:
            raise ValueError('a device counter must be an int64 tensor on the store\'s device')
        ctr_ptr = counter.data_ptr()
    elif counter is not None:
        ctr_value = int(counter) & (2 ** 64 - 1)
    else:
        raise ValueError('drawing indices needs a counter (int or device tensor)')
    meta = meta or {}
    mout, src, dst, nbytes = {}, [], [], []
    for k, col in meta.items():
        if col.device != dev or not col.is_contiguous() or col.shape[0] != N:
            raise ValueError(f'metadata column {k!r} must be a contiguous [{N}, ...] tensor on {dev}')
        o = torch.empty((batch,) + tuple(col.shape[1:]), dtype=col.dtype, device=dev)
        mout[k] = o
        src.append(col.data_ptr())
        dst.append(o.data_ptr())
        nbytes.append(col[0].numel() * col.element_size())
    lut = device_lut(cfg, dev)
    ext.replay_sample(store.data_ptr(), int(count), out.data_ptr(), lut.data_ptr(), batch, H, W, C, cfg.cout,
                      cfg.cmap, int(cfg.flip), OUT_DTYPES[cfg.dtype], LAYOUTS[cfg.layout], int(seed) & (2 ** 64 - 1),
                      ctr_ptr, ctr_value, idx_in, idx_out.data_ptr(), src, dst, nbytes,
                      _stream(dev), table_only(cfg, dev))
    return out, idx_out, mout


def color4x4(images, M=None, bias=(0.0, 0.0, 0.0, 0.0), gamma=None, flip=False, cout=4, jitter=None, pivot=127.5):
    """out[b,c] = M[c,:] . g(in[b,:,y,x]) + bias[c] on the MFMA units (fp32).

    ``M`` [4, 4] (one transform) or [B, 4, 4] with ``bias`` [4] / [B, 4] (one
    per image); or ``jitter`` [B, 4] colour-jitter factors (B <= 64), whose
    transforms the kernel builds itself (:func:`color_jitter_matrix` about
    ``pivot``, in the units of ``g``: 0..255)."""
    import torch
    ext = hip_ext()
    x = images.contiguous()
    B, H, W, C = x.shape
    if C != 4:
        raise ValueError('color4x4 needs RGBA input')
    if (H * W) % 256 or W % 4:
        raise ValueError('color4x4 needs H*W % 256 == 0 and W % 4 == 0')
    if jitter is not None:
        f = np.ascontiguousarray(jitter, np.float32)
        if f.shape != (B, 4) or B > 64:
            raise ValueError('color4x4: jitter must be [B, 4] with B <= 64')
        lut = device_lut(DecodeConfig(channels='rgba', gamma=gamma, color_matrix=np.eye(4)), x.device)
        out = torch.empty((B, cout, H, W), dtype=torch.float32, device=x.device)
        ext.color4x4(x.data_ptr(), out.data_ptr(), lut.data_ptr(), 0, 0, 0, B, H, W, cout, int(flip),
                     _stream(x.device), 3, 0, f.reshape(-1).tolist(), float(pivot))
        return out
    Mt_in = M.detach().to(torch.float32) if isinstance(M, torch.Tensor) else None
    Mn = None if Mt_in is not None else np.ascontiguousarray(M, np.float32)
    shape = tuple(Mt_in.shape) if Mt_in is not None else Mn.shape
    if len(shape) == 3:
        if shape != (B, 4, 4):
            raise ValueError(f'color4x4: per-image M must be [{B}, 4, 4]')
        # one transform per image: [B, 16 + 4] rows on the device
        Mt = Mt_in.to(x.device).reshape(B, 16) if Mt_in is not None else torch.from_numpy(Mn.reshape(B, 16)).to(x.device)
        bt = torch.as_tensor(np.asarray(bias, np.float32) if not isinstance(bias, torch.Tensor) else bias,
                             dtype=torch.float32, device=x.device)
        bt = bt.expand(B, 4) if bt.dim() == 1 else bt
        rows = torch.cat([Mt, bt.reshape(B, 4)], dim=1).contiguous()
        lut = device_lut(DecodeConfig(channels='rgba', gamma=gamma, color_matrix=np.eye(4)), x.device)
        out = torch.empty((B, cout, H, W), dtype=torch.float32, device=x.device)
        ext.color4x4(x.data_ptr(), out.data_ptr(), lut.data_ptr(), 0, 0, 0, B, H, W, cout, int(flip),
                     _stream(x.device), 2, rows.data_ptr(), [], 0.0)
        return out
    if Mn is None:
        Mn = Mt_in.cpu().numpy()
    if Mn.shape != (4, 4):
        raise ValueError(f'color4x4: M must be [4, 4] or [{B}, 4, 4]')
    bn = np.ascontiguousarray(bias, np.float32)
    key = ('color4x4', Mn.tobytes(), bn.tobytes(), gamma, str(x.device))
    cached = _lut_cache.get(key)
    if cached is None:   # LUT + matrix + bias uploaded once per (M, bias, gamma, device)
        cfg = DecodeConfig(channels='rgba', gamma=gamma, color_matrix=tuple(map(tuple, Mn)))
        cached = (device_lut(cfg, x.device), torch.from_numpy(Mn).to(x.device), torch.from_numpy(bn).to(x.device))
        _lut_cache[key] = cached
    lut, Mt, bt = cached
    out = torch.empty((B, cout, H, W), dtype=torch.float32, device=x.device)
    ext.color4x4(x.data_ptr(), out.data_ptr(), lut.data_ptr(), Mt.data_ptr(), bt.data_ptr(), 0, B, H, W, cout,
                 int(flip), _stream(x.device))
    return out


def project(points, PV, V, W, H, upper_left=True):
    """Batched world->pixel projection on the GPU (fp32)."""
    import torch
    ext = hip_ext()
    p = points.to(torch.float32).contiguous()
    dev = p.device
    PVt = torch.as_tensor(np.asarray(PV, np.float32), device=dev).contiguous()
    Vt = torch.as_tensor(np.asarray(V, np.float32), device=dev).contiguous()
    N = p.shape[0]
    px = torch.empty((N, 2), dtype=torch.float32, device=dev)
    depth = torch.empty((N,), dtype=torch.float32, device=dev)
    ext.project(p.data_ptr(), N, PVt.data_ptr(), Vt.data_ptr(), W, H, int(upper_left), px.data_ptr(),
                depth.data_ptr(), _stream(dev))
    return px, depth


# ---------------------------------------------------------------------------
# consumer-model op: adaptive average pooling on channels-last activations

_DT_CODES = {}


def _dt(x):
    """Kernel dtype code of a tensor (None when unsupported); keyed by the
    torch dtype object, so the per-call cost is one dict lookup."""
    if not _DT_CODES:
        import torch
        _DT_CODES.update({torch.float32: 0, torch.bfloat16: 1})
    return _DT_CODES.get(x.dtype)


# Host-side count of launches of the consumer-model kernels, by kernel name.
# Tests assert the fused gfx950 path ran on the bench shapes instead of the
# PyTorch fallback the modules take for unsupported inputs (a captured HIP
# graph counts once, at capture).
KERNEL_CALLS = {}


def _count(name):
    KERNEL_CALLS[name] = KERNEL_CALLS.get(name, 0) + 1


def _pool_launch(name, src, dst, N, H, W, C, OH, OW):
    ext = hip_ext()
    _count(name)
    getattr(ext, name)(src.data_ptr(), dst.data_ptr(), N, H, W, C, OH, OW, _dt(src),
                       _stream(src.device))


def _as_nhwc(x):
    """[N,C,H,W] tensor -> its [N,H,W,C] storage view (copies unless channels-last;
    the kernels' 16-byte vector accesses also need a 16-byte aligned base)."""
    xs = x.permute(0, 2, 3, 1).contiguous()
    return xs if xs.data_ptr() % 16 == 0 else xs.clone()


def _pool_function():
    import torch

    class _AdaptiveAvgPoolNHWC(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, oh, ow):
            N, C, H, W = x.shape
            xs = _as_nhwc(x)
            y = torch.empty((N, oh, ow, C), dtype=x.dtype, device=x.device)
            _pool_launch('adaptive_avgpool_nhwc', xs, y, N, H, W, C, oh, ow)
            ctx.shape = (N, C, H, W, oh, ow)
            return y.permute(0, 3, 1, 2)

        @staticmethod
        def backward(ctx, gy):
            N, C, H, W, oh, ow = ctx.shape
            gys = _as_nhwc(gy)
            gx = torch.empty((N, H, W, C), dtype=gy.dtype, device=gy.device)
            _pool_launch('adaptive_avgpool_nhwc_bwd', gys, gx, N, H, W, C, oh, ow)
            return gx.permute(0, 3, 1, 2), None, None

    return _AdaptiveAvgPoolNHWC


_POOL_FN = None


def adaptive_avg_pool_nhwc(x, output_size):
    """``F.adaptive_avg_pool2d`` for GPU activations on the gfx950 kernels
    (fp32 or bf16; the result and the input gradient are channels-last)."""
    global _POOL_FN
    if _POOL_FN is None:
        _POOL_FN = _pool_function()
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    if x.dim() != 4 or _dt(x) is None:
        raise ValueError(f'adaptive_avg_pool_nhwc needs a 4-D float32/bfloat16 tensor, got {x.dtype} {tuple(x.shape)}')
    return _POOL_FN.apply(x, oh, ow)


def reference_adaptive_avg_pool(x, output_size):
    """fp32 reference (PyTorch)."""
    import torch.nn.functional as F
    return F.adaptive_avg_pool2d(x.float(), output_size)


_POOL_MODULE = None


def _pool_module():
    import torch.nn as nn
    import torch.nn.functional as F

    class AdaptiveAvgPool2d(nn.Module):
        """Drop-in ``nn.AdaptiveAvgPool2d``: GPU fp32/bf16 inputs run the gfx950
        kernels, anything else (CPU tensors, other dtypes) the PyTorch op."""

        def __init__(self, output_size):
            super().__init__()
            self.output_size = output_size

        def forward(self, x):
            if x.is_cuda and _dt(x) is not None:
                return adaptive_avg_pool_nhwc(x, self.output_size)
            return F.adaptive_avg_pool2d(x, self.output_size)

        def extra_repr(self):
            return f'output_size={self.output_size}'

    AdaptiveAvgPool2d.__module__ = __name__
    return AdaptiveAvgPool2d


# ---------------------------------------------------------------------------
# gradient sinks: parameters whose gradient lives in a persistent flat bucket
# (parallel.GradBuckets) get it written there by the backward kernel itself

# Gradient-completion listener (parallel.GradBuckets.arm): called with a
# parameter right after the launch that writes its bucket-view gradient for
# the last time in this backward is enqueued, so a data-parallel step can
# enqueue a bucket's all-reduce as soon as every gradient in it is written,
# ahead of the rest of the backward.  _GRAD_LATE is called when a parameter
# whose bucket view was already written gets another contribution.
_GRAD_DONE = None
_GRAD_LATE = None


def _grad_done(*params):
    if _GRAD_DONE is not None:
        for p in params:
            if p is not None:
                _GRAD_DONE(p)


def grad_sink(param):
    """The persistent gradient view of ``param`` installed by
    ``parallel.GradBuckets`` (same shape and strides), or None."""
    return getattr(param, '_bt_grad_sink', None)


def _grad_sink_ready(param):
    """Would :func:`_grad_dest` write ``param``'s gradient into its bucket view
    (fp32, contiguous)?  Consumes nothing."""
    import torch
    sink = grad_sink(param) if param is not None else None
    return (sink is not None and param.grad is sink and (getattr(param, '_bt_grad_fresh', False)
                                                          or getattr(param, '_bt_grad_fresh2', False))
            and sink.dtype == torch.float32 and sink.is_contiguous())


def _grad_dest(param, like=None):
    """(tensor the backward kernel writes ``param``'s gradient into, whether
    that is the param's bucket view).  The first gradient after
    ``GradBuckets.zero_()`` is written straight into the bucket and the op
    returns None for that input (no AccumulateGrad kernel); any further one
    in the same step (several backward passes before the optimizer step)
    goes to a fresh tensor that autograd adds into ``param.grad`` -- the
    usual accumulate semantics either way -- or, with a second bucket view
    (``GradBuckets(second_sinks=True)``), the second one into that view,
    which :class:`FusedAdam` adds in its update kernel.  A bucket view that is no longer
    ``param.grad`` (e.g. after ``zero_grad(set_to_none=True)``) is ignored."""
    import torch
    sink = grad_sink(param) if param is not None else None
    if sink is not None and param.grad is sink and getattr(param, '_bt_grad_fresh', False):
        param._bt_grad_fresh = False
        return sink, True
    if sink is not None and param.grad is sink and getattr(param, '_bt_grad_fresh2', False):
        # the second contribution of the step (GradBuckets(second_sinks=True)): into the
        # second bucket view, which the FusedAdam update adds -- no AccumulateGrad launch
        param._bt_grad_fresh2 = False
        param._bt_grad_second = True
        return param._bt_grad_sink2, True
    if sink is not None and _GRAD_LATE is not None:
        _GRAD_LATE(param)
    if sink is not None:
        _count('grad_dest_autograd_add')   # a bucketed gradient autograd will add (one launch)
    return torch.empty_like(param if like is None else like), False


# ---------------------------------------------------------------------------
# consumer-model op: one-launch fp32 -> bf16 cast of a parameter list

def _dense(t):
    """Non-overlapping and dense (any dimension order we produce: contiguous or channels-last)."""
    import torch
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _cast_function():
    import torch

    def launch(srcs, outs, mode):
        ext = hip_ext()
        _count('multi_cast')
        ext.multi_cast([t.data_ptr() for t in srcs], [o.data_ptr() for o in outs], [t.numel() for t in srcs], mode,
                       _stream(srcs[0].device))

    class _CastBF16(torch.autograd.Function):
        """fp32 tensors -> bf16 copies (forward) and bf16 gradients -> fp32
        (backward), each direction ONE multi-tensor kernel (autocast casts
        every weight, and every weight gradient back, separately)."""

        @staticmethod
        def forward(ctx, *ws):
            outs = [torch.empty_like(w, dtype=torch.bfloat16) for w in ws]
            launch(ws, outs, 0)
            return tuple(outs)

        @staticmethod
        def backward(ctx, *gs):
            have = [g for g in gs if g is not None]
            dense = [g if _dense(g) else g.contiguous() for g in have]
            outs = [torch.empty_like(g, dtype=torch.float32) for g in dense]
            if dense:
                launch(dense, outs, 1)
            it = iter(outs)
            return tuple(next(it) if g is not None else None for g in gs)

    return _CastBF16


_CAST_FN = None


def cast_bf16(*tensors):
    """bf16 copies of GPU fp32 ``tensors`` (differentiable) in one gfx950
    launch per direction -- the consumer step's weight casts without a
    separate cast kernel per layer.  Tensors must be dense (any strides)."""
    import torch
    global _CAST_FN
    if _CAST_FN is None:
        _CAST_FN = _cast_function()
    if len(tensors) > 32:
        raise ValueError('cast_bf16 takes at most 32 tensors per call')
    for t in tensors:
        if not (t.is_cuda and t.dtype == torch.float32 and _dense(t)):
            raise ValueError('cast_bf16 needs dense fp32 GPU tensors')
    return _CAST_FN.apply(*tensors)


# ---------------------------------------------------------------------------
# consumer-model op: training BatchNorm2d fused with LeakyReLU (channels-last)

class BnAccumulator:
    """Zeroed fp64 statistics accumulators of one BatchNorm+LeakyReLU call
    (csrc/gpu/kernels.h ``BnAcc``): the producing kernel -- the convolution's
    forward epilogue (``fwd``) or the consuming convolution's data-gradient
    epilogue (``bwd``) -- adds its per-tile channel sums into them with fp64
    atomics (order-independent at fp32 precision), and one finalize block
    folds and clears them again: no per-tile partial rows, no per-step
    memset, and the finalize is one memory latency instead of a walk over
    ~4800 rows per channel.  ``R`` replicas per channel spread the atomics."""
    __slots__ = ('fwd', 'bwd', 'R')

    def __init__(self, C, device):
        import torch
        ext = hip_ext()
        self.R = int(ext.bn_acc_replicas(int(C)))
        n = int(ext.bn_acc_elems(int(C)))
        if self.R <= 0 or n <= 0:
            raise ValueError(f'BnAccumulator: unsupported channel count {C}')
        self.fwd = torch.zeros(n, dtype=torch.float64, device=device)
        self.bwd = torch.zeros(n, dtype=torch.float64, device=device)


def bn_acc_supported(C):
    """True when :class:`BnAccumulator` takes ``C`` channels."""
    return int(hip_ext().bn_acc_replicas(int(C))) > 0


class BnLink:
    """Hand-off between a training :class:`BatchNormLeakyReLU2d` and the
    convolution that consumes its output (:func:`conv4x4s2` ``bn_link=``).

    The BN forward records what its backward needs (its input ``x``, batch
    ``mean``/``invstd``, affine ``w``/``b``, ``slope``).  The convolution's
    backward, which runs first, computes the BN's gy as its data gradient and
    has the MFMA kernel's epilogue sum gz and gz * xhat per tile into
    ``part``; the BN backward then only finalizes and applies (one pass over
    the activation fewer).  ``part`` is consumed once."""
    __slots__ = ('x', 'mean', 'invstd', 'w', 'b', 'slope', 'part', 'rows', 'gy', 'acc', 'params', 'dw', 'db',
                 'dw_sunk', 'db_sunk', 'folded', 'defer_fold', 'applied')

    def __init__(self):
        self.x = self.mean = self.invstd = self.w = self.b = self.part = self.gy = None
        self.slope, self.rows = 0.0, 0
        self.acc = None      # BnAccumulator of the BN call (accumulator mode: part = acc.bwd, rows = -R)
        self.params = None   # the BN's (weight, bias) parameters
        # accumulator mode: the BN's weight / bias gradients when the consuming
        # conv's weight-gradient launch already folded the accumulator into them
        self.dw = self.db = None
        self.dw_sunk = self.db_sunk = self.folded = False
        # the BN hands its backward to the convolution that produced its input
        # (BnDeferred, BnBwdFold): that one folds the accumulator, not the consumer
        self.defer_fold = False
        # the consumer (the fused head) applied this BN's backward itself: its
        # gradient IS the BN's input gradient, dw / db are in dw / db
        self.applied = False

    def fold_args(self, M):
        """``(acc, R, C, M, dw, db)`` for ``conv_wgrad(fold=)``: fold this BN's
        backward accumulator into its weight / bias gradients -- their
        bucket views when fresh (``parallel.GradBuckets``), else new tensors
        the BN backward returns.  Marks the link folded."""
        import torch
        self.dw, self.dw_sunk = _grad_dest(self.params[0], self.w)
        self.db, self.db_sunk = _grad_dest(self.params[1], self.b)
        if self.dw.dtype != torch.float32 or not self.dw.is_contiguous():
            self.dw, self.dw_sunk = torch.empty_like(self.w), False
        if self.db.dtype != torch.float32 or not self.db.is_contiguous():
            self.db, self.db_sunk = torch.empty_like(self.b), False
        self.folded = True
        return (self.acc.bwd.data_ptr(), self.acc.R, int(self.w.numel()), int(M), self.dw.data_ptr(),
                self.db.data_ptr())

    def ready(self, dx):
        """True when the recorded BN input matches ``dx`` (shape, bf16 NHWC)."""
        import torch
        x = self.x
        return (x is not None and x.dtype == torch.bfloat16 and dx.dtype == torch.bfloat16
                and tuple(x.shape) == (dx.shape[0], dx.shape[2], dx.shape[3], dx.shape[1]) and x.is_contiguous())

    def take(self, gys):
        """The epilogue partials, if they were computed for exactly ``gys``
        (``rows < 0``: accumulator mode, ``part`` = the ``-rows``-replica
        accumulator).  An accumulator filled for another gradient is cleared."""
        part, rows, gy = self.part, self.rows, self.gy
        self.part = self.gy = None
        if part is None or gy is None or gys.data_ptr() != gy.data_ptr():
            if part is not None and rows < 0:
                part.zero_()
            return None, 0
        return part, rows


class BnBwdFold:
    """A BatchNorm+LeakyReLU backward handed to the weight gradient of the
    convolution that produced the BN's input (:class:`BnDeferred`,
    ``conv_wgrad(bn_dy=)``): the BN's saved input ``x`` (NHWC), batch
    ``mean``/``invstd``, affine ``w``/``b``, ``slope``, its accumulator
    ``acc`` (the backward sums the consumer's data gradient -- or the head --
    added), the destinations of its ``dw``/``db`` gradients (``done``: the
    parameters whose bucket views they are) and ``gx_out``, the BN's input
    gradient (set by the convolution for its data gradient)."""
    __slots__ = ('x', 'mean', 'invstd', 'w', 'b', 'slope', 'acc', 'dw', 'db', 'done', 'gx_out', 'assign')

    def __init__(self, x, mean, invstd, w, b, slope, acc, dw, db, done, assign=()):
        self.x, self.mean, self.invstd, self.w, self.b, self.slope = x, mean, invstd, w, b, slope
        self.acc, self.dw, self.db, self.done = acc, dw, db, done
        # (param, tensor): gradients that are not bucket views, set on the parameters once the kernel
        # that writes them is enqueued (returning them from the BN backward would let autograd copy
        # them before they are written)
        self.assign = assign
        self.gx_out = None


class BnDeferred:
    """Hand-off of a BatchNorm+LeakyReLU backward to the 4-channel first
    convolution that produced the BN's input (:func:`conv4x4s2` ``bn_out=``).

    That convolution's input is the frames (no data gradient), so the BN's
    input gradient gx feeds nothing but its weight-gradient kernel, which
    can compute gx itself while staging it (``conv_wgrad(bn_dy=)``): the BN
    backward then skips its apply pass -- one read of the activation and of
    its gradient and one write fewer -- and passes its output gradient on.
    ``armed``: set by the convolution (it accepts the hand-off); ``pending``:
    the BN's saved tensors and folded sums, set by its backward, taken once."""
    __slots__ = ('armed', 'pending')

    def __init__(self):
        self.armed = False
        self.pending = None

    def take(self):
        p, self.pending = self.pending, None
        return p


class BnActLazy:
    """Hand-off of a training BatchNorm+LeakyReLU's FORWARD apply to the op
    that consumes its output (the next MFMA convolution, :func:`conv4x4s2`
    ``act=``, or the fused discriminator head, :func:`disc_head_bce`
    ``act=``): the BN call returns its input ``y``
    unchanged and records here what the consumer needs to compute
    ``leaky(bn(y))`` itself while it reads ``y`` -- the statistics
    accumulator its blocks fold (block 0 writes mean / invstd and the running
    statistics, the last clears it), the affine parameters and the slope
    (``csrc/gpu/kernels.h`` ``BnActIn``).  No apply pass, no activation
    tensor.  ``args`` is consumed once."""
    __slots__ = ('args', 'keep')

    def __init__(self):
        self.args = None
        self.keep = None

    def take(self):
        a, self.args = self.args, None
        if a is None:
            raise RuntimeError('BnActLazy: no pending BatchNorm apply (never set, or already consumed)')
        return a


class BnProduced:
    """Hand-off of a training BatchNorm+LeakyReLU's FORWARD apply to the
    convolution that PRODUCES its input (the u8 first layer, :func:`conv_fwd`
    ``out_bn=``): made by the BN module (:meth:`BatchNormLeakyReLU2d.produced_by_conv`)
    before the convolution runs, so the kernel has the affine parameters and
    the mean / invstd / running-statistics destinations; the kernel waits for
    every block's statistics at a grid barrier, folds them and writes
    ``y = leaky(bn(z))`` next to ``z``.  The BN call then launches nothing and
    returns ``y`` (``z`` stays its saved input).  ``y`` / ``z``: set by the
    convolution when it applied the BN (else None: the BN applies itself)."""
    __slots__ = ('w', 'b', 'mean', 'invstd', 'eps', 'momentum', 'slope', 'rm', 'rv', 'tracked', 'y', 'z')

    def __init__(self, w, b, mean, invstd, eps, momentum, slope, rm, rv, tracked):
        self.w, self.b, self.mean, self.invstd = w, b, mean, invstd
        self.eps, self.momentum, self.slope = float(eps), float(momentum), float(slope)
        self.rm, self.rv, self.tracked = rm, rv, tracked
        self.y = self.z = None

    def args(self, acc, R, M):
        """The kernel's BnActIn tuple for accumulator ``acc`` (fp64, ``R``
        replicas) over ``M`` elements per channel."""
        ptr = (lambda t: t.data_ptr() if t is not None else 0)
        return (acc.data_ptr(), int(R), int(M), self.eps, self.momentum, self.w.data_ptr(), self.b.data_ptr(),
                self.slope, self.mean.data_ptr(), self.invstd.data_ptr(), ptr(self.rm), ptr(self.rv),
                ptr(self.tracked))


def _bn_function():
    import torch

    class _BatchNormLeakyReLU(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, slope, tracked=None,
                    stats=None, link=None, defer=None, lazy=None):
            ext = hip_ext()
            N, C, H, W = x.shape
            M = N * H * W
            dt = _dt(x)
            xs = _as_nhwc(x)
            w = weight.detach().float().contiguous()
            b = bias.detach().float().contiguous()
            mean = torch.empty(C, dtype=torch.float32, device=x.device)
            invstd = torch.empty_like(mean)
            rm = running_mean.data_ptr() if running_mean is not None else 0
            rv = running_var.data_ptr() if running_var is not None else 0
            tr = tracked.data_ptr() if tracked is not None else 0
            if lazy is not None and not (isinstance(stats, BnAccumulator) and dt == OUT_DTYPES['bfloat16']):
                raise ValueError('BatchNormLeakyReLU2d(lazy=): bf16 input with accumulated statistics only')
            produced = lazy if isinstance(lazy, BnProduced) else None
            if produced is not None:
                lazy = None
                if produced.y is None or produced.z is None or produced.z.data_ptr() != xs.data_ptr():
                    raise RuntimeError('BatchNormLeakyReLU2d: the producing convolution did not apply this BN')
            y = xs if lazy is not None else (_as_nhwc(produced.y) if produced is not None else torch.empty_like(xs))
            if produced is not None:
                # the producing convolution applied this op after its statistics (BnProduced): no launch
                _count('bn_forward_by_producer')
                w, b, mean, invstd = produced.w, produced.b, produced.mean, produced.invstd
                produced.y = produced.z = None
            elif lazy is not None:
                # the consumer applies this op while it reads x (BnActLazy): no launch here
                _count('bn_forward_lazy')
                lazy.args = (stats.fwd.data_ptr(), stats.R, M, float(eps), float(momentum), w.data_ptr(),
                             b.data_ptr(), float(slope), mean.data_ptr(), invstd.data_ptr(), rm, rv, tr)
                lazy.keep = (stats, w, b, mean, invstd)
            elif isinstance(stats, BnAccumulator):
                # sums accumulated by the producing conv's epilogue; folded by the apply kernel
                _count('bn_forward_from_stats')
                _count('bn_forward_acc')
                ext.bn_forward_acc(xs.data_ptr(), y.data_ptr(), M, C, dt, stats.fwd.data_ptr(), stats.R, float(eps),
                                   float(momentum), mean.data_ptr(), invstd.data_ptr(), rm, rv, w.data_ptr(),
                                   b.data_ptr(), float(slope), _stream(x.device), tr)
            elif stats is not None:
                # per-tile sums from the producing conv's epilogue (conv_fwd): no reduction pass over x
                _count('bn_forward_from_stats')
                ext.bn_forward_from_stats(xs.data_ptr(), y.data_ptr(), M, C, dt, stats.data_ptr(),
                                          stats.numel() // (2 * C), float(eps), float(momentum), mean.data_ptr(),
                                          invstd.data_ptr(), rm, rv, w.data_ptr(), b.data_ptr(), float(slope),
                                          _stream(x.device), tr)
            else:
                part = torch.empty(ext.bn_partial_floats(M, C, dt), dtype=torch.float32, device=x.device)
                _count('bn_forward')
                ext.bn_forward(xs.data_ptr(), y.data_ptr(), M, C, dt, part.data_ptr(), float(eps), float(momentum),
                               mean.data_ptr(), invstd.data_ptr(), rm, rv, w.data_ptr(), b.data_ptr(), float(slope),
                               _stream(x.device), tr)
            ctx.save_for_backward(xs, w, b, mean, invstd)
            ctx.slope = float(slope)
            ctx.link = link
            ctx.defer = defer if (defer is not None and defer.armed and dt == OUT_DTYPES['bfloat16']) else None
            ctx.params = (weight, bias)
            ctx.acc = stats if isinstance(stats, BnAccumulator) else None
            if link is not None:
                link.x, link.mean, link.invstd, link.w, link.b, link.slope = xs, mean, invstd, w, b, float(slope)
                link.part = link.gy = None
                link.acc = ctx.acc
                link.params = (weight, bias)
                link.dw = link.db = None
                link.folded = False
                link.applied = False
                link.defer_fold = ctx.defer is not None and ctx.acc is not None
            return y.permute(0, 3, 1, 2)   # (lazy: a view of the input, the pre-BN values)

        @staticmethod
        def backward(ctx, gy):
            ext = hip_ext()
            xs, w, b, mean, invstd = ctx.saved_tensors
            N, H, W, C = xs.shape
            M = N * H * W
            dt = _dt(xs)
            gys = _as_nhwc(gy if gy.dtype == xs.dtype else gy.to(xs.dtype))
            gx = torch.empty_like(xs)
            lk = ctx.link
            if lk is not None and lk.applied:
                # the fused head applied this backward (disc_head_bce with the BN's sums
                # worked out in its forward): gy is the input gradient already
                lk.applied = False
                out_w = None if lk.dw_sunk else lk.dw
                out_b = None if lk.db_sunk else lk.db
                lk.dw = lk.db = None
                lk.part = lk.gy = None
                _count('bn_backward_by_head')
                return (gys.permute(0, 3, 1, 2), out_w, out_b, None, None, None, None, None, None, None, None, None,
                        None)
            folded = lk is not None and lk.folded
            part, rows = lk.take(gys) if lk is not None else (None, 0)
            if folded and part is not None and rows < 0:
                # the consuming conv's weight-gradient launch folded dw, db: apply only
                _count('bn_backward_from_stats')
                _count('bn_backward_acc')
                _count('bn_backward_folded')
                out_w = None if lk.dw_sunk else lk.dw
                out_b = None if lk.db_sunk else lk.db
                if ctx.defer is not None:
                    # the producing first convolution applies this backward while it
                    # stages its weight gradient's dY (BnDeferred): pass gy on unchanged
                    _count('bn_backward_deferred')
                    ctx.defer.pending = (xs, mean, invstd, w, b, lk.dw, lk.db, ctx.slope)
                    gx = gys
                else:
                    ext.bn_bwd_apply(xs.data_ptr(), gys.data_ptr(), gx.data_ptr(), M, C, dt, mean.data_ptr(),
                                     invstd.data_ptr(), w.data_ptr(), b.data_ptr(), lk.dw.data_ptr(),
                                     lk.db.data_ptr(), ctx.slope, _stream(xs.device))
                lk.dw = lk.db = None
                lk.folded = False
                return (gx.permute(0, 3, 1, 2), out_w, out_b, None, None, None, None, None, None, None, None, None,
                        None)
            if (not folded and ctx.defer is not None and ctx.acc is not None and part is not None and rows < 0
                    and part.data_ptr() == ctx.acc.bwd.data_ptr()):
                # the consumer filled the backward accumulator: the convolution that produced x
                # folds it and applies this backward while staging its weight gradient's dY
                # (BnBwdFold) -- gy passes on unchanged.  The dw / db it writes must not be
                # accumulated into an existing .grad before that launch: bucket views or unset.
                # eligibility first, without consuming the bucket views' fresh flags: a
                # fall-through must leave both for the general path's _grad_dest below
                # (else its parameter reports late and its bucket loses the overlap)
                if all(p.grad is None or _grad_sink_ready(p) for p in ctx.params):
                    dw, w_sunk = _grad_dest(ctx.params[0], w)
                    db, b_sunk = _grad_dest(ctx.params[1], b)
                    _count('bn_backward_from_stats')   # (the sums: from the consumer's epilogue)
                    _count('bn_backward_deferred_fold')
                    sunk = (w_sunk, b_sunk)
                    ctx.defer.pending = BnBwdFold(xs, mean, invstd, w, b, ctx.slope, ctx.acc, dw, db,
                                                  tuple(p for p, sk in zip(ctx.params, sunk) if sk),
                                                  tuple((p, g) for p, g, sk in zip(ctx.params, (dw, db), sunk)
                                                        if not sk and p.requires_grad))
                    return (gys.permute(0, 3, 1, 2), None, None, None, None, None, None, None, None, None, None,
                            None, None)
            if folded:
                raise RuntimeError('BatchNormLeakyReLU2d: its statistics were folded for another gradient')
            # (not before the folded branch: the fold already took the bucket views)
            dw, w_sunk = _grad_dest(ctx.params[0], w)
            db, b_sunk = _grad_dest(ctx.params[1], b)
            if dw.dtype != torch.float32 or not dw.is_contiguous():
                dw, w_sunk = torch.empty_like(w), False
            if db.dtype != torch.float32 or not db.is_contiguous():
                db, b_sunk = torch.empty_like(b), False
            if ctx.acc is not None and (part is None or rows < 0):
                # accumulator mode: the consuming conv's dgrad epilogue summed into
                # acc.bwd (part), or this launch reduces into it first
                _count('bn_backward_from_stats' if part is not None else 'bn_backward')
                _count('bn_backward_acc')
                ext.bn_backward_acc(xs.data_ptr(), gys.data_ptr(), gx.data_ptr(), M, C, dt, ctx.acc.bwd.data_ptr(),
                                    ctx.acc.R, mean.data_ptr(), invstd.data_ptr(), w.data_ptr(), b.data_ptr(),
                                    dw.data_ptr(), db.data_ptr(), ctx.slope, _stream(xs.device), part is None)
            elif part is not None:
                # the consuming convolution's data-gradient epilogue already summed gz, gz * xhat
                _count('bn_backward_from_stats')
                ext.bn_backward_from_stats(xs.data_ptr(), gys.data_ptr(), gx.data_ptr(), M, C, dt, part.data_ptr(),
                                           rows, mean.data_ptr(), invstd.data_ptr(), w.data_ptr(), b.data_ptr(),
                                           dw.data_ptr(), db.data_ptr(), ctx.slope, _stream(xs.device))
            else:
                part = torch.empty(ext.bn_partial_floats(M, C, dt), dtype=torch.float32, device=xs.device)
                _count('bn_backward')
                ext.bn_backward(xs.data_ptr(), gys.data_ptr(), gx.data_ptr(), M, C, dt, part.data_ptr(),
                                mean.data_ptr(), invstd.data_ptr(), w.data_ptr(), b.data_ptr(), dw.data_ptr(),
                                db.data_ptr(), ctx.slope, _stream(xs.device))
            _grad_done(ctx.params[0] if w_sunk else None, ctx.params[1] if b_sunk else None)
            return (gx.permute(0, 3, 1, 2), None if w_sunk else dw, None if b_sunk else db,
                    None, None, None, None, None, None, None, None, None, None)

    return _BatchNormLeakyReLU


_BN_FN = None
_BN_SHAPES = {}


def bn_supported(x):
    """True when the fused kernels take ``x`` (GPU fp32/bf16, 16-byte channel
    groups that tile a 256-lane block)."""
    dt = _dt(x)
    if dt is None or not x.is_cuda or x.dim() != 4:
        return False
    N, C, H, W = x.shape
    key = (C, dt)
    ok = _BN_SHAPES.get(key)
    if ok is None:     # the kernels' shape rule depends on C and dtype only
        ok = _BN_SHAPES[key] = hip_ext().bn_partial_floats(1, C, dt) > 0
    return ok


def batch_norm_leaky_relu(x, weight, bias, running_mean=None, running_var=None, eps=1e-5, momentum=0.1,
                          slope=0.2):
    """``leaky_relu(batch_norm(x, training=True), slope)`` on the gfx950
    kernels; updates ``running_mean``/``running_var`` in place like PyTorch
    (unbiased variance, ``momentum``)."""
    global _BN_FN
    if _BN_FN is None:
        _BN_FN = _bn_function()
    if not bn_supported(x):
        raise ValueError(f'batch_norm_leaky_relu: unsupported input {x.dtype} {tuple(x.shape)} on {x.device}')
    return _BN_FN.apply(x, weight, bias, running_mean, running_var, eps, momentum, slope)


def _bn_apply_unchecked(x, weight, bias, running_mean, running_var, eps, momentum, slope, tracked=None,
                        stats=None, link=None, defer=None, lazy=None):
    return _BN_FN.apply(x, weight, bias, running_mean, running_var, eps, momentum, slope, tracked, stats, link,
                        defer, lazy)


def reference_batch_norm_leaky_relu(x, weight, bias, running_mean=None, running_var=None, eps=1e-5, momentum=0.1,
                                    slope=0.2):
    """fp32 reference (PyTorch)."""
    import torch.nn.functional as F
    y = F.batch_norm(x.float(), running_mean, running_var, weight, bias, training=True, momentum=momentum, eps=eps)
    return F.leaky_relu(y, slope)


_BN_MODULE = None


def _bn_module():
    import torch.nn as nn
    import torch.nn.functional as F

    class BatchNormLeakyReLU2d(nn.BatchNorm2d):
        """``nn.BatchNorm2d`` followed by ``LeakyReLU(slope)``; same parameters
        and buffers as ``nn.BatchNorm2d`` (state dicts interchange).  Training
        steps on GPU fp32/bf16 inputs run the fused gfx950 kernels; eval mode
        and other inputs run the PyTorch ops."""

        def __init__(self, num_features, slope=0.2, **kw):
            super().__init__(num_features, **kw)
            self.slope = slope

        def forward(self, x):
            if (self.training and self.affine and self.track_running_stats and self.momentum is not None
                    and bn_supported(x)):
                global _BN_FN
                if _BN_FN is None:
                    _BN_FN = _bn_function()
                # num_batches_tracked is incremented by the finalize kernel (one launch fewer)
                return _bn_apply_unchecked(x, self.weight, self.bias, self.running_mean, self.running_var,
                                           self.eps, self.momentum, self.slope, self.num_batches_tracked)
            return F.leaky_relu(super().forward(x), self.slope)

        def fused_with_stats(self, x):
            """True when :meth:`forward_from_stats` applies to ``x``."""
            return (self.training and self.affine and self.track_running_stats and self.momentum is not None
                    and bn_supported(x))

        def accumulator(self, device):
            """The next :class:`BnAccumulator` of this module's ring (4 per
            device): each training call takes its own, so the backward sums of
            up to 4 calls in flight (e.g. a real and a simulated batch through
            the same discriminator) never share one.  Not part of the state."""
            ring = self.__dict__.get('_bt_acc_ring')
            if ring is None or ring[0][0].fwd.device != device:
                ring = self.__dict__['_bt_acc_ring'] = [[BnAccumulator(self.num_features, device) for _ in range(4)],
                                                        0]
            accs, i = ring
            ring[1] = (i + 1) % len(accs)
            return accs[i]

        def produced_by_conv(self, device):
            """A :class:`BnProduced` for the convolution that produces this
            module's next training input: it may apply this op itself (pass
            it to :meth:`forward_from_stats` as ``lazy`` afterwards)."""
            import torch
            mean = torch.empty(self.num_features, dtype=torch.float32, device=device)
            return BnProduced(self.weight.detach().float().contiguous(), self.bias.detach().float().contiguous(),
                              mean, torch.empty_like(mean), self.eps, self.momentum, self.slope, self.running_mean,
                              self.running_var, self.num_batches_tracked)

        def forward_from_stats(self, x, stats, link=None, defer=None, lazy=None):
            """Training forward with the batch statistics already summed by
            the producing kernel (``conv_fwd``'s epilogue rows, see
            :func:`conv4x4s2`, or a :class:`BnAccumulator` it added into:
            then one apply launch folds them): finalize + apply only.  ``link``: a
            :class:`BnLink` shared with the convolution that consumes the
            output (its data-gradient epilogue then does this op's backward
            reduction).  ``defer``: a :class:`BnDeferred` armed by the first
            convolution that produced ``x`` (it then applies this op's
            backward itself).  ``lazy``: a :class:`BnActLazy` -- the
            consumer applies this op itself; returns ``x`` (pre-BN) -- or a
            :class:`BnProduced` the producing convolution filled (returns its
            ``y``; when the convolution did not apply it, pass None instead)."""
            global _BN_FN
            if _BN_FN is None:
                _BN_FN = _bn_function()
            return _bn_apply_unchecked(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps,
                                       self.momentum, self.slope, self.num_batches_tracked, stats, link, defer,
                                       lazy)

        def extra_repr(self):
            return super().extra_repr() + f', slope={self.slope}'

    BatchNormLeakyReLU2d.__module__ = __name__
    return BatchNormLeakyReLU2d


# ---------------------------------------------------------------------------
# consumer-model op: 4x4 / stride-2 / pad-1 convolution with a gfx950 MFMA
# weight gradient (csrc/gpu/conv.hip)

def conv_wgrad_supported(x, weight):
    """True when :func:`conv4x4s2` can take ``x`` (bf16 channels-last GPU
    activations) and ``weight`` ([Cout, Cin, 4, 4] fp32) on the MFMA path."""
    import torch
    if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.uint8) and x.dim() == 4 and weight.dim() == 4):
        return False
    cout, cin, kh, kw = weight.shape
    xc = x.shape[1]
    big = xc == cin and cin % 32 == 0 and cout % 64 == 0 and x.dtype == torch.bfloat16
    # RGBA-fed first layer: decoded bf16 frames, or the raw u8 frames (decode fused, lut=)
    first = xc == 4 and cin in (3, 4) and cout % 32 == 0
    return (kh, kw) == (4, 4) and (big or first) and x.is_contiguous(memory_format=torch.channels_last)


_LUTS = {}


def decode_lut_bf16(cfg: DecodeConfig, device):
    """bf16 [4 * 256] value table of ``cfg`` (RNE of :func:`build_lut`'s fp32
    table) on ``device``: what the first convolution reads raw u8 RGBA frames
    through (``conv4x4s2(..., lut=)``) -- the same values the decode kernel
    writes for a bf16 NHWC RGBA output.  Cached per (config, device)."""
    import torch
    if cfg.cmap != [0, 1, 2, 3] or cfg.flip or cfg.colour_kernel:
        raise ValueError('decode_lut_bf16: RGBA identity channel map, no flip, no colour matrix')
    key = (cfg, str(device))
    t = _LUTS.get(key)
    if t is None:
        t = _LUTS[key] = torch.from_numpy(build_lut(cfg).reshape(-1).copy()).to(torch.bfloat16).to(device)
    return t


# ops.FusedAdam.attach_reduce: the backward's last weight-gradient slice reduce
# handed to the optimizer's update launch (AdamParams::fr) instead of a launch
# of its own.  {'params': ids of the parameters the update takes, 'got': the
# deferred reduce (ext tuple, tensors to keep alive, param, device) or None}
_REDUCE_CLAIM = None


def _claim_flush():
    """Run a claimed slice reduce now (another weight gradient follows it in
    the backward, or no update takes it)."""
    c = _REDUCE_CLAIM
    if c is not None and c['got'] is not None:
        res, _keep, param, device = c['got']
        c['got'] = None
        hip_ext().conv_wgrad_reduce(res, _stream(device))
        _count('conv_wgrad_reduce_claim_flushed')
        _grad_done(param)


class WgradChain:
    """Weight-gradient launches of one backward pass that hand their slice
    reduce forward: each :func:`conv_wgrad` in the chain leaves its reduce to
    the next one, which runs it as extra blocks of its own launch; the call
    marked ``last`` runs its own (and the one handed to it) -- one reduce
    launch per chain instead of one per layer.  ``flush()`` runs a reduce
    left pending (a chain that ended before its ``last`` call)."""
    __slots__ = ('pending', 'keep', 'param')

    def __init__(self):
        self.pending = None   # the deferred reduce (ext tuple)
        self.keep = None      # its partial scratch and output, alive until run
        self.param = None     # the parameter whose (bucket-view) gradient it completes

    def flush(self, device):
        if self.pending is not None:
            side = _SIDE_STREAMS.get(device) if device in _SIDE_PENDING else None
            if side is not None:   # the pending reduce's partials may have been written on the side stream
                import torch
                torch.cuda.current_stream(device).wait_stream(side)
            hip_ext().conv_wgrad_reduce(self.pending, _stream(device))
            _grad_done(self.param)
            self.pending = self.keep = self.param = None


_WGRAD_BLOCKS = int(os.environ.get('BT_WGRAD_BLOCKS', '512'))
_C4W_BLOCKS = int(os.environ.get('BT_C4W_BLOCKS', str(_WGRAD_BLOCKS)))
# weight gradients on a side stream, concurrent with the data-gradient chain (BT_WGRAD_SIDE=1).  Off:
# measured 13.7k img/s against 19.5k in line -- each concurrent pair of latency-bound kernels ran ~1.8x
# its solo time (profiles/r5/b6: wgrad 44 us, dgrad 43 us side by side, 24 / 22 us alone)
_SIDE_WGRAD = os.environ.get('BT_WGRAD_SIDE', '0') not in ('', '0')
_SIDE_STREAMS = {}
_SIDE_KEEP = []   # main-stream tensors the side stream reads, until it joins the main stream
# devices whose side stream holds weight-gradient work of this backward not yet joined to the
# main stream: only then must a reduce or a gradient bucket's all-reduce wait for it (a stream
# that exists from an earlier run is not waited on -- inside a later capture that wait would
# reach work recorded outside the capture)
_SIDE_PENDING = set()


def _side_stream(device):
    import torch
    s = _SIDE_STREAMS.get(device)
    if s is None:
        s = _SIDE_STREAMS[device] = torch.cuda.Stream(device)
    return s


def set_side_wgrad(on):
    """Weight gradients on a side stream (True) or in line with the data
    gradients (False, the default); returns the previous setting."""
    global _SIDE_WGRAD
    prev, _SIDE_WGRAD = _SIDE_WGRAD, bool(on)
    return prev
# a layer's data and weight gradients in one launch (dgrad_wgrad_kernel; BT_FUSE_DW=0: two launches)
_FUSE_DW = os.environ.get('BT_FUSE_DW', '1') not in ('', '0')


def set_fuse_dw(on):
    """Data and weight gradients of a tap-GEMM layer in one launch (True, the
    default) or two (False); returns the previous setting."""
    global _FUSE_DW
    prev, _FUSE_DW = _FUSE_DW, bool(on)
    return prev


# first layer on raw u8 frames: its forward writes the decoded frames for its weight gradient (BT_C4_DECODED)
_C4_DECODED = os.environ.get('BT_C4_DECODED', '0') not in ('', '0')


def conv_wgrad(x, dy, out, target_blocks=None, chain=None, last=True, lut=None, fold=None, bn_dy=None, param=None,
               fold_params=()):
    """fp32 weight gradient of a 4x4/s2/p1 convolution into ``out`` ([Cout, Cin,
    4, 4], any strides): MFMA tiles over pixel slices + one slice-reduce
    launch.  ``x`` [N, Cin, H, W] and ``dy`` [N, Cout, H/2, W/2] are bf16 with
    channels-last memory.  ``chain`` (:class:`WgradChain`): run the chain's
    pending reduce inside this launch, and leave this layer's to the next
    call unless ``last`` -- ``out`` is then complete only after that call.
    ``lut``: ``x`` is raw u8 RGBA frames read through this decode table
    (:func:`decode_lut_bf16`).  ``bn_dy``: ``dy`` is the output gradient of
    the BatchNorm+LeakyReLU that follows this convolution, whose backward the
    kernel applies to ``dy`` while staging it (:class:`BnDeferred`) -- a
    :class:`BnBwdFold` (the kernel folds the BN's backward accumulator
    itself, writes the BN's dw / db and, for a layer with a data gradient,
    gx into ``gx_out``), or on the 4-channel first layer that BN's ``(x,
    mean, invstd, w, b, dw, db, slope)`` with the sums already folded.  ``param`` / ``fold_params``: the parameters
    whose bucket-view gradients ``out`` / the fold complete (reported to
    the gradient-completion listener once their launch is enqueued)."""
    import torch
    ext = hip_ext()
    N, Cin, H, W = x.shape
    Cout, Ho, Wo = dy.shape[1], dy.shape[2], dy.shape[3]
    cin_out = out.shape[1] if (Cin == 4 and out.dim() == 4 and out.shape[1] == 3) else Cin
    if dy.shape[0] != N or tuple(out.shape) != (Cout, cin_out, 4, 4) or out.dtype != torch.float32:
        raise ValueError(f'conv_wgrad: x {tuple(x.shape)}, dy {tuple(dy.shape)}, out {tuple(out.shape)} do not match')
    cl = torch.channels_last
    if not (x.is_contiguous(memory_format=cl) and dy.is_contiguous(memory_format=cl)):
        raise ValueError('conv_wgrad needs channels-last x and dy')
    M = N * Ho * Wo
    if target_blocks is None:
        # 2 blocks per CU (profiles/r2/conv_bench_v2.jsonl); BT_WGRAD_BLOCKS overrides (sweeps);
        # the first layer's kernel: BT_C4W_BLOCKS
        target_blocks = _C4W_BLOCKS if Cin == 4 else _WGRAD_BLOCKS
    slices = ext.conv_wgrad_slices(M, Cin, Cout, target_blocks)
    if slices <= 0:
        raise ValueError(f'conv_wgrad: unsupported channels Cin={Cin} Cout={Cout} (Cin % 32, Cout % 64)')
    px = -(-M // slices)
    px = -(-px // 32) * 32
    slices = -(-M // px)
    # the u8 first layer from a decoded input patch: its slices are bands of whole output rows
    rows = ext.conv_c4p_rows(N, H, W, Ho, Wo, Cout) if (lut is not None and Cin == 4) else 0
    if rows > 0:
        px = rows * Wo
        slices = M // px
    partial = torch.empty(slices * Cout * 16 * Cin, dtype=torch.float32, device=x.device)
    _count('conv_wgrad')
    _claim_flush()   # a reduce handed to the optimizer is not the backward's last after all
    side = chain.pending if chain is not None else None
    defer = chain is not None and not last
    # this layer's own reduce handed to the optimizer update (FusedAdam.attach_reduce): the first
    # contribution of this step, written into the parameter's gradient bucket view
    claim = _REDUCE_CLAIM
    hand = (not defer and claim is not None and param is not None and id(param) in claim['params']
            and _GRAD_DONE is None and not _SIDE_WGRAD and out is grad_sink(param))
    if (lut is not None) != (x.dtype == torch.uint8) or (lut is not None and Cin != 4):
        raise ValueError('conv_wgrad: u8 input (4 channels) needs its decode table lut, and only u8 takes one')
    bnt = None
    bn_done = ()
    if bn_dy is not None:
        if isinstance(bn_dy, BnBwdFold):   # sums folded in the kernel, gx written for the data gradient
            by, bmean, binv, bw, bb, bslope = bn_dy.x, bn_dy.mean, bn_dy.invstd, bn_dy.w, bn_dy.b, bn_dy.slope
            sums = (bn_dy.dw, bn_dy.db)
            gxo = bn_dy.gx_out
            if gxo is not None and (gxo.shape != dy.shape or gxo.dtype != torch.bfloat16
                                    or not gxo.is_contiguous(memory_format=cl) or Cin == 4):
                raise ValueError('conv_wgrad(bn_dy=): gx_out is shaped like dy (a layer with a data gradient)')
        else:
            by, bmean, binv, bw, bb, bdw, bdb, bslope = bn_dy
            sums = (bdw, bdb)
            if Cin != 4:
                raise ValueError('conv_wgrad(bn_dy=): given sums on the 4-channel first layer only')
        if tuple(by.shape) != (N, Ho, Wo, Cout) or by.dtype != torch.bfloat16 or not by.is_contiguous():
            raise ValueError('conv_wgrad(bn_dy=): BN input [N, Ho, Wo, Cout] bf16 NHWC')
        for t in (bmean, binv, bw, bb) + sums:
            if t.dtype != torch.float32 or t.numel() != Cout or not t.is_contiguous():
                raise ValueError('conv_wgrad(bn_dy=): fp32 [Cout] BN statistics / parameters / sums')
        _count('conv_wgrad_bn_dy')
        if isinstance(bn_dy, BnBwdFold):
            _count('conv_wgrad_bn_dy_fold')
            bnt = (by.data_ptr(), bmean.data_ptr(), binv.data_ptr(), bw.data_ptr(), bb.data_ptr(), 0, 0,
                   float(bslope), bn_dy.acc.bwd.data_ptr(), bn_dy.acc.R, bn_dy.dw.data_ptr(), bn_dy.db.data_ptr(),
                   gxo.data_ptr() if gxo is not None else 0)
            bn_done = bn_dy.done
        else:
            bnt = (by.data_ptr(), bmean.data_ptr(), binv.data_ptr(), bw.data_ptr(), bb.data_ptr(), bdw.data_ptr(),
                   bdb.data_ptr(), float(bslope))
    res = ext.conv_wgrad(x.data_ptr(), dy.data_ptr(), partial.data_ptr(), N, H, W, Cin, Ho, Wo, Cout, slices, px,
                         out.data_ptr(), out.stride(0), out.stride(1), out.stride(2), out.stride(3), _stream(x.device),
                         cin_out, defer or hand, side, lut.data_ptr() if lut is not None else 0, fold, bnt)
    if hand:
        if int(res[12]) > 0:   # the ordered reduce: the update sums it (AdamParams::fr)
            claim['got'] = (res, (partial, out), param, x.device)
            _count('conv_wgrad_reduce_handed')
        else:
            ext.conv_wgrad_reduce(res, _stream(x.device))
            hand = False
    if fold is not None:
        _count('conv_wgrad_bn_fold')
        _grad_done(*fold_params)
    if bn_done:
        _grad_done(*bn_done)
    if isinstance(bn_dy, BnBwdFold):
        for prm, grad in bn_dy.assign:   # (unset .grad, checked by the BN backward)
            prm.grad = grad if prm.grad is None else prm.grad + grad
    if chain is not None:
        if side is not None:
            _count('conv_wgrad_side_reduce')
            _grad_done(chain.param)
        chain.pending, chain.keep = (res, (partial, out)) if defer else (None, None)
        chain.param = param if defer else None
    if not defer and not hand:
        _grad_done(param)
    return out


def conv_fwd(x, w16, stats=None, acc_r=0, lut=None, act=None, act_out=None, out_bn=None):
    """y = conv2d(x, w16, stride 2, pad 1) on the gfx950 MFMA kernel: ``x``
    [N, Cin, H, W] bf16 channels-last, ``w16`` [Cout, Cin, 4, 4] bf16
    channels-last; returns channels-last bf16 y.  ``stats`` (optional fp32
    tensor of ``conv_fwd_stats_rows(M, Cout) * 2 * Cout``) receives per-tile
    BatchNorm sums of y, channel-major: ``stats.view(2, Cout, rows)`` holds
    the sums, then the sums of squares (see :func:`batch_norm_from_stats`).
    ``acc_r`` > 0: ``stats`` is a :class:`BnAccumulator`'s zeroed fp64
    ``fwd`` tensor with ``acc_r`` replicas, added into with atomics.
    ``lut`` (first layer): ``x`` is the raw u8 RGBA frames ([N, 4, H, W],
    channels-last) and ``lut`` their bf16 decode table (:func:`decode_lut_bf16`):
    the decode happens in the convolution's tile loads (``act_out``, bf16 like
    ``x``: also receives the decoded frames, for the weight gradient).  ``act``: the
    :class:`BnActLazy` of the BatchNorm+LeakyReLU whose INPUT ``x`` is -- the
    convolution applies it to its operand tiles; ``act_out`` (same shape as
    ``x``, optional) receives that activation.  ``out_bn`` (first layer, u8
    frames, accumulator): a :class:`BnProduced` of the BatchNorm+LeakyReLU
    whose input y is -- when :func:`conv1_bn_apply_fits`, the kernel applies it
    after a grid barrier and ``out_bn.y`` receives the activation (else
    ``out_bn.y`` stays None and the BN applies itself)."""
    import torch
    ext = hip_ext()
    N, Cin, H, W = x.shape
    if act_out is not None and (act is None and lut is None or act_out.shape != x.shape
                                or act_out.dtype != torch.bfloat16
                                or not act_out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError('conv_fwd: act_out is the activation of act (or, with lut, the decoded frames), '
                         'shaped and laid out like x')
    Cout = w16.shape[0]
    cl = torch.channels_last
    # first layer fed RGBA: a 3-input-channel weight, the 4th input channel ignored
    wc = 3 if (Cin == 4 and w16.shape[1] == 3) else Cin
    xdt = torch.uint8 if lut is not None else torch.bfloat16
    if tuple(w16.shape) != (Cout, wc, 4, 4) or w16.dtype != torch.bfloat16 or x.dtype != xdt:
        raise ValueError(f'conv_fwd: x {x.dtype} {tuple(x.shape)} / w {w16.dtype} {tuple(w16.shape)}')
    if lut is not None and (Cin != 4 or lut.dtype != torch.bfloat16 or lut.numel() != 1024 or lut.device != x.device):
        raise ValueError('conv_fwd: u8 input takes 4 channels and a bf16 [1024] decode table (decode_lut_bf16)')
    if not (x.is_contiguous(memory_format=cl) and w16.is_contiguous(memory_format=cl)):
        raise ValueError('conv_fwd needs channels-last x and weight')
    Ho, Wo = (H - 2) // 2 + 1, (W - 2) // 2 + 1
    y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=cl)
    _count('conv_fwd')
    if acc_r and (stats is None or stats.dtype != torch.float64 or stats.numel() < 2 * Cout * acc_r):
        raise ValueError('conv_fwd: acc_r needs an fp64 accumulator of 2 * Cout * acc_r elements')
    if act is not None:
        _count('conv_fwd_act')
    oargs, oy = None, None
    if out_bn is not None:
        out_bn.y = out_bn.z = None
        if acc_r and act is None and (lut is not None or Cin != 4) and conv_out_bn_fits(N, Ho, Wo, Cin, Cout,
                                                                                      x.device):
            oy = torch.empty_like(y)
            oargs = out_bn.args(stats, acc_r, N * Ho * Wo)
            _count('conv_fwd_bn_apply')
            _grid_barrier_armed()
    actp = act.take() if act is not None else None

    def launch(oargs, oy):
        ext.conv_fwd(x.data_ptr(), w16.data_ptr(), y.data_ptr(), stats.data_ptr() if stats is not None else 0,
                     N, H, W, Cin, Ho, Wo, Cout, _stream(x.device), wc if Cin == 4 else 0, int(acc_r),
                     lut.data_ptr() if lut is not None else 0, actp,
                     act_out.data_ptr() if act_out is not None else 0, oargs, oy.data_ptr() if oy is not None else 0)
    if oargs is not None:
        try:
            launch(oargs, oy)
        except RuntimeError:
            # the cooperative launch of the grid-barrier kernel was refused (its grid is
            # not co-resident with what else runs on the device): nothing ran -- the
            # plain forward, and the BatchNorm applies itself
            _count('conv_fwd_bn_apply_refused')
            oargs, oy = None, None
            launch(None, None)
    else:
        launch(None, None)
    if oy is not None:
        out_bn.y, out_bn.z = oy, y
    return y


def conv_out_bn_fits(N, Ho, Wo, Cin, Cout, device):
    """True when the forward kernel of a layer of this shape can also apply
    the BatchNorm+LeakyReLU of its output (:class:`BnProduced`; every block
    of the launch resident at once -- the occupancy is queried once; asked on
    every call, since the tile overrides (:func:`conv_set_tiles`) change the
    answer).  ``BT_CONV1_BN=0`` / ``BT_CONV_OUT_BN=0`` turn it off for the
    first layer / the others."""
    return bool(hip_ext().conv_out_bn_fits(int(N), int(Ho), int(Wo), int(Cin), int(Cout)))


def conv1_bn_apply_fits(N, Ho, Wo, Cout, device):
    """:func:`conv_out_bn_fits` of the 4-channel (u8 frames) first layer."""
    return conv_out_bn_fits(N, Ho, Wo, 4, Cout, device)


def conv_grid_barrier_timeouts():
    """Grid-barrier waits of the BN-applying forward kernels that gave up
    (the block went on instead of hanging the GPU); stays 0."""
    return int(hip_ext().conv_grid_barrier_timeouts())


# set once a grid-barrier (BN-applying forward) launch has been enqueued in this process
GRID_BARRIER_USED = False


class GridBarrierError(RuntimeError):
    """A BN-applying forward kernel's grid barrier timed out: some of its
    blocks were not co-resident (e.g. another stream or process held CUs), so
    the launch folded incomplete BatchNorm statistics."""


def _grid_barrier_armed():
    global GRID_BARRIER_USED
    if not GRID_BARRIER_USED:
        # host-mapped failure word, armed outside any capture the first time the
        # path is taken (the same launch's shape also ran eagerly before capture)
        if not hip_ext().conv_grid_barrier_arm():
            raise RuntimeError('conv_fwd: could not map the grid-barrier failure flag')
        GRID_BARRIER_USED = True
    check_grid_barrier()


def check_grid_barrier():
    """Raise :class:`GridBarrierError` if any grid barrier enqueued so far has
    been seen to give up.  A plain read of a host-mapped word (no HIP call, no
    synchronisation): a failure surfaces at the first check after the kernel
    ran.  Called by :func:`conv_fwd` and after every :class:`CapturedStep`;
    ``bench.py`` checks once more after its final synchronize.  The flag is
    sticky: :func:`clear_grid_barrier` resets it (tests)."""
    if GRID_BARRIER_USED and hip_ext().conv_grid_barrier_failed() > 0:
        raise GridBarrierError(
            f'a BN-applying convolution\'s grid barrier timed out ({conv_grid_barrier_timeouts()} waits gave up): '
            'the launch was not co-resident and folded incomplete BatchNorm statistics.  Run without '
            'BT_CONV1_BN / BT_CONV_OUT_BN, or keep other work off the GPU during the step')


def clear_grid_barrier(_simulate_failure=False):
    """Reset the sticky failure flag (``_simulate_failure``: set it, for tests)."""
    if GRID_BARRIER_USED:
        hip_ext().conv_grid_barrier_clear(1 if _simulate_failure else 0)


def conv_weights_t(weights):
    """[Cin*16*Cout] bf16 transposes ([ci][kh][kw][co]) of channels-last bf16
    conv weights, all in one launch: the data-gradient operands of a model's
    layers, made once per step (``conv_dgrad(..., wt=)``)."""
    import torch
    ws = [w.detach() for w in weights]
    outs = [torch.empty(w.numel(), dtype=torch.bfloat16, device=w.device) for w in ws]
    if ws:
        for w in ws:
            if not (w.dtype == torch.bfloat16 and w.is_contiguous(memory_format=torch.channels_last)):
                raise ValueError('conv_weights_t needs channels-last bf16 weights')
        _count('conv_weight_t_multi')
        hip_ext().conv_weight_t_multi([w.data_ptr() for w in ws], [o.data_ptr() for o in outs],
                                      [int(w.shape[0]) for w in ws], [int(w.shape[1]) for w in ws],
                                      _stream(ws[0].device))
    return outs


def conv_dgrad(dy, w16, in_shape, wt=None, bn=None):
    """Data gradient of :func:`conv_fwd` on the same MFMA kernel (four
    stride-2 parity classes, 4 taps each): ``dy`` [N, Cout, H/2, W/2] bf16
    channels-last, ``w16`` [Cout, Cin, 4, 4] bf16 channels-last -> dx
    [N, Cin, H, W] bf16 channels-last.

    ``bn`` (a :class:`BnLink` whose BatchNorm+LeakyReLU produced this
    convolution's input): dx is that BN backward's gy, and the kernel's
    epilogue also writes the BN backward's per-tile sums (``bn.part``), so the
    BN backward skips its reduction pass."""
    import torch
    ext = hip_ext()
    N, Cin, H, W = in_shape
    Cout = w16.shape[0]
    cl = torch.channels_last
    if not (dy.is_contiguous(memory_format=cl) and w16.is_contiguous(memory_format=cl)):
        raise ValueError('conv_dgrad needs channels-last dy and weight')
    if tuple(dy.shape) != (N, Cout, H // 2, W // 2) or dy.dtype != torch.bfloat16 or w16.dtype != torch.bfloat16:
        raise ValueError(f'conv_dgrad: dy {dy.dtype} {tuple(dy.shape)} / w {tuple(w16.shape)} vs input {in_shape}')
    if wt is None:
        wt = torch.empty(Cin * 16 * Cout, dtype=torch.bfloat16, device=dy.device)
        ext.conv_weight_t(w16.data_ptr(), wt.data_ptr(), Cout, Cin, _stream(dy.device))
    elif wt.numel() != Cin * 16 * Cout or wt.dtype != torch.bfloat16:
        raise ValueError('conv_dgrad: wt is not this weight\'s transpose (conv_weights_t)')
    dx = torch.empty((N, Cin, H, W), dtype=torch.bfloat16, device=dy.device, memory_format=cl)
    _count('conv_dgrad')
    if bn is not None and bn.ready(dx):
        _count('conv_dgrad_bn')
        if bn.acc is not None:
            # add into the BN call's zeroed backward accumulator (no partial rows, no finalize)
            part, acc_r, rows = bn.acc.bwd, bn.acc.R, -bn.acc.R
        else:
            acc_r, rows = 0, int(ext.conv_dgrad_bn_rows(N, H, W, Cin))
            part = torch.empty(2 * Cin * rows, dtype=torch.float32, device=dy.device)
        ext.conv_dgrad(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, _stream(dy.device),
                       bn.x.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(), bn.w.data_ptr(), bn.b.data_ptr(),
                       bn.slope, part.data_ptr(), max(rows, 0), acc_r)
        bn.part, bn.rows, bn.gy = part, rows, dx
    else:
        ext.conv_dgrad(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, _stream(dy.device))
    return dx


def conv_dgrad_supported(x, w):
    """True when :func:`conv_dgrad` takes the gradient of ``conv_fwd(x, w)``."""
    return (conv_fwd_supported(x, w) and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0
            and bool(hip_ext().conv_dgrad_supported(int(w.shape[1]), int(w.shape[0]))))


def conv_fwd_supported(x, w):
    import torch
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4):
        return False
    if not (x.dtype == torch.bfloat16 or (x.dtype == torch.uint8 and x.shape[1] == 4)):
        return False
    cout, cin, kh, kw = w.shape
    xc = x.shape[1]
    channels_ok = (xc == cin and cin >= 8 and cin & (cin - 1) == 0) or (xc == 4 and cin in (3, 4))
    return ((kh, kw) == (4, 4) and channels_ok and cout % 32 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and w.is_contiguous(memory_format=torch.channels_last))


def conv_fwd_stats_rows(M, Cout):
    """Partial-statistics rows :func:`conv_fwd` writes for M output pixels
    and Cout channels (one per pixel tile; the tile height depends on the
    GEMM's size)."""
    return int(hip_ext().conv_fwd_tiles(int(M), int(Cout)))


def conv_set_tiles(bm=0, bn=0, staging=-1, dgrad_cls=0):
    """Force the tap-GEMM tile: ``bm`` pixels (64/128) by ``bn`` output
    channels (32/64/128), its staging (0 = register ring, 2/3 = LDS-DMA
    stages) and the data gradient's parity classes per block (1 or 4); 0
    (-1 for staging) restores the automatic choice.  For tests and sweeps:
    call it between steps, never between sizing a statistics buffer
    (:func:`conv_fwd_stats_rows`) and the launch that fills it."""
    hip_ext().conv_set_tiles(int(bm), int(bn), int(staging), int(dgrad_cls))


def _conv_function():
    import torch
    import torch.nn.functional as F

    class _Conv4x4s2(torch.autograd.Function):
        """y = conv2d(x, w16, stride 2, pad 1) with MIOpen; backward: MIOpen
        data gradient, gfx950 MFMA weight gradient written in fp32 straight
        into the master weight's gradient (no bf16 round trip, no cast)."""

        @staticmethod
        def forward(ctx, x, w32, w16, with_stats=False, wt=None, bn_link=None, wchain=None, wlast=True, lut=None,
                    bn_out=None, act=None, bn_early=None):
            ctx.set_materialize_grads(False)   # no zero-filled gradient for the stats output
            if act is not None:
                # x is the input of the BN that produced this layer's input (BnActLazy): the
                # kernel applies it and writes the activation, which the weight gradient reads
                if not (isinstance(with_stats, BnAccumulator) and lut is None):
                    raise ValueError('conv4x4s2(act=): accumulator statistics on bf16 input only')
                xa = torch.empty_like(x, memory_format=torch.channels_last)
                ctx.save_for_backward(xa, w16)
                ctx.w32, ctx.wt, ctx.bn_link = w32, wt, bn_link
                ctx.wchain, ctx.wlast, ctx.lut, ctx.bn_out = wchain, wlast, None, None
                if bn_out is not None and w32.requires_grad:
                    bn_out.armed = True
                    ctx.bn_out = bn_out
                return conv_fwd(x, w16, with_stats.fwd, with_stats.R, act=act, act_out=xa)
            ctx.save_for_backward(x, w16)
            ctx.w32, ctx.wt, ctx.bn_link = w32, wt, bn_link
            ctx.wchain, ctx.wlast, ctx.lut = wchain, wlast, lut
            # the BN that consumes the output may hand its backward to this layer's
            # weight gradient (BnDeferred): with the sums already folded only without a
            # data gradient (frames in), else folded by the kernel (BnBwdFold)
            ctx.bn_out = None
            if bn_out is not None and w32.requires_grad:
                bn_out.armed = True
                ctx.bn_out = bn_out
            if lut is not None:   # raw u8 frames: the decode runs in the MFMA kernels' loads
                if isinstance(with_stats, BnAccumulator):
                    if _C4_DECODED and w32.requires_grad and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 \
                            and int(hip_ext().conv_tile_channels(int(w16.shape[0]), True)) == w16.shape[0]:
                        # the forward also writes the decoded frames: the weight gradient reads
                        # those (bf16) instead of decoding the u8 frames again
                        xd = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device,
                                         memory_format=torch.channels_last)
                        # (bn_early: the BN that consumes y is applied here too, BnProduced)
                        y = conv_fwd(x, w16, with_stats.fwd, with_stats.R, lut=lut, act_out=xd, out_bn=bn_early)
                        ctx.save_for_backward(xd, w16)
                        ctx.lut = None
                        return y
                    return conv_fwd(x, w16, with_stats.fwd, with_stats.R, lut=lut, out_bn=bn_early)
                if with_stats:
                    raise ValueError('conv4x4s2: u8 input takes accumulator statistics only')
                return conv_fwd(x, w16, lut=lut)
            if isinstance(with_stats, BnAccumulator):
                return conv_fwd(x, w16, with_stats.fwd, with_stats.R, out_bn=bn_early)
            if with_stats:
                N, _, H, W = x.shape
                M = N * ((H - 2) // 2 + 1) * ((W - 2) // 2 + 1)
                stats = torch.empty(conv_fwd_stats_rows(M, w16.shape[0]) * 2 * w16.shape[0], dtype=torch.float32,
                                    device=x.device)
                y = conv_fwd(x, w16, stats)
                ctx.mark_non_differentiable(stats)
                return y, stats
            if conv_fwd_supported(x, w16):
                return conv_fwd(x, w16)
            if w16.shape[1] != x.shape[1]:
                raise ValueError('conv4x4s2: an RGB weight on RGBA input needs the MFMA forward')
            return F.conv2d(x, w16, None, 2, 1)

        @staticmethod
        def backward(ctx, gy, gstats=None):
            x, w16 = ctx.saved_tensors
            bn_dy = ctx.bn_out.take() if ctx.bn_out is not None else None
            if gy is None:
                if ctx.wchain is not None and ctx.wlast:
                    ctx.wchain.flush(x.device)
                return None, None, None, None, None, None, None, None, None, None, None, None
            fold_bn = isinstance(bn_dy, BnBwdFold)
            if bn_dy is not None and ctx.needs_input_grad[0] and not fold_bn:
                raise RuntimeError('conv4x4s2: a deferred BN backward with folded sums needs a layer without a '
                                   'data gradient')
            gy = gy.contiguous(memory_format=torch.channels_last)
            gx = gw = None
            gy_dgrad = gy
            # the weight gradient on a side stream, concurrent with the data
            # gradient and the backward chain that follows it: both kernels are
            # latency-bound at a few waves per SIMD, so the other one's waves
            # fill the idle issue slots (a chain of weight gradients -- one
            # deferred reduce riding in the next launch -- stays on the side
            # stream).  The BN backward's statistics fold then runs in its own
            # apply launch instead of as an extra block of this weight
            # gradient (which would put it back on the critical path).  A
            # data-parallel bucket completed here is all-reduced on the side
            # stream, behind its weight gradients (GradBuckets._issue).
            side = None
            wg_done = False
            if (_SIDE_WGRAD and x.is_cuda and ctx.needs_input_grad[1] and ctx.wchain is not None
                    and not (fold_bn and ctx.needs_input_grad[0])):
                side = _side_stream(x.device)
                side.wait_stream(torch.cuda.current_stream(x.device))   # gy (and everything before it) is ready
                if ctx.needs_input_grad[0]:
                    # fork now: the weight gradient is enqueued before the data gradient
                    gw = _Conv4x4s2._wgrad_side(ctx, x, gy, bn_dy, side)
                    wg_done = True
            if fold_bn and ctx.needs_input_grad[0]:
                # the weight gradient runs first: it applies the BN backward to gy and writes
                # the BN's input gradient, this layer's true output gradient, for the data gradient
                bn_dy.gx_out = gy_dgrad = torch.empty_like(gy, memory_format=torch.channels_last)
                gw = _Conv4x4s2._wgrad(ctx, x, gy, None, None, bn_dy)
                bn_dy = None
            held = False
            if ctx.needs_input_grad[0]:
                if conv_dgrad_supported(x, w16):
                    # the data gradient held for the weight gradient below: both in one launch
                    # (dgrad_wgrad_kernel), unless the weight gradient runs elsewhere
                    hold = (_FUSE_DW and side is None and gy_dgrad is gy and ctx.needs_input_grad[1]
                            and x.is_cuda)
                    ext = hip_ext()
                    if hold:
                        ext.conv_dgrad_hold(1)
                    try:
                        gx = conv_dgrad(gy_dgrad, w16, tuple(x.shape), ctx.wt, ctx.bn_link)
                    finally:
                        if hold:
                            ext.conv_dgrad_hold(0)
                    held = hold and bool(ext.conv_dgrad_held())
                    if held:
                        _count('conv_dgrad_held')
                else:
                    wfull = w16
                    if w16.shape[1] != x.shape[1]:   # RGBA-fed RGB weight: zero weight on the extra channel
                        wfull = torch.cat([w16, w16.new_zeros(w16.shape[0], x.shape[1] - w16.shape[1], 4, 4)], 1)
                        wfull = wfull.contiguous(memory_format=torch.channels_last)
                    gx = torch.ops.aten.convolution_backward(gy_dgrad, x, wfull, None, [2, 2], [1, 1], [1, 1],
                                                             False, [0, 0], 1, [True, False, False])[0]
            if wg_done:
                pass
            elif gy_dgrad is gy and side is not None:   # (no data gradient: the chain's last, the first layer)
                gw = _Conv4x4s2._wgrad_side(ctx, x, gy, bn_dy, side)
            elif gy_dgrad is gy:   # (not already run before the data gradient)
                prior = _SIDE_STREAMS.get(x.device) if x.is_cuda and x.device in _SIDE_PENDING else None
                if prior is not None and ctx.wchain is not None and ctx.wchain.pending is not None:
                    # the chain's pending reduce reads partials an earlier launch wrote on the side stream
                    torch.cuda.current_stream(x.device).wait_stream(prior)
                fold = None
                bl = ctx.bn_link
                if gx is not None and bl is not None and bl.acc is not None and bl.part is not None and bl.rows < 0 \
                        and bl.params is not None and ctx.needs_input_grad[1] and x.shape[1] != 4 \
                        and not bl.defer_fold and not held:
                    # the data gradient just filled the BN's backward accumulator: the
                    # weight-gradient launch folds it in one extra block (not when both
                    # share a launch: the BN backward's apply folds it then)
                    fold = bl.fold_args(x.shape[0] * x.shape[2] * x.shape[3])
                try:
                    gw = _Conv4x4s2._wgrad(ctx, x, gy, fold, bl, bn_dy)
                finally:
                    if held:
                        hip_ext().conv_dgrad_flush()   # (no-op once the weight gradient launched both)
            return gx, gw, None, None, None, None, None, None, None, None, None, None

        @staticmethod
        def _wgrad_side(ctx, x, gy, bn_dy, side):
            """The weight gradient on the side stream (forked before the data
            gradient was enqueued, see backward): the stream joins the main one
            after the chain's last launch, or at once for a gradient autograd
            accumulates itself."""
            main = torch.cuda.current_stream(x.device)
            with torch.cuda.stream(side):
                _SIDE_PENDING.add(x.device)
                gw = _Conv4x4s2._wgrad(ctx, x, gy, None, ctx.bn_link, bn_dy)
            # x and gy live in main-stream memory the side stream still reads: they
            # stay referenced until the join (a block freed earlier could be handed
            # to a later main-stream tensor -- also inside a graph capture, where
            # record_stream does not order the reuse)
            _SIDE_KEEP.extend((x, gy))
            if ctx.wlast or gw is not None:
                main.wait_stream(side)
                _SIDE_KEEP.clear()
                _SIDE_PENDING.discard(x.device)
            return gw

        @staticmethod
        def _wgrad(ctx, x, gy, fold, bl, bn_dy):
            if not ctx.needs_input_grad[1]:
                if ctx.wchain is not None:
                    ctx.wchain.flush(x.device)
                return None
            out, sunk = _grad_dest(ctx.w32)
            # a chained (deferred) reduce only into a bucket view: a returned
            # gradient must be complete when autograd accumulates it
            chain = ctx.wchain if (sunk or ctx.wlast) else None
            if ctx.wchain is not None and chain is None:
                ctx.wchain.flush(x.device)
            fold_params = ()
            if fold is not None:
                fold_params = tuple(p for p, sk in zip(bl.params, (bl.dw_sunk, bl.db_sunk)) if sk)
            gw = conv_wgrad(x, gy, out, chain=chain, last=ctx.wlast or chain is None, lut=ctx.lut, fold=fold,
                            bn_dy=bn_dy, param=ctx.w32 if sunk else None, fold_params=fold_params)
            return None if sunk else gw   # (sunk: written into the parameter's bucket view)

    return _Conv4x4s2


_CONV_FN = None


def conv4x4s2(x, w32, w16, with_stats=False, wt=None, bn_link=None, wchain=None, wlast=True, lut=None,
              bn_out=None, act=None, bn_early=None):
    """4x4 / stride-2 / pad-1 convolution of bf16 channels-last ``x`` with the
    bf16 copy ``w16`` of fp32 weight ``w32``; the gradient goes to ``w32``
    (fp32, from the MFMA weight-gradient kernel).  See :func:`conv_wgrad_supported`.
    ``with_stats``: return ``(y, stats)``, the per-tile BatchNorm sums of y
    from the forward kernel's epilogue (for ``BatchNormLeakyReLU2d.forward_from_stats``);
    or a :class:`BnAccumulator` that the epilogue adds the sums into (returns y only).
    ``bn_link``: the :class:`BnLink` of the BatchNorm+LeakyReLU that produced
    ``x``; the data gradient then also computes that BN's backward sums.
    ``wchain`` / ``wlast``: the :class:`WgradChain` of the model's backward;
    ``wlast`` marks the layer whose weight gradient is computed last (the
    first layer).  ``lut``: ``x`` is raw u8 RGBA frames decoded through this
    table inside the kernels (:func:`decode_lut_bf16`; no gradient for ``x``).
    ``bn_out`` (with ``lut``): a :class:`BnDeferred` shared with the
    BatchNorm+LeakyReLU that consumes the output -- its backward apply then
    runs inside this layer's weight-gradient kernel.  ``act``: the
    :class:`BnActLazy` of the BatchNorm+LeakyReLU whose input ``x`` is (it
    skipped its apply): the forward kernel applies it while staging its
    operand tiles and writes the activation for the weight gradient.
    ``bn_early`` (with ``lut`` and a :class:`BnAccumulator`): a
    :class:`BnProduced` of the BatchNorm+LeakyReLU that consumes the output
    -- the forward kernel applies it too when :func:`conv1_bn_apply_fits`
    (check ``bn_early.y`` afterwards)."""
    global _CONV_FN
    if _CONV_FN is None:
        _CONV_FN = _conv_function()
    if with_stats and not conv_fwd_supported(x, w16):
        raise ValueError('conv4x4s2(with_stats=True) needs the MFMA forward (see conv_fwd_supported)')
    return _CONV_FN.apply(x, w32, w16.detach(), with_stats, wt, bn_link, wchain, wlast, lut, bn_out, act, bn_early)


# ---------------------------------------------------------------------------
# consumer-model op: the discriminator head (pool -> conv -> sigmoid -> BCE)
# in 2 + 2 launches (csrc/gpu/head.hip)

def _head_function():
    import torch

    class _DiscHeadBCE(torch.autograd.Function):
        @staticmethod
        def forward(ctx, z, w, target, oh, ow, bn_link=None, act=None):
            ctx.set_materialize_grads(False)   # no zero-filled gradient for the logits output
            ext = hip_ext()
            N, C, H, W = z.shape
            dev = z.device
            pooled = torch.empty(N * oh * ow * C, dtype=torch.float32, device=dev)
            # (4 per cell: the lean BN-applying forward writes one partial logit per wave, head.hip kHeadParts)
            partial = torch.empty(N * oh * ow * 4, dtype=torch.float32, device=dev)
            loss = torch.empty((), dtype=torch.float32, device=dev)
            dlogit = torch.empty(N, dtype=torch.float32, device=dev)
            logit = torch.empty(N, dtype=torch.float32, device=dev)
            tptr, tval = 0, 1.0
            if isinstance(target, torch.Tensor):
                target = target.to(device=dev, dtype=torch.float32).contiguous()
                tptr = target.data_ptr()
            else:
                tval = float(target)
            _count('head_forward')
            # the BN's backward sums worked out here, factored through dlogit (head_fwd_act_kernel):
            # the backward then applies that BN's backward itself (no apply launch)
            bn_ab = bn_sums = None
            if (act is not None and _HEAD_BN_BWD and bn_link is not None and bn_link.acc is not None
                    and bn_link.params is not None and not bn_link.defer_fold and act.args is not None
                    and ext.head_bn_bwd_supported(N, H, W, C, oh, ow, int(act.args[1]))):
                bn_ab = _head_bn_scratch(dev, N, C)
                bn_sums = torch.empty(2 * C, dtype=torch.float32, device=dev)
                _count('head_bn_sums')
            ext.head_forward(z.data_ptr(), w.data_ptr(), w.stride(1), w.stride(2), w.stride(3), N, H, W, C, oh, ow,
                             tptr, tval, pooled.data_ptr(), partial.data_ptr(), loss.data_ptr(), dlogit.data_ptr(),
                             logit.data_ptr(), _stream(dev), _head_ticket(dev).data_ptr(),
                             act.take() if act is not None else None,
                             bn_ab.data_ptr() if bn_ab is not None else 0,
                             bn_sums.data_ptr() if bn_sums is not None else 0)
            ctx.bn_sums = bn_sums
            ctx.save_for_backward(w, pooled, dlogit)
            ctx.wparam = w
            ctx.bn_link = bn_link
            ctx.zshape, ctx.pool = (N, C, H, W), (oh, ow)
            ctx.mark_non_differentiable(logit)
            return loss, logit

        @staticmethod
        def backward(ctx, gloss, glogit=None):
            if gloss is None:
                return None, None, None, None, None, None, None
            ext = hip_ext()
            w, pooled, dlogit = ctx.saved_tensors
            N, C, H, W = ctx.zshape
            oh, ow = ctx.pool
            g = gloss.to(torch.float32).reshape(1).contiguous()
            dz = torch.empty((N, C, H, W), dtype=torch.bfloat16, device=w.device, memory_format=torch.channels_last)
            dw, sunk = _grad_dest(ctx.wparam, w)
            if dw.stride() != w.stride():
                dw, sunk = torch.empty_like(w), False
            _count('head_backward')
            bn = ctx.bn_link
            if ctx.bn_sums is not None and bn is not None and bn.ready(dz) and bn.params is not None:
                # the BN's backward applied here: dz receives its INPUT gradient gx, the
                # BN backward passes it on (BnLink.applied)
                _count('head_backward_bn_apply')
                bdw, w_sunk = _grad_dest(bn.params[0], bn.w)
                bdb, b_sunk = _grad_dest(bn.params[1], bn.b)
                if bdw.dtype != torch.float32 or not bdw.is_contiguous():
                    bdw, w_sunk = torch.empty_like(bn.w), False
                if bdb.dtype != torch.float32 or not bdb.is_contiguous():
                    bdb, b_sunk = torch.empty_like(bn.b), False
                ext.head_backward(w.data_ptr(), w.stride(1), w.stride(2), w.stride(3), N, H, W, C, oh, ow,
                                  pooled.data_ptr(), dlogit.data_ptr(), g.data_ptr(), dz.data_ptr(), dw.data_ptr(),
                                  _stream(w.device), bn.x.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                                  bn.w.data_ptr(), bn.b.data_ptr(), bn.slope, 0, 0, ctx.bn_sums.data_ptr(),
                                  bdw.data_ptr(), bdb.data_ptr())
                bn.dw, bn.db, bn.dw_sunk, bn.db_sunk, bn.applied = bdw, bdb, w_sunk, b_sunk, True
                bn.part = bn.gy = None
                _grad_done(bn.params[0] if w_sunk else None, bn.params[1] if b_sunk else None)
            elif bn is not None and bn.acc is not None and bn.ready(dz) and (C // 8) <= 256 and 256 % (C // 8) == 0:
                # dz is the gy of the BN+LeakyReLU that produced z: sum its backward
                # statistics here, into the BN call's accumulator
                _count('head_backward_bn')
                ext.head_backward(w.data_ptr(), w.stride(1), w.stride(2), w.stride(3), N, H, W, C, oh, ow,
                                  pooled.data_ptr(), dlogit.data_ptr(), g.data_ptr(), dz.data_ptr(), dw.data_ptr(),
                                  _stream(w.device), bn.x.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                                  bn.w.data_ptr(), bn.b.data_ptr(), bn.slope, bn.acc.bwd.data_ptr(), bn.acc.R)
                bn.part, bn.rows, bn.gy = bn.acc.bwd, -bn.acc.R, dz
            else:
                ext.head_backward(w.data_ptr(), w.stride(1), w.stride(2), w.stride(3), N, H, W, C, oh, ow,
                                  pooled.data_ptr(), dlogit.data_ptr(), g.data_ptr(), dz.data_ptr(), dw.data_ptr(),
                                  _stream(w.device))
            if sunk:
                _grad_done(ctx.wparam)
            return dz, None if sunk else dw, None, None, None, None, None

    return _DiscHeadBCE


_HEAD_FN = None
# the fused head works out the BN's backward sums in its forward and applies that backward in
# its own (BT_HEAD_BN_BWD=0: the head sums into the BN's accumulator and the BN applies)
_HEAD_BN_BWD = os.environ.get('BT_HEAD_BN_BWD', '1') not in ('', '0')


_HEAD_TICKETS = {}
_HEAD_BN_SCRATCH = {}


def _head_bn_scratch(dev, N, C):
    """The zeroed [2][N][C] fp64 A / B scratch of the head forward's BN sums
    (cleared again by the kernel's last block; fp64 so the per-window adds
    give the same sums in any order -- the step stays deterministic)."""
    import torch
    key = (dev, int(N), int(C))
    t = _HEAD_BN_SCRATCH.get(key)
    if t is None:
        t = _HEAD_BN_SCRATCH[key] = torch.zeros(2 * N * C, dtype=torch.float64, device=dev)
    return t


def _head_ticket(dev):
    """The zeroed ticket word the one-launch head forward hands its partial
    logits over with (reset by the kernel's last block)."""
    import torch
    t = _HEAD_TICKETS.get(dev)
    if t is None:
        t = _HEAD_TICKETS[dev] = torch.zeros(4, dtype=torch.int32, device=dev)
    return t


def disc_head_bce(z, w, target=1.0, pool=(4, 4), bn_link=None, act=None):
    """``BCELoss()(sigmoid(conv2d(adaptive_avg_pool2d(z, pool), w)).view(-1), target)``
    for a head conv that consumes the whole pooled map (``w``: fp32
    [1, C, pool_h, pool_w]); ``z`` bf16 channels-last [N, C, H, W] on the GPU.
    Returns ``(loss, logits)``; gradients flow to ``z`` (bf16) and ``w``
    (fp32).  Pool, dot products and loss run in fp32.  ``bn_link``: the
    :class:`BnLink` of the BatchNorm+LeakyReLU that produced ``z`` (in
    accumulator mode): the backward then also sums that BN's backward
    statistics.  ``act``: that BN's :class:`BnActLazy` -- ``z`` is then the
    BN's INPUT and the head's pooling applies the BN (its forward launch
    skipped the apply)."""
    import torch
    global _HEAD_FN
    if _HEAD_FN is None:
        _HEAD_FN = _head_function()
    oh, ow = pool
    if not (z.is_cuda and z.dtype == torch.bfloat16 and z.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError('disc_head_bce needs bf16 channels-last GPU features')
    if tuple(w.shape) != (1, z.shape[1], oh, ow) or w.dtype != torch.float32 or z.shape[1] % 8:
        raise ValueError(f'disc_head_bce: weight {tuple(w.shape)} {w.dtype} does not fit features {tuple(z.shape)}')
    return _HEAD_FN.apply(z, w, target, oh, ow, bn_link, act)


def __getattr__(name):
    # built on first use so importing ``blendtorch.ops`` does not import torch
    global _POOL_MODULE, _BN_MODULE
    if name == 'AdaptiveAvgPool2d':
        if _POOL_MODULE is None:
            _POOL_MODULE = _pool_module()
        return _POOL_MODULE
    if name == 'BatchNormLeakyReLU2d':
        if _BN_MODULE is None:
            _BN_MODULE = _bn_module()
        return _BN_MODULE
    if name == 'FusedAdam':
        from .adam import FusedAdam
        return FusedAdam
    raise AttributeError(f'module {__name__!r} has no attribute {name!r}')
