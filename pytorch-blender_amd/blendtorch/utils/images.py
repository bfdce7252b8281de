"""Image grids as PNG files without torchvision (not installed here).

The densityopt example of the reference writes the target and simulated
batches every 5 epochs with ``torchvision.utils.save_image(x, path,
normalize=True)`` (reference: examples/densityopt/densityopt.py:321-323).
:func:`save_image` reproduces that output: the batch is tiled into a grid of
``nrow`` columns with ``padding`` pixels of ``pad_value`` between tiles
(``make_grid``), scaled min-max to [0, 1] over the whole tensor when
``normalize`` (before padding, as torchvision does), quantised as
``clamp(x * 255 + 0.5, 0, 255)`` and written as an 8-bit RGB (or grey) PNG
with the standard library's zlib.
"""
from __future__ import annotations

import struct
import zlib
from pathlib import Path

import numpy as np

__all__ = ['make_grid', 'save_image', 'write_png', 'read_png']


def _to_numpy(x):
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return x.detach().float().cpu().numpy()
    except ImportError:   # pragma: no cover - torch is always present in this repo
        pass
    return np.asarray(x, dtype=np.float32)


def make_grid(x, nrow: int = 8, padding: int = 2, normalize: bool = False, pad_value: float = 0.0) -> np.ndarray:
    """[B, C, H, W] (or [C, H, W]) -> one float32 [C, gh, gw] image of the
    batch in rows of ``nrow`` tiles, ``padding`` pixels apart."""
    a = _to_numpy(x).astype(np.float32)
    if a.ndim == 3:
        a = a[None]
    if a.ndim != 4:
        raise ValueError(f'make_grid: expected [B, C, H, W], got shape {a.shape}')
    if a.shape[1] == 1:
        a = np.repeat(a, 3, axis=1)
    if normalize:
        lo, hi = float(a.min()), float(a.max())
        a = (a - lo) / max(hi - lo, 1e-5)
    B, C, H, W = a.shape
    cols = min(nrow, B)
    rows = -(-B // cols)
    hh, ww = H + padding, W + padding
    grid = np.full((C, rows * hh + padding, cols * ww + padding), pad_value, dtype=np.float32)
    for k in range(B):
        r, c = divmod(k, cols)
        grid[:, r * hh + padding:r * hh + padding + H, c * ww + padding:c * ww + padding + W] = a[k]
    return grid


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)


def write_png(path, img: np.ndarray, level: int = 6):
    """Write a u8 [H, W] (grey) or [H, W, 3] (RGB) array as a PNG."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim == 2:
        ctype = 0
    elif img.ndim == 3 and img.shape[2] == 3:
        ctype = 2
    else:
        raise ValueError(f'write_png: expected [H, W] or [H, W, 3] u8, got {img.shape}')
    h, w = img.shape[:2]
    rows = img.reshape(h, -1)
    raw = np.empty((h, rows.shape[1] + 1), dtype=np.uint8)
    raw[:, 0] = 0                       # filter type None per scanline
    raw[:, 1:] = rows
    png = b'\x89PNG\r\n\x1a\n' + _chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, 8, ctype, 0, 0, 0))
    png += _chunk(b'IDAT', zlib.compress(raw.tobytes(), level)) + _chunk(b'IEND', b'')
    Path(path).write_bytes(png)


def read_png(path) -> np.ndarray:
    """Read back a PNG written by :func:`write_png` (8-bit grey/RGB, filter 0)."""
    data = Path(path).read_bytes()
    if data[:8] != b'\x89PNG\r\n\x1a\n':
        raise ValueError('not a PNG')
    pos, idat, hdr = 8, b'', None
    while pos < len(data):
        n, tag = struct.unpack('>I4s', data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if tag == b'IHDR':
            hdr = struct.unpack('>IIBBBBB', body)
        elif tag == b'IDAT':
            idat += body
        pos += 12 + n
    w, h, depth, ctype = hdr[0], hdr[1], hdr[2], hdr[3]
    ch = {0: 1, 2: 3}[ctype]
    raw = np.frombuffer(zlib.decompress(idat), dtype=np.uint8).reshape(h, 1 + w * ch)
    if (raw[:, 0] != 0).any() or depth != 8:
        raise ValueError('read_png: only 8-bit, unfiltered scanlines')
    img = raw[:, 1:].reshape(h, w, ch)
    return img[:, :, 0] if ch == 1 else img


def save_image(x, path, nrow: int = 8, padding: int = 2, normalize: bool = False, pad_value: float = 0.0):
    """``torchvision.utils.save_image`` equivalent for [B, C, H, W] batches
    (C = 1 or 3; a 4th channel is dropped)."""
    a = _to_numpy(x)
    if a.ndim == 4 and a.shape[1] == 4:
        a = a[:, :3]
    grid = make_grid(a, nrow=nrow, padding=padding, normalize=normalize, pad_value=pad_value)
    u8 = np.clip(grid * 255.0 + 0.5, 0, 255).astype(np.uint8).transpose(1, 2, 0)
    write_png(path, u8)
    return u8
