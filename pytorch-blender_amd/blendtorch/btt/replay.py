"""HBM-resident replay of rendered frames.

The reference replays recordings from disk. :class:`FileDataset` unpickles every
``.btr`` message on every epoch, in DataLoader workers, and collates on the host
(pkg_pytorch/blendtorch/btt/dataset.py:119-153, file.py:81-132).
:class:`DeviceReplayBuffer` keeps the raw u8 frames in GPU memory instead. An
MI355X has 288 GB of HBM3E, which holds about 230k 640x480 RGBA frames. Every
epoch after the first then runs at HBM speed without touching the host:

* ``from_recordings(prefix)``: the ``.btr`` files are memory-mapped, and each
  message is scanned in place by the native pickle codec (zero-copy views, no
  unpickling of the image). The image bytes are staged through a pinned buffer
  into the device store in large chunks.
* ``extend(images, **meta)``: append frames (ring semantics: the oldest are
  overwritten once ``capacity`` is reached). The frames can be device tensors,
  e.g. a :class:`~blendtorch.btt.gpu.DeviceLoader` with
  ``DecodeConfig.raw()`` output, or host arrays.
* ``sample(B, decode)`` / ``batches(B, decode)``: draw random (or shuffled)
  indices on the device and decode them with ONE fused gather+decode kernel
  (``ops.decode_gather``: the kernel reads frame ``index[b]`` straight from the
  store; the gathered u8 batch is never materialised). Per-item metadata
  (``btid``, ``frameid``, ``xy``, ...) is gathered on the device too.

On a CPU device the same API runs with the fp32 reference ops (tests, hosts
without a GPU). On a GPU device the HIP kernels are required and fail loudly
if the extension is missing.
"""
from __future__ import annotations

import mmap
from glob import glob
from typing import Dict, Iterator, Optional

import numpy as np
import torch

from .. import ops
from ..ops import DecodeConfig

__all__ = ['DeviceReplayBuffer']


def _as_tensor(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device)
    return torch.as_tensor(np.asarray(x), device=device)


class DeviceReplayBuffer:
    """Ring buffer of raw u8 ``H x W x C`` frames (+ numeric metadata) on one device.

    Params
    ------
    capacity: int
        Frames held; the store is ``capacity x H x W x C`` bytes, allocated
        on the first ``extend`` (when the frame shape is known).
    device: torch.device / str
        Where frames live (``'cuda:N'`` for HBM, ``'cpu'`` for the reference path).
    image_key: str
        Message key of the image when filling from recordings / loaders.
    """

    def __init__(self, capacity: int, device=None, image_key: str = 'image', seed: Optional[int] = None):
        if capacity < 1:
            raise ValueError('capacity must be >= 1')
        self.capacity = int(capacity)
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.image_key = image_key
        self.store: Optional[torch.Tensor] = None     # [capacity, H, W, C] u8
        self.meta: Dict[str, torch.Tensor] = {}
        self._size = 0
        self._next = 0
        # sampler state of the fused kernel: Philox key and counter (host-side
        # for eager sampling: one launch per batch; graphed samplers keep a
        # device counter the captured graph advances itself)
        self.seed = int(torch.initial_seed() if seed is None else seed) & (2 ** 64 - 1)
        self._ctr = 0
        if self.device.type == 'cuda':
            ops.hip_ext()   # fail loudly here, not at the first sample()

    # -- filling ---------------------------------------------------------------
    def __len__(self):
        return self._size

    @property
    def frame_shape(self):
        return None if self.store is None else tuple(self.store.shape[1:])

    @property
    def nbytes(self):
        return 0 if self.store is None else self.store.numel()

    def _alloc(self, shape, meta):
        self.store = torch.empty((self.capacity,) + tuple(shape), dtype=torch.uint8, device=self.device)
        for k, v in meta.items():
            v = _as_tensor(v, self.device)
            self.meta[k] = torch.zeros((self.capacity,) + tuple(v.shape[1:]), dtype=v.dtype, device=self.device)

    def extend(self, images, **meta):
        """Append ``n`` frames (u8 ``[n,H,W,C]`` or ``[n,H,W]``; tensor or ndarray)
        and per-frame metadata arrays of leading length ``n``."""
        imgs = images if isinstance(images, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(images))
        if imgs.dtype != torch.uint8:
            raise TypeError('frames must be uint8')
        if imgs.dim() == 3:
            imgs = imgs.unsqueeze(-1)
        n = int(imgs.shape[0])
        meta = {k: v for k, v in meta.items() if v is not None}
        if self.store is None:
            self._alloc(imgs.shape[1:], {k: v[:1] if len(v) else v for k, v in meta.items()})
        if tuple(imgs.shape[1:]) != self.frame_shape:
            raise ValueError(f'frame shape {tuple(imgs.shape[1:])} != store {self.frame_shape}')
        if set(meta) != set(self.meta):
            raise ValueError(f'metadata keys {sorted(meta)} != {sorted(self.meta)}')
        if n > self.capacity:   # only the newest `capacity` frames survive
            imgs = imgs[n - self.capacity:]
            meta = {k: v[n - self.capacity:] for k, v in meta.items()}
            n = self.capacity
        pos = 0
        while pos < n:
            k = min(n - pos, self.capacity - self._next)
            self.store[self._next:self._next + k].copy_(imgs[pos:pos + k], non_blocking=True)
            for key, v in meta.items():
                self.meta[key][self._next:self._next + k].copy_(_as_tensor(v[pos:pos + k], self.device))
            self._next = (self._next + k) % self.capacity
            pos += k
        self._size = min(self.capacity, self._size + n)
        return self

    def fill_from(self, batches, max_items: int):
        """Append frames from an iterable of batch dicts (e.g. a
        ``DeviceLoader(..., decode=DecodeConfig.raw())``) until ``max_items``."""
        got = 0
        for b in batches:
            img = b[self.image_key]
            take = min(len(img), max_items - got)
            meta = {k: v[:take] for k, v in b.items()
                    if k != self.image_key and isinstance(v, (torch.Tensor, np.ndarray))}
            self.extend(img[:take], **meta)
            got += take
            if got >= max_items:
                break
        return self

    @classmethod
    def from_recordings(cls, record_path_prefix: str, device=None, capacity: Optional[int] = None,
                        image_key: str = 'image', meta_keys=('btid', 'frameid'), chunk: int = 64):
        """Load every ``{prefix}_*.btr`` recording (FileRecorder format) into a
        new buffer.  Images are located in the memory-mapped files by the
        native codec (no unpickling of pixel data) and uploaded ``chunk``
        frames at a time through pinned memory."""
        from .file import FileReader
        from .. import _native
        fnames = sorted(glob(f'{record_path_prefix}_*.btr'))
        assert fnames, f'Found no recording files with prefix {record_path_prefix}'
        spans = []
        for f in fnames:
            offs = FileReader.read_offsets(f)
            spans.append((f, offs))
        total = sum(len(o) for _, o in spans)
        buf = cls(capacity or max(1, total), device=device, image_key=image_key)
        pin = None
        stage_imgs, stage_meta = [], {k: [] for k in meta_keys}

        def flush():
            nonlocal pin
            if not stage_imgs:
                return
            arr = np.stack(stage_imgs)
            t = torch.from_numpy(arr)
            if buf.device.type == 'cuda':
                if pin is None or pin.shape[1:] != t.shape[1:] or pin.shape[0] < len(t):
                    pin = torch.empty((chunk,) + tuple(t.shape[1:]), dtype=torch.uint8).pin_memory()
                pin[:len(t)].copy_(t)
                t = pin[:len(t)]
            buf.extend(t, **{k: np.asarray(v) for k, v in stage_meta.items() if v})
            if buf.device.type == 'cuda':
                torch.cuda.current_stream(buf.device).synchronize()   # `pin` is reused
            stage_imgs.clear()
            for v in stage_meta.values():
                v.clear()

        for fname, offs in spans:
            with open(fname, 'rb') as fp, mmap.mmap(fp.fileno(), 0, access=mmap.ACCESS_READ) as mm:
                view = memoryview(mm)
                ends = list(offs[1:]) + [len(mm)]
                for o, e in zip(offs, ends):
                    msg = view[int(o):int(e)]
                    try:
                        item = _native.fast_loads(msg)
                    except ValueError:   # outside the codec's fast path
                        import pickle
                        item = pickle.loads(msg)
                    img = np.asarray(item[image_key])
                    stage_imgs.append(np.array(img, dtype=np.uint8, copy=True))
                    for k in meta_keys:
                        if k in item:
                            stage_meta[k].append(item[k])
                    del item, img, msg
                    if len(stage_imgs) == chunk:
                        flush()
                flush()
                view.release()
        return buf

    def save_recordings(self, record_path_prefix: str, files: int = 1, chunk: int = 64):
        """Write the stored frames (oldest first) as ``.btr`` recordings,
        ``{prefix}_{i:02d}.btr`` for i < ``files``: one message per frame,
        ``{image_key: u8 HxWxC, **metadata}``. The files are the format
        ``FileRecorder`` writes, so ``FileDataset`` (CPU) and
        :meth:`from_recordings` (GPU) read them back. This is how a stream
        consumed on the GPU path gets recorded."""
        from .file import FileRecorder
        n = self._size
        start = self._next if n == self.capacity else 0   # ring order: oldest first
        order = [(start + i) % self.capacity for i in range(n)]
        per = [order[i::files] for i in range(files)]
        paths = []
        for fi, idxs in enumerate(per):
            path = FileRecorder.filename(record_path_prefix, fi)
            with FileRecorder(path, max_messages=max(1, len(idxs))) as rec:
                for s in range(0, len(idxs), chunk):
                    sel = torch.as_tensor(idxs[s:s + chunk], dtype=torch.int64, device=self.device)
                    imgs = self.store.index_select(0, sel).cpu().numpy()
                    meta = {k: v.index_select(0, sel).cpu().numpy() for k, v in self.meta.items()}
                    for j in range(len(imgs)):
                        item = {self.image_key: imgs[j]}
                        for k, v in meta.items():
                            item[k] = v[j].item() if v[j].ndim == 0 else v[j]
                        rec.save(item, is_pickled=False)
            paths.append(path)
        return paths

    # -- sampling --------------------------------------------------------------
    def _fused(self, decode: DecodeConfig):
        return self.device.type == 'cuda' and not decode.colour_kernel and self.store.is_contiguous()

    def _decode(self, idx: torch.Tensor, decode: DecodeConfig):
        if self.device.type == 'cuda' and not decode.colour_kernel:
            return ops.decode_gather(self.store, idx, decode)
        imgs = self.store.index_select(0, idx)
        if self.device.type == 'cuda':
            return ops.decode(imgs, decode)
        return ops.reference_decode(imgs, decode)

    def gather(self, idx: torch.Tensor, decode: DecodeConfig = DecodeConfig()):
        """Decoded frames ``idx`` (device int tensor) + their metadata.  On a
        GPU: one fused launch decodes the frames and gathers every metadata
        column (``ops.replay_sample`` with given indices)."""
        if self._size == 0:
            raise IndexError('empty replay buffer')
        idx = idx.to(self.device, torch.int64)
        if self._fused(decode):
            img, idx, meta = ops.replay_sample(self.store, self._size, int(idx.numel()), decode, index=idx,
                                               meta=self.meta)
            return {self.image_key: img, **meta, 'index': idx}
        out = {self.image_key: self._decode(idx, decode)}
        for k, v in self.meta.items():
            out[k] = v.index_select(0, idx)
        out['index'] = idx
        return out

    def sample(self, batch_size: int, decode: DecodeConfig = DecodeConfig(), generator=None, _counter=None):
        """Uniform random batch (with replacement).  On a GPU (no ``generator``)
        ONE fused launch draws the indices (Philox), decodes the frames and
        gathers their metadata; with a ``torch.Generator`` the indices come
        from ``torch.randint`` instead."""
        if self._size == 0:
            raise IndexError('empty replay buffer')
        if generator is None and self._fused(decode):
            ctr = _counter
            if ctr is None:
                ctr, self._ctr = self._ctr, self._ctr + batch_size
            img, idx, meta = ops.replay_sample(self.store, self._size, batch_size, decode, seed=self.seed,
                                               counter=ctr, meta=self.meta)
            return {self.image_key: img, **meta, 'index': idx}
        idx = torch.randint(0, self._size, (batch_size,), device=self.device, generator=generator)
        return self.gather(idx, decode)

    def graphed_sampler(self, batch_size: int, decode: DecodeConfig = DecodeConfig(), warmup: int = 3):
        """``sample(batch_size, decode)`` captured once as a HIP graph.

        A batch-8 sample is a handful of small launches (index draw, offset
        scale, the fused gather+decode, one gather per metadata key), so its
        cost is launch overhead. Replaying the captured graph issues all of
        them at once. The returned callable replays the graph and returns the
        same static output dict every time: consume (or clone) a batch before
        the next call. The number of stored frames is frozen into the graph,
        so capture again after ``extend``.
        """
        if self.device.type != 'cuda':
            return lambda: self.sample(batch_size, decode)
        # the captured sample reads its Philox counter from device memory and
        # advances it there: every replay draws new indices
        counter = torch.tensor([self._ctr], dtype=torch.int64, device=self.device)
        self._ctr += 1 << 40          # disjoint from later eager draws
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):   # allocations, LUT upload, kernel selection outside the capture
                self.sample(batch_size, decode, _counter=counter)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self.sample(batch_size, decode, _counter=counter)

        def replay():
            graph.replay()
            return out
        replay.graph = graph
        return replay

    def batches(self, batch_size: int, decode: DecodeConfig = DecodeConfig(), shuffle: bool = True,
                drop_last: bool = True, epochs: int = 1, generator=None) -> Iterator[dict]:
        """Epochs over the stored frames (a device-side permutation each epoch)."""
        for _ in range(epochs):
            order = (torch.randperm(self._size, device=self.device, generator=generator) if shuffle
                     else torch.arange(self._size, device=self.device))
            stop = self._size - (self._size % batch_size if drop_last else 0)
            for s in range(0, stop, batch_size):
                yield self.gather(order[s:s + batch_size], decode)
