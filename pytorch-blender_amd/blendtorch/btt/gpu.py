"""Device-resident streaming: producer frames -> decoded batches in HBM.

:class:`DeviceLoader` is the MI355X-native counterpart of
``DataLoader(RemoteIterableDataset(...), batch_size=B, num_workers=W)``
(reference: pkg_pytorch/blendtorch/btt/dataset.py:14-117 and
benchmarks/benchmark.py:24-41).  Instead of W forked worker processes that
unpickle each frame, run numpy transforms, ``default_collate`` the batch and
ship it through shared memory, one native pipeline per GPU rank
(``csrc/gpu/loader.cpp``) takes frames from the producers' pinned
shared-memory ring (or receives them into pinned slots) and runs the fused
gfx950 decode kernel, which reads them over PCIe itself, into a tensor the
consumer's stream waits on.  Nothing round-trips through pageable memory.

Semantics kept from the reference:

* PULL sockets connect to every address; fair-queued fan-in with RCVHWM
  backpressure; each message goes to exactly one consumer.
* ``max_items`` bounds the stream (``stream_length``); silence longer than
  ``timeoutms`` raises (``dataset.py:98-99``).
* Every non-image key of the producer dict is collated like
  ``default_collate`` would (ints -> int64 tensor, ndarrays stacked, ...).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Optional, Sequence

import numpy as np
import torch
from torch.utils.data import default_collate

from .. import ops
from ..ops import DecodeConfig
from ..utils import trace_range
from .constants import DEFAULT_TIMEOUTMS

logger = logging.getLogger('blendtorch')

__all__ = ['DeviceLoader', 'DecodeConfig']


def _default_io_threads(addresses) -> int:
    n = len(addresses)
    if not any(str(a).startswith('tcp://') for a in addresses):
        return max(1, min(4, n))
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 4
    return max(1, min(n, max(4, cpus - 2)))


class DeviceLoader:
    """Iterate decoded batches of producer frames resident on a GPU.

    Params
    ------
    addresses: list of str
        Producer PUSH addresses (``launch_info.addresses['DATA']``).
    batch_size: int
        Items per batch (B).
    decode: DecodeConfig
        What the decode kernel does (channels, gamma, normalisation, dtype,
        layout, flip, optional colour matrix).
    device: torch.device / int / str
        Target GPU (default: current device).
    max_items: int, optional
        Total items to deliver; the stream ends after ``max_items // B``
        batches.  None streams forever.
    timeoutms: int
        Max wait for the next batch before ``TimeoutError``.
    prefetch: int
        Output batches the native pipeline may run ahead of the consumer.
    io_threads: int, optional
        Receive IO threads (default: one per address, at most 4 for ipc://
        addresses -- shared-memory descriptors and local frames -- and up to
        the process's usable CPUs minus two for tcp:// ones, whose inline
        frames each thread copies out of its sockets).
    image_key: str
        Dict key holding the u8 HxWxC image.
    skip_bad: bool
        Drop malformed messages instead of failing the stream.
    meta_to_device: bool
        Move collated metadata tensors to the device as well.
    h2d: str
        ``'auto'`` (default): when a batch's frames all sit in device-visible
        pinned host memory (the producers' shared-memory ring, or the
        loader's pinned receive slots) the decode kernel reads them over PCIe
        itself -- one fused pass, no staging copy; otherwise the frames are
        DMA'd into a device staging ring first.  ``'copy'``: always DMA.
    launch_depth: int
        Direct-path decode launches the loader keeps queued on its stream.
        Batches completing while that many are in flight wait and go out
        together in one launch (fewer kernel ramp-up/tail phases when the GPU
        side is the bottleneck).  0: hold batches until 64 images are pending
        or the stream ends (tests / maximal coalescing).
    copy_streams: int
        Copy path (``h2d='copy'`` or frames that are not device-visible): the
        frames of a batch are spread over this many HIP streams so several
        DMA engines pull from host memory concurrently (1: one stream).
    log_every: float, optional
        Log :meth:`metrics` on the ``'blendtorch'`` logger every that many
        seconds while iterating.
    host_sync: bool, optional
        (default: True.)
        Order the loader against the consumer on the host (event queries)
        rather than with cross-stream waits: a posted buffer is written once
        its post event has completed, and a batch is handed out once its
        copies/kernel have completed -- the consumer's stream never waits on
        the loader's.  ROCm's hipStreamWaitEvent costs 28-430 us of host time
        per call (profiles/r2/hip_api_cost.json), and a stream of
        cross-stream waits keeps a HIP runtime thread busy for a whole core
        (profiles/r4/cpu_per_frame.md: 23 of the consumer's 43 CPU-us per
        frame); False restores the GPU-side waits.
    defer_post: bool
        Hand the loader a fresh output buffer only when the consumer calls
        :meth:`release` (or, failing that, when it asks for the next batch)
        instead of before each batch is yielded.  The buffer's copies are
        gated on the consumer stream at that point, so a training step can
        place the next frames' DMA behind its forward pass, onto the
        compute-bound backward kernels (bench.py --dma-phase mid: DMA that
        overlaps the memory-bound forward slows it by ~20%).
    """

    def __init__(self, addresses: Sequence[str], batch_size: int = 8, decode: DecodeConfig = DecodeConfig(),
                 device=None, max_items: Optional[int] = None, timeoutms: int = DEFAULT_TIMEOUTMS,
                 rcvhwm: int = 10, prefetch: int = 4, io_threads: Optional[int] = None, image_key: str = 'image',
                 skip_bad: bool = False, meta_to_device: bool = False, staging_depth: int = 3, h2d: str = 'auto',
                 launch_depth: int = 2, log_every: Optional[float] = None, copy_streams: int = 2,
                 defer_post: bool = False, host_sync: Optional[bool] = None, reuse_buffers: bool = False):
        if h2d not in ('auto', 'copy'):
            raise ValueError("h2d must be 'auto' or 'copy'")
        self.h2d = h2d
        self.launch_depth = int(launch_depth)
        self.copy_streams = max(1, min(4, int(copy_streams)))
        if isinstance(addresses, str):
            addresses = [addresses]
        self.addresses = list(addresses)
        self.batch_size = int(batch_size)
        self.decode = decode
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device())
        self.device = torch.device(device) if not isinstance(device, int) else torch.device('cuda', device)
        if self.device.index is None:
            self.device = torch.device('cuda', torch.cuda.current_device())
        self.max_items = max_items
        self.timeoutms = timeoutms
        self.rcvhwm = rcvhwm
        self.prefetch = max(1, int(prefetch))
        # one receive thread per producer up to 4: a thread copying inline
        # 1.2 MB frames out of sockets tops out near 7-9k frames/s
        # (profiles/reference_harness.md), shm descriptors cost it little;
        # over TCP (remote producers, inline frames) every pipe gets its own
        # thread, up to the CPUs this process may use minus the worker and
        # the consumer
        self.io_threads = io_threads or _default_io_threads(self.addresses)
        self.image_key = image_key
        self.skip_bad = skip_bad
        self.meta_to_device = meta_to_device
        self.staging_depth = staging_depth
        self._loader = None
        self._live = None          # native pipeline while iterating
        self.shape = None          # (H, W, C) of incoming frames
        self.stats = {}
        self.log_every = log_every
        self._t_start = self._t_end = None
        self._wait_s = 0.0
        self.defer_post = bool(defer_post)
        # default: host ordering on both paths.  (Round 2 measured the direct
        # path 42.0k vs 38.7k img/s with GPU-side waits; with 8 posted buffers
        # the two are level, 42.1-42.3k, and host ordering halves the
        # consumer process's CPU per frame: profiles/r4/cpu_per_frame.md)
        self.host_sync = True if host_sync is None else bool(host_sync)
        self._owed = 0             # deferred posts not yet made
        self._post_fn = None
        # reuse_buffers: output tensors come from a fixed ring of prefetch + 2,
        # so a consumer that captures one graph per input tensor
        # (parallel.step.CapturedStep static_inputs) reads them in place.  The
        # tensor of batch j is posted again when batch j + 2 is handed out (its
        # refill is ordered behind the consumer's stream work on it): a
        # consumer may keep the previous batch, never the one before that.
        # The ring is rebuilt at every __iter__ and whenever the output shape
        # or dtype changes (another frame size), so no differently sized
        # tensor is ever posted to the native decode
        self.reuse_buffers = bool(reuse_buffers)
        self._ring = []
        self._ring_i = 0

    @classmethod
    def from_config(cls, addresses: Sequence[str], config, decode: DecodeConfig = DecodeConfig(), device=None,
                    max_items: Optional[int] = None) -> 'DeviceLoader':
        """Build from a :class:`blendtorch.utils.StreamConfig`."""
        return cls(addresses, decode=decode, device=device, max_items=max_items, **config.kwargs())

    def __len__(self):
        if self.max_items is None:
            raise TypeError('infinite stream has no length')
        return self.max_items // self.batch_size

    def stream_length(self, max_items):
        self.max_items = max_items
        return self

    # -- native pipeline -----------------------------------------------------
    def _make(self):
        ext = ops.hip_ext()
        cfg = self.decode
        lut = ops.build_table(cfg).tolist()
        matrix = [] if cfg.color_matrix is None else np.asarray(cfg.color_matrix, np.float32).reshape(-1).tolist()
        bias = [] if cfg.color_matrix is None else list(cfg.color_bias or (0.0, 0.0, 0.0, 0.0))
        # per-image colour transforms on the same MFMA kernel: one per batch position,
        # or random jitter drawn per image in the loader (factors in batch['color_jitter'])
        matrices, jitter, seed = [], [], 0
        if cfg.color_matrices is not None:
            if len(cfg.color_matrices) != self.batch_size:
                raise ValueError(f'DecodeConfig.color_matrices holds {len(cfg.color_matrices)} transforms for '
                                 f'batch_size {self.batch_size}')
            m = np.asarray(cfg.color_matrices, np.float32).reshape(self.batch_size, 16)
            matrices = np.concatenate([m, np.asarray(cfg.color_biases, np.float32)], axis=1).reshape(-1).tolist()
        if cfg.color_jitter is not None:
            j = cfg.color_jitter
            jitter = [j.brightness, j.contrast, j.saturation, j.hue, cfg.jitter_pivot]
            seed = int(j.seed) & ((1 << 64) - 1)
        max_batches = -1 if self.max_items is None else self.max_items // self.batch_size
        return ext.StreamLoader(
            self.addresses, self.batch_size, self.image_key, self.rcvhwm, self.io_threads, self.device.index,
            max_batches, 0, 0, self.staging_depth, self.skip_bad, cfg.cout, list(cfg.cmap) + [0] * (4 - len(cfg.cmap)),
            int(cfg.flip), ops.OUT_DTYPES[cfg.dtype], ops.LAYOUTS[cfg.layout], lut, matrix, bias,
            self.h2d == 'auto', self.launch_depth, self.copy_streams, self.host_sync, matrices, jitter, seed)

    def _post(self, loader, stream):
        shape = self.decode.out_shape(self.batch_size, *self.shape[:2])
        if self.reuse_buffers:
            dt = self.decode.torch_dtype()
            if self._ring and (tuple(self._ring[0].shape) != tuple(shape) or self._ring[0].dtype != dt
                               or self._ring[0].device != self.device):
                self._ring, self._ring_i = [], 0
            if len(self._ring) < self.prefetch + 2:
                self._ring.append(torch.empty(shape, dtype=self.decode.torch_dtype(), device=self.device))
                out = self._ring[-1]
            else:
                out = self._ring[self._ring_i % len(self._ring)]
                self._ring_i += 1
            loader.post(out.data_ptr(), stream.cuda_stream)
            return out
        out = torch.empty(shape, dtype=self.decode.torch_dtype(), device=self.device)
        loader.post(out.data_ptr(), stream.cuda_stream)
        return out

    def _collate_meta(self, meta):
        """Natively collated metadata (key -> ndarray, or per-item list for
        values that do not stack) -> what ``default_collate`` would give."""
        out = {}
        for k, v in meta.items():
            if isinstance(v, np.ndarray):
                v = torch.from_numpy(v)
            else:
                try:
                    v = default_collate(v)
                except (TypeError, RuntimeError):
                    pass
            if self.meta_to_device and isinstance(v, torch.Tensor):
                v = v.to(self.device, non_blocking=True)
            out[k] = v
        return out

    def metrics(self) -> dict:
        """Pipeline counters: live while iterating, final afterwards.

        ``frames_per_s`` / ``h2d_gbytes_per_s``: delivered frames and the image
        bytes they moved host -> device, over the time since the first frame;
        ``frames_per_producer``: frames per producer ``btid`` (provenance, as
        the reference's messages carry it); ``gpu_us_per_image``: device time
        (H2D copies + decode kernel) per image, sampled every 16th launch with
        timing events; ``images_per_launch``: launch coalescing;
        ``consumer_wait_s``: time the consumer spent blocked on the next batch.
        """
        s = self._live.stats() if self._live is not None else dict(self.stats)
        if not s or self._t_start is None:
            return {}
        elapsed = max(1e-9, (self._t_end or time.perf_counter()) - self._t_start)
        per = {int(k): int(v) for k, v in s.get('frames_per_btid', {}).items()}
        timed = s.get('timed_images', 0)
        return {
            'elapsed_s': elapsed,
            'frames': s['frames'],
            'batches': s['batches'],
            'frames_per_s': s['frames'] / elapsed,
            'h2d_gbytes_per_s': s.get('image_bytes', 0) / elapsed / 1e9,
            'frames_per_producer': per,
            'producer_frames_per_s': {k: v / elapsed for k, v in per.items()},
            'gpu_us_per_image': s['timed_gpu_ms'] * 1e3 / timed if timed else None,
            'launches': s['launches'],
            'images_per_launch': s['frames'] / s['launches'] if s['launches'] else None,
            'direct_batches': s['direct_batches'],
            'staged_frames': s.get('staged_frames', 0),
            'consumer_wait_s': self._wait_s,
            'bad': s['bad'], 'shm_stale': s['shm_stale'], 'shm_torn': s['shm_torn'],
            'pool_fallbacks': s['pool_fallbacks'],
        }

    def release(self):
        """``defer_post=True``: give the loader the output buffers owed for
        the batches delivered so far, gating their copies on the current
        stream position (call it where the next frames' DMA should start)."""
        if self._post_fn is not None:
            self._post_fn()

    def snapshot(self) -> dict:
        """Raw cumulative pipeline counters at this instant (plus the wall
        clock and the consumer's accumulated wait).  Two snapshots bracket a
        timed region; :meth:`window` turns them into rates for that region
        only -- unlike :meth:`metrics`, which spans the whole run including
        start-up and warm-up (reference timing: benchmarks/benchmark.py:33-47
        excludes the first batch the same way)."""
        s = self._live.stats() if self._live is not None else dict(self.stats)
        s = dict(s)
        s['t'] = time.perf_counter()
        s['consumer_wait_s'] = self._wait_s
        return s

    @staticmethod
    def window(s0: dict, s1: dict) -> dict:
        """Rates between two :meth:`snapshot` results (the timed window)."""
        if not s0 or not s1 or 'frames' not in s0 or 'frames' not in s1:
            return {}
        dt = max(1e-9, s1['t'] - s0['t'])
        d = {k: s1.get(k, 0) - s0.get(k, 0) for k in ('frames', 'batches', 'launches', 'image_bytes', 'timed_images',
                                                      'timed_gpu_ms', 'shm_stale', 'shm_torn', 'bad')}
        p0 = {int(k): int(v) for k, v in s0.get('frames_per_btid', {}).items()}
        p1 = {int(k): int(v) for k, v in s1.get('frames_per_btid', {}).items()}
        cnt = {k: v - p0.get(k, 0) for k, v in sorted(p1.items())}
        per = {k: round(c / dt, 1) for k, c in cnt.items()}
        # fair fan-in check (reference: every consumer interleaves all producers
        # fairly, examples/datagen/Readme.md:177): max/min of the producers'
        # frame counts in the window; None when a known producer sent nothing
        lo = min(cnt.values()) if cnt else 0
        out = {
            'window_s': dt,
            'frames': d['frames'],
            'frames_per_s': d['frames'] / dt,
            'h2d_gbytes_per_s': d['image_bytes'] / dt / 1e9,
            'gpu_us_per_image': d['timed_gpu_ms'] * 1e3 / d['timed_images'] if d['timed_images'] else None,
            'timed_images': d['timed_images'],
            'images_per_launch': d['frames'] / d['launches'] if d['launches'] else None,
            'producer_frames_per_s': per,
            'producer_frames': cnt,
            'producer_share_max_over_min': (round(max(cnt.values()) / lo, 4) if lo > 0 else None),
            'producers_starved': sum(1 for c in cnt.values() if c == 0),
            'consumer_wait_ms_per_batch': ((s1['consumer_wait_s'] - s0['consumer_wait_s']) * 1e3 / d['batches']
                                           if d['batches'] else None),
            'shm_stale': d['shm_stale'], 'shm_torn': d['shm_torn'], 'bad': d['bad'],
        }
        # producer ring occupancy (frames rendered and not yet handed back) at both ends:
        # a window that starts on a full ring and ends on an empty one measured a drain
        for tag, s in (('t0', s0), ('t1', s1)):
            if 'ring_slots' in s:
                out[f'ring_{tag}'] = {'published': s.get('ring_published', 0), 'held': s.get('ring_held', 0),
                                      'slots': s['ring_slots']}
        # a window no longer than the frames already rendered at its start could
        # have been served from that backlog alone: it proves the loader's rate,
        # not the producers' sustained rate
        if 'ring_t0' in out:
            out['backlog_covers_window'] = out['ring_t0']['published'] >= d['frames']
        return out

    def _log_metrics(self):
        m = self.metrics()
        if m:
            logger.info('DeviceLoader: %.0f frames/s, %.1f GB/s H2D, %s us/image on the GPU, %.2f images/launch, '
                        'consumer wait %.2fs, producers %s', m['frames_per_s'], m['h2d_gbytes_per_s'],
                        'n/a' if m['gpu_us_per_image'] is None else '%.1f' % m['gpu_us_per_image'],
                        m['images_per_launch'] or 0.0, m['consumer_wait_s'], m['frames_per_producer'])

    def __iter__(self):
        loader = self._make()
        loader.start()
        self._live = loader
        self._ring, self._ring_i = [], 0     # a new stream: a fresh output ring
        self._t_start = self._t_end = None
        self._wait_s = 0.0
        try:
            with torch.cuda.device(self.device):
                stream = torch.cuda.current_stream(self.device)
                shape = None
                t0 = time.time()
                while shape is None:
                    shape = loader.wait_shape(200)
                    if shape is None and (time.time() - t0) * 1000 > self.timeoutms:
                        raise TimeoutError('No response within timeout interval.')
                self.shape = tuple(shape)
                self._t_start = time.perf_counter()
                last_log = self._t_start
                n_batches = None if self.max_items is None else self.max_items // self.batch_size
                pending = [self._post(loader, stream) for _ in range(self.prefetch if n_batches is None
                                                                        else min(self.prefetch, n_batches))]
                posted = len(pending)
                delivered = 0

                def post_owed():
                    while self._owed:
                        self._owed -= 1
                        pending.append(self._post(loader, stream))
                self._post_fn = post_owed
                while n_batches is None or delivered < n_batches:
                    post_owed()            # the consumer did not release() them itself
                    t0 = time.time()
                    tw = time.perf_counter()
                    r = None
                    while r is None:
                        with trace_range('btt.DeviceLoader.next'):
                            r = loader.next_collated(stream.cuda_stream, 200)
                        if r is None and (time.time() - t0) * 1000 > self.timeoutms:
                            raise TimeoutError('No response within timeout interval.')
                    self._wait_s += time.perf_counter() - tw
                    if self.log_every is not None and tw - last_log >= self.log_every:
                        last_log = tw
                        self._log_metrics()
                    idx, metas, _ = r
                    if idx < 0:
                        break
                    out = pending.pop(0)
                    if n_batches is None or posted < n_batches:
                        if self.defer_post:
                            self._owed += 1
                        else:
                            pending.append(self._post(loader, stream))
                        posted += 1
                    batch = {self.image_key: out}
                    batch.update(self._collate_meta(metas))
                    delivered += 1
                    yield batch
        finally:
            self._post_fn = None
            self._owed = 0
            self.stats = loader.stats()
            self._t_end = time.perf_counter()
            self._live = None
            loader.stop()
