"""Observability and configuration helpers.

The reference's only instrumentation is wall-clock timing in
benchmarks/benchmark.py:33-47 and the ``'blendtorch'`` logger (SURVEY.md
§5.1, §5.5).  Added here:

* :class:`Meter` -- rate/latency counters (items/s, ms per stage) that can be
  dumped as a dict or logged;
* :func:`trace_range` -- a roctx range (visible in ``rocprofv3
  --marker-trace`` timelines) around host-side stages with ``BLENDTORCH_ROCTX=1``;
* :class:`StreamConfig` -- one place for the GPU streaming knobs whose
  defaults reproduce the reference's behaviour (HWM 10, 10 s timeout, batch
  of dicts);
* :func:`ensure_hw_queues` -- enough HIP hardware queues per process for
  the loader's streams, the compute stream and RCCL's.
"""
from __future__ import annotations

import contextlib
import dataclasses
import logging
import os
import time
from typing import Dict, Optional

logger = logging.getLogger('blendtorch')

__all__ = ['Meter', 'trace_range', 'StreamConfig', 'get_logger', 'ensure_hw_queues']

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues per process (4 by
# default) round-robin.  A rank's loader uses 2-3 streams (decode, copies),
# the consumer one, and an RCCL communicator adds its own: with 4 queues the
# loader's streams then share queues with RCCL's and serialise behind them.
# Measured on one MI355X (profiles/r4/pg_tax.md): a live 1-rank RCCL process
# group cost streaming 3.6 % (shard) / 5.3 % (scatter) at 4 queues and 0.0 % /
# 0.7 % at 8 -- but the graphed training step with its in-graph RCCL
# all-reduce ran 27 % SLOWER at 8 queues (0.6 % tax at 4), so training
# consumers keep 4 (bench.py picks per run).
DEFAULT_HW_QUEUES = 8


def ensure_hw_queues(n: int = DEFAULT_HW_QUEUES, exact: bool = False) -> int:
    """Set ``GPU_MAX_HW_QUEUES`` for this process (and the processes it
    starts) unless ``BT_HW_QUEUES`` pins a value (1..32, the runtime refuses
    more).  ``exact=False`` raises an inherited count to at least ``n``;
    ``exact=True`` sets exactly ``n`` -- for a graphed training step, which an
    inherited 8 slows by 27 % (the warning names the override).  Only
    effective before the HIP runtime initialises (the first GPU call), so
    call it at program start.  Returns the value in force."""
    pinned = os.environ.get('BT_HW_QUEUES')
    if pinned:
        try:
            v = int(pinned)
        except ValueError:
            raise ValueError(f'BT_HW_QUEUES={pinned!r}: expected an integer 1..32') from None
        if not 1 <= v <= 32:
            raise ValueError(f'BT_HW_QUEUES={v}: the HIP runtime accepts 1..32 hardware queues')
        os.environ['GPU_MAX_HW_QUEUES'] = str(v)
        return v
    n = max(1, min(32, int(n)))
    raw = os.environ.get('GPU_MAX_HW_QUEUES')
    try:
        cur = int(raw) if raw else 4     # unset: HIP's default, 4
    except ValueError:
        cur = 4
    if exact and raw and cur != n:
        logger.warning('GPU_MAX_HW_QUEUES=%s inherited; this process uses %d (BT_HW_QUEUES pins a value)', raw, n)
    if cur < n or (exact and cur != n):
        os.environ['GPU_MAX_HW_QUEUES'] = str(n)
        return n
    return cur


def get_logger():
    return logger


class Meter:
    """Accumulates counts and durations per named stage.

    >>> m = Meter()
    >>> with m.time('recv'):
    ...     pass
    >>> m.count('frames', 8)
    >>> sorted(m.summary())  # doctest: +ELLIPSIS
    ['elapsed_s', 'frames', 'frames_per_s', 'recv_ms', 'recv_ms_avg']
    """

    def __init__(self):
        self.t0 = time.perf_counter()
        self.counts: Dict[str, float] = {}
        self.ms: Dict[str, float] = {}
        self.calls: Dict[str, int] = {}

    def count(self, name, n=1):
        self.counts[name] = self.counts.get(name, 0) + n

    @contextlib.contextmanager
    def time(self, name):
        t = time.perf_counter()
        try:
            yield
        finally:
            self.ms[name] = self.ms.get(name, 0.0) + (time.perf_counter() - t) * 1e3
            self.calls[name] = self.calls.get(name, 0) + 1

    def summary(self) -> Dict[str, float]:
        el = max(time.perf_counter() - self.t0, 1e-9)
        out = {'elapsed_s': el}
        for k, v in self.counts.items():
            out[k] = v
            out[f'{k}_per_s'] = v / el
        for k, v in self.ms.items():
            out[f'{k}_ms'] = v
            out[f'{k}_ms_avg'] = v / max(1, self.calls[k])
        return out

    def log(self, level=logging.INFO):
        logger.log(level, ' '.join(f'{k}={v:.4g}' for k, v in self.summary().items()))


class _RoctxRange:
    __slots__ = ('name',)

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        import torch
        torch.cuda.nvtx.range_push(self.name)

    def __exit__(self, *exc):
        import torch
        torch.cuda.nvtx.range_pop()
        return False


_NO_RANGE = contextlib.nullcontext()
_roctx_on = None


def trace_range(name: str):
    """roctx range around a host-side stage (ROCm maps torch's nvtx API to
    roctx) when ``BLENDTORCH_ROCTX=1`` (as the native ranges) and a GPU is present; otherwise one shared
    no-op context (the per-batch loops call this: ~0.1 us instead of the
    ~6 us a generator-based context manager plus the roctx calls cost)."""
    global _roctx_on
    if _roctx_on is None:
        try:
            import torch
            _roctx_on = os.environ.get('BLENDTORCH_ROCTX') == '1' and torch.cuda.is_available()
        except Exception:
            _roctx_on = False
    return _RoctxRange(name) if _roctx_on else _NO_RANGE


@dataclasses.dataclass
class StreamConfig:
    """Knobs of the device streaming path in one place (defaults = reference
    behaviour where the reference has the knob).

    Pass it as ``DeviceLoader.from_config(addresses, cfg, decode=...)``;
    every field maps onto the :class:`~blendtorch.btt.DeviceLoader` argument
    of the same name.

    batch_size: items per batch; rcvhwm: receive queue per producer (the
    reference's ``queue_size``, 10); timeoutms: max silence before failing
    (10 s, ``btt/constants.py``); prefetch: output batches the native
    pipeline may run ahead; io_threads: receive IO threads (None: one per
    producer, at most 4); staging_depth: device staging buffers of the copy
    path; h2d: 'auto' (zero-copy reads of pinned frames when possible) or
    'copy'; launch_depth: decode launches queued before batches coalesce;
    image_key: dict key of the image; skip_bad: drop malformed messages
    instead of failing; meta_to_device: move collated metadata to the GPU;
    log_every: seconds between metric log lines (None: off).
    """
    batch_size: int = 8
    rcvhwm: int = 10
    timeoutms: int = 10000
    prefetch: int = 4
    io_threads: Optional[int] = None
    staging_depth: int = 3
    h2d: str = 'auto'
    launch_depth: int = 2
    image_key: str = 'image'
    skip_bad: bool = False
    meta_to_device: bool = False
    log_every: Optional[float] = None

    def __post_init__(self):
        if self.h2d not in ('auto', 'copy'):
            raise ValueError("h2d must be 'auto' or 'copy'")
        if self.batch_size < 1 or self.prefetch < 1:
            raise ValueError('batch_size and prefetch must be >= 1')

    def kwargs(self) -> dict:
        return dataclasses.asdict(self)
