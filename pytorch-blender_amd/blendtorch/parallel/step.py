"""Whole training steps as one HIP graph, data-parallel included.

A consumer step on the streamed batches (DCGAN discriminator, keypoint CNN)
is ~60-100 small kernels: eager PyTorch spends as long dispatching them as the
GPU spends running them (profiles/consumer_step.md: 1.07 ms eager vs 0.81 ms
graphed).  :class:`CapturedStep` captures forward, backward, the gradient
all-reduce and the optimizer update once and replays the graph per batch.

``DistributedDataParallel`` cannot live inside a captured graph (its reducer
hooks run host-side bookkeeping per step), so the data-parallel reduction is
done here explicitly, with nothing per step but the collective itself:

* gradients live permanently in flat buckets (:class:`~.grads.GradBuckets`);
  the gfx950 backward kernels write straight into them;
* each bucket is ONE in-place RCCL all-reduce enqueued on the compute stream
  (:class:`~.comm.DeviceComm`) -- inside the captured graph it is one more
  node of the same linear queue, not a fork/join onto c10d's stream;
* ``1/world`` is folded into ``ops.FusedAdam`` (``grad_scale``); other
  optimizers get an averaging all-reduce (``ncclAvg``).

A model of ~0.7 M parameters is one 2.8 MB bucket: one collective per step,
which suits xGMI's point-to-point links (per-collective latency dominates).
The previous per-step pack (``torch.cat``) / ``div_`` / ``_foreach_copy_``
cost 45 % of the step on one GPU (profiles/r3/dp_tax.md);
:func:`allreduce_gradients` keeps that path for callers without buckets.

The reference trains on the CPU-collated batches in eager PyTorch
(examples/densityopt/densityopt.py:257-331) and has no data parallelism.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

__all__ = ['allreduce_gradients', 'CapturedStep', 'ReplayWatchdog']


def _buckets(params: Sequence[torch.Tensor], bucket_bytes: int) -> List[List[torch.Tensor]]:
    out, cur, size = [], [], 0
    for p in params:
        nb = p.numel() * p.element_size()
        if cur and (size + nb > bucket_bytes or p.dtype != cur[0].dtype):
            out.append(cur)
            cur, size = [], 0
        cur.append(p)
        size += nb
    if cur:
        out.append(cur)
    return out


def allreduce_gradients(params: Sequence[torch.nn.Parameter], group=None, bucket_mb: float = 64.0,
                        average: bool = True, force: bool = False) -> int:
    """Average ``p.grad`` over the process group in flat buckets (one
    all-reduce each).  Capturable: no host synchronisation, no allocation
    outside the current stream's pool.  Returns the number of collectives.
    ``force`` issues the collectives even on a 1-rank group (rehearsal)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    world = dist.get_world_size(group)
    grads = [p.grad for p in params if p.grad is not None]
    if (world == 1 and not force) or not grads:
        return 0
    n = 0
    for b in _buckets(grads, int(bucket_mb * (1 << 20))):
        flat = torch.cat([g.reshape(-1) for g in b])
        dist.all_reduce(flat, group=group)
        if average:
            flat.div_(world)
        torch._foreach_copy_(b, [v.view_as(g) for v, g in zip(torch.split(flat, [g.numel() for g in b]), b)])
        n += 1
    return n


class ReplayWatchdog:
    """Host-side bound on steps that never finish (a collective waiting on a
    dead or diverged peer hangs the replay, and with it the whole job, with
    no message).  After every step an event is recorded; once more than
    ``depth`` steps are in flight the oldest one must complete within
    ``timeout_s`` or :class:`RuntimeError` names this rank and RCCL's
    asynchronous error state.  Costs one event record and one query per step
    (the oldest event is normally long done: the host waits on nothing).

    ``make_event`` / ``clock`` are injectable (CPU tests)."""

    def __init__(self, timeout_s: float, depth: int = 8, describe: Optional[Callable[[], str]] = None,
                 make_event: Optional[Callable[[], object]] = None, clock=None, sleep=None):
        import collections
        import time
        self.timeout_s, self.depth = float(timeout_s), max(1, int(depth))
        self.describe = describe or (lambda: '')
        self._make = make_event or self._cuda_event
        self._clock = clock or time.monotonic
        self._sleep = sleep or time.sleep
        self._q = collections.deque()
        self.steps = 0
        self.max_wait_s = 0.0

    @staticmethod
    def _cuda_event():
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def record(self):
        self._q.append((self.steps, self._make()))
        self.steps += 1
        while len(self._q) > self.depth:
            self._wait(*self._q.popleft())

    def drain(self):
        while self._q:
            self._wait(*self._q.popleft())

    def _wait(self, step, ev):
        if ev.query():
            return
        t0 = self._clock()
        while not ev.query():
            waited = self._clock() - t0
            if waited > self.timeout_s:
                raise RuntimeError(f'CapturedStep: step {step} did not complete within {self.timeout_s:.0f} s '
                                   f'({self.steps - step - 1} later steps enqueued behind it); '
                                   f'{self.describe()}')
            self._sleep(1e-3)
        self.max_wait_s = max(self.max_wait_s, self._clock() - t0)


class CapturedStep:
    """``step(x) -> loss`` for a fixed input shape, replayed from one HIP graph.

    Params
    ------
    model, optimizer: a torch optimizer must be created with
        ``capturable=True`` (its step counters then live on the GPU);
        ``ops.FusedAdam`` always is.
    loss_fn: ``loss_fn(model, x) -> scalar loss`` (forward + loss; may use
        autocast -- pass ``cache_enabled=False`` so replays recast live weights).
    allreduce: average gradients over the process group inside the step
        (data parallel without DDP); ``'always'`` also on a 1-rank group
        (rehearses the collective path on one GPU).
    warmup: eager steps on a side stream before capture (allocator, MIOpen
        algorithm search, optimizer state).
    graph: False runs the same step eagerly (fallback / comparison).
    comm: a :class:`~.comm.DeviceComm` to reduce over (default: one is
        created on the world group -- a collective call on every rank).
    buckets: False keeps the legacy per-step pack/all-reduce/copy-back path
        (:func:`allreduce_gradients`; comparison only).

    static_inputs: up to this many input tensors get a graph of their own
        that reads the tensor in place (captured the first time its storage
        shows up, sharing the first graph's memory pool) -- no per-step copy
        into a static buffer.  For a loader that cycles a fixed set of output
        tensors (``btt.DeviceLoader(reuse_buffers=True)``); further inputs
        are copied into a private buffer with a graph of its own.  Not with
        ``split``.
    overlap: (data parallel with buckets) two gradient buckets, and each
        bucket's all-reduce enqueued as soon as its gradients are written
        (:meth:`~.grads.GradBuckets.arm`): the last layers' bucket goes ahead of
        the first layers' weight gradients.  Only for a ``loss_fn`` whose
        parameters each get one gradient contribution per backward.
    group_steps: (with ``static_inputs``) that many consecutive steps per
        replay: steps are held until the group's last input arrives, then all
        run from one graph captured for that tuple of input tensors (the GPU
        idles ~13 us between two replays, profiles/r4/SUMMARY.md).  A held
        step returns ``None``; :meth:`flush` runs held steps one by one -- it
        runs by itself before the model's or the optimizer's ``state_dict()``
        and a step object dropped with steps held warns.  ``pair_steps=True``
        is ``group_steps=2``.  Every step's loss of the last call that ran
        steps is in :meth:`last_losses`.
    reuse_distance: how many later inputs the caller hands in before it may
        rewrite an input tensor in place (``btt.DeviceLoader(reuse_buffers=
        True)`` re-posts a ring tensor for refilling when the batch two
        behind it is handed out: 2, the default).  A held input must stay
        unchanged until its group replays, so ``group_steps`` may not exceed
        it.  An input modified in place while held (``x.copy_(batch);
        step(x)``, seen through the tensor's version counter) raises instead
        of training twice on the last batch.
    watchdog_s: a :class:`ReplayWatchdog` bound on each step's completion,
        checked once ``watchdog_depth`` later steps are enqueued: a step
        (collective) that hangs raises with the rank and RCCL's asynchronous
        error instead of hanging the job.  Default: 300 s when the step
        all-reduces over more than one rank, off otherwise (0 / None: off).
    strict: a capture failure raises instead of falling back to eager
        steps.  Default: on when the step all-reduces over more than one rank
        (a rank silently stepping eagerly replays its collectives in another
        form than its peers' graphs).
    split: capture forward+loss and backward+update as two graphs sharing one
        memory pool, so a caller can act between them: ``step(x, mid=fn)``
        runs ``fn()`` after enqueuing the forward (e.g. to gate the next
        batches' host->device DMA onto the backward's conv kernels instead of
        the memory-bound forward, see bench.py --dma-phase).

    ``state`` is ``'graph'`` after a successful capture, ``'eager'`` otherwise.
    An input whose layout (shape, strides, dtype, offset) differs from the
    captured one runs an eager step; a graph is never replayed for it.
    ``collectives`` is the number of all-reduces per step.

    Gradients of a bucketed step are never ``None``: a parameter that gets no
    gradient in some step sees a zero gradient, and Adam's moments still move
    it (``torch.optim.Adam`` after ``zero_grad(set_to_none=True)`` would skip
    it).  Keep such parameters out of the optimizer, or use ``buckets=False``.
    """

    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer,
                 loss_fn: Callable[[torch.nn.Module, torch.Tensor], torch.Tensor], allreduce=True,
                 warmup: int = 3, graph: bool = True, group=None, bucket_mb: float = 256.0, split: bool = False,
                 comm=None, buckets: bool = True, static_inputs: int = 0, overlap: bool = False,
                 pair_steps: bool = False, group_steps: int = 1, reuse_distance: int = 2,
                 watchdog_s: Optional[float] = -1.0, watchdog_depth: int = 8, strict: Optional[bool] = None):
        self.model, self.opt, self.loss_fn = model, optimizer, loss_fn
        self.split = split
        self.static_inputs = 0 if split else max(0, int(static_inputs))
        self._by_input = {}   # input data_ptr -> (graph, input tensor, loss)
        self.graph_bwd: Optional[torch.cuda.CUDAGraph] = None
        self.allreduce, self.warmup, self.group, self.bucket_mb = allreduce, warmup, group, bucket_mb
        self.state = 'pending' if graph else 'eager'
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.x = None
        self.loss = None
        self.collectives = 0
        self.error = None
        self.comm = None
        self.grads = None
        self._op = 'sum'
        active = bool(allreduce) and dist.is_available() and dist.is_initialized() and (
            dist.get_world_size(group) > 1 or allreduce == 'always')
        self._legacy = active and not buckets
        self._active = active
        self.overlap = bool(overlap) and active and buckets
        self._memset = True
        self._seed = None
        # persistent gradient buckets: always for a collective; without one too
        # when the optimizer clears the gradients it consumes (ops.FusedAdam):
        # then the step needs neither per-step gradient allocations nor a fill
        zeroing = hasattr(optimizer, 'set_zero_grads')
        if buckets and (active or zeroing):
            from .grads import GradBuckets
            self.grads = GradBuckets(model.parameters(), bucket_mb=bucket_mb, n_buckets=2 if self.overlap else 0)
            if zeroing:
                optimizer.set_zero_grads(True)
                # the optimizer clears only the gradients it consumes: a model
                # parameter outside it would accumulate across steps, so the
                # buckets are then cleared per step as well
                opt_ids = {id(p) for grp in optimizer.param_groups for p in grp['params']}
                self._memset = any(id(p) not in opt_ids for p in self.grads.params)
        self._static_mode = bool(self.static_inputs)
        self._copy_failed = False
        n = max(int(group_steps), 2 if pair_steps else 1)
        if n > 1 and self._static_mode and n > int(reuse_distance):
            raise ValueError(f'CapturedStep: group_steps={n} holds inputs longer than their reuse distance '
                             f'({reuse_distance}): a held buffer would be refilled before its group replays')
        self.group_steps = n if self._static_mode else 1
        self._held = []            # group_steps: (input, its version counter) of steps not yet enqueued
        self._groups = {}          # (data_ptr, ...) -> (graph, inputs, per-step losses)
        self._group_failed = False
        self._last_losses = []
        self._ran = None
        if self.group_steps > 1:
            # a checkpoint must not miss held steps: flush before either state_dict
            import weakref
            ref = weakref.ref(self)

            def _flush_hook(*_a, **_k):
                st = ref()
                if st is not None and st._held:
                    st.flush()
            for obj in (model, optimizer):
                reg = getattr(obj, 'register_state_dict_pre_hook', None)
                if reg is not None:
                    reg(_flush_hook)
        if active and buckets:
            from .comm import DeviceComm
            self.comm = comm if comm is not None else DeviceComm(group, dedicated=True)
            if hasattr(optimizer, 'set_grad_scale'):
                optimizer.set_grad_scale(1.0 / self.comm.world)   # folded into the update kernel
            else:
                self._op = 'avg'
        multi = active and dist.get_world_size(group) > 1
        self.strict = multi if strict is None else bool(strict)
        if watchdog_s is not None and watchdog_s < 0:
            watchdog_s = 300.0 if multi else None
        self.watchdog = None
        on_gpu = any(p.is_cuda for p in model.parameters())
        if watchdog_s and on_gpu:
            self.watchdog = ReplayWatchdog(watchdog_s, watchdog_depth, describe=self._describe)

    def _describe(self) -> str:
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        err = ''
        if self.comm is not None:
            try:
                err = self.comm.async_error()
            except Exception as e:     # (the report must not hide the hang)
                err = f'<async_error failed: {e}>'
        return f'rank {rank}/{world}, state {self.state!r}, RCCL async error: {err or "none"}'

    def _forward(self, x):
        if self.grads is not None:
            self.grads.zero_(memset=self._memset)
        else:
            self.opt.zero_grad(set_to_none=True)
        return self.loss_fn(self.model, x)

    def _backward(self, loss):
        # the backward's seed gradient: one persistent tensor of ones, not a
        # fill kernel per step
        if self._seed is None or self._seed.shape != loss.shape or self._seed.device != loss.device \
                or self._seed.dtype != loss.dtype:
            self._seed = torch.ones_like(loss)
        # ops.FusedAdam: the step's schedule rides in a launch of the backward (its first fused
        # data + weight gradient, or its last slice reduce: one launch fewer per step)
        attach = getattr(self.opt, 'attach_schedule', None)
        if attach is not None:
            attach()
        # ... and, with no collective reading the gradients before the update, the backward's last
        # slice reduce rides in the update launch (FusedAdam.attach_reduce)
        fuse = not self._active and getattr(self.opt, 'attach_reduce', None) is not None and self.opt.attach_reduce()
        try:
            self._backward_only(loss)
        except BaseException:
            if attach is not None:
                self.opt.detach_schedule()
            if fuse:
                self.opt.detach_reduce()
            raise
        try:
            self.opt.step()
        finally:
            if fuse:
                self.opt.detach_reduce()
        return loss.detach()

    def _backward_only(self, loss):
        if self.overlap and self.grads is not None and self.comm is not None:
            # each bucket's all-reduce is enqueued the moment its last gradient is
            # (the last layers' bucket ahead of the first layers' weight gradients)
            self.grads.arm(self.comm, self._op)
            try:
                loss.backward(self._seed)
            except BaseException:
                self.grads.disarm()
                raise
            self.collectives = self.grads.finish()
        elif self.grads is not None and self.comm is not None:
            loss.backward(self._seed)
            self.collectives = self.grads.all_reduce(self.comm, self._op)
        elif self._legacy:
            loss.backward(self._seed)
            self.collectives = allreduce_gradients(self.model.parameters(), self.group, self.bucket_mb,
                                                   force=self.allreduce == 'always')
        else:
            loss.backward(self._seed)

    def _train(self, x):
        return self._backward(self._forward(x))

    def _capture(self, x):
        if self.static_inputs:
            self.x = x                       # read in place (the caller keeps it alive and unchanged)
        else:
            self.x = torch.empty_like(x)     # same strides (channels-last stays channels-last)
            self.x.copy_(x)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self._train(self.x)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        try:
            if self.grads is None:
                self.opt.zero_grad(set_to_none=True)
            if self.split:
                with torch.cuda.graph(g, capture_error_mode='thread_local'):
                    loss = self._forward(self.x)
                gb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb, pool=g.pool(), capture_error_mode='thread_local'):
                    self.loss = self._backward(loss)
                del loss
                self.graph_bwd = gb
            else:
                # thread_local: the stream loader's worker thread keeps making
                # HIP calls (event queries, copies) while this thread captures
                with torch.cuda.graph(g, capture_error_mode='thread_local'):
                    self.loss = self._train(self.x)
            self.graph, self.state = g, 'graph'
            if self.static_inputs:
                self._by_input[self.x.data_ptr()] = (g, self.x, self.loss)
        except RuntimeError as e:          # keep the run alive; callers report which mode ran
            self.error = str(e)
            self.state = 'eager'
            if self.strict:
                raise RuntimeError(f'CapturedStep: capture failed ({self._describe()}): {e}') from e

    def _same_layout(self, x):
        return (x.shape == self.x.shape and x.stride() == self.x.stride() and x.dtype == self.x.dtype
                and x.device == self.x.device and x.storage_offset() == self.x.storage_offset())

    def _capture_for(self, x, key=None):
        """One more graph of the step, reading ``x`` in place, in the first
        graph's memory pool (the graphs replay one at a time on one stream)."""
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, pool=self.graph.pool(), capture_error_mode='thread_local'):
                loss = self._train(x)
        except RuntimeError as e:
            self.error = str(e)
            self.static_inputs = self._n_static()        # no more in-place captures
            if key == 'copy':
                self._copy_failed = True                 # recorded once: later misses run eagerly
            return None
        ent = (g, x, loss)
        self._by_input[x.data_ptr() if key is None else key] = ent
        return ent

    def _n_static(self):
        return len(self._by_input) - ('copy' in self._by_input)

    def _lookup(self, x):
        """The graph that runs the step on ``x`` in static-input mode, or None
        (the caller then steps eagerly).  A graph is only ever replayed for
        an input of exactly the captured layout: a cache hit on the data
        pointer alone (e.g. ``x[:4]`` or a dtype view of a captured buffer)
        would replay the step for the captured shape."""
        if not self._same_layout(x):
            return None
        ent = self._by_input.get(x.data_ptr())
        if ent is None and self._n_static() < self.static_inputs:
            ent = self._capture_for(x)
        if ent is None and not self._copy_failed:
            # past the cap: copy into a private buffer with a graph of its own
            # (the captured inputs are callers' tensors, never written)
            ent = self._by_input.get('copy')
            if ent is None:
                ent = self._capture_for(torch.empty_like(x), key='copy')
            if ent is not None:
                ent[1].copy_(x)
        return ent

    def _group_entry(self, xs):
        """The graph that runs the steps on ``xs`` in order (captured on
        first use, in the first graph's pool), or None."""
        key = tuple(x.data_ptr() for x in xs)
        ent = self._groups.get(key)
        if ent is None and not self._group_failed and len(self._groups) < self.static_inputs:
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, pool=self.graph.pool(), capture_error_mode='thread_local'):
                    losses = [self._train(x) for x in xs]
            except RuntimeError as e:
                self.error = str(e)
                self._group_failed = True      # recorded once: single steps from here on
                return None
            ent = (g, tuple(xs), losses)
            self._groups[key] = ent
        return ent

    def _static_step(self, x, mid):
        # x is a caller's tensor (e.g. a loader ring buffer): never written
        ent = self._lookup(x)
        if ent is None:
            return self._eager(x, mid)
        ent[0].replay()
        if mid is not None:
            mid()
        return ent[2]

    def flush(self) -> Optional[torch.Tensor]:
        """group_steps: enqueue the held steps one by one (no-op otherwise).
        Returns the last step's loss (every step's in :meth:`last_losses`)."""
        held, self._held = self._held, []
        if not held:
            return None
        self._check_held(held)
        inside = self._ran is not None      # flushed by a call that runs a step of its own next
        losses = []
        for i, (x, _) in enumerate(held):
            loss = self._static_step(x, None)
            # two steps on one input replay one graph: keep the earlier value
            losses.append(loss.clone() if (inside or i + 1 < len(held)) and loss is not None else loss)
        if inside:
            self._ran.extend(losses)
        else:
            self._last_losses = losses
        return losses[-1]

    def last_losses(self) -> List[torch.Tensor]:
        """The loss of every step run by the last call that ran steps (a
        group replay runs ``group_steps``, :meth:`flush` the held ones), in
        step order.  Graph outputs: valid until the same graph replays again
        -- clone what must outlive that."""
        return list(self._last_losses)

    @staticmethod
    def _check_held(held):
        for x, ver in held:
            if x._version != ver:
                raise RuntimeError('CapturedStep: an input held for a grouped replay was modified in place before '
                                   'its group ran (e.g. x.copy_(batch); step(x)): its step would train on the '
                                   'later data.  Pass a distinct tensor per step, or use group_steps=1')

    def __del__(self):
        if getattr(self, '_held', None):
            import warnings
            warnings.warn(f'CapturedStep dropped with {len(self._held)} held step(s) never run: call flush()',
                          RuntimeWarning, stacklevel=2)

    def _eager(self, x, mid):
        loss = self._forward(x)
        if mid is not None:
            mid()
        return self._backward(loss)

    def _replay(self, mid):
        self.graph.replay()
        if self.graph_bwd is not None:
            if mid is not None:
                mid()
            self.graph_bwd.replay()
        elif mid is not None:
            mid()

    def __call__(self, x: torch.Tensor, mid: Optional[Callable[[], None]] = None) -> Optional[torch.Tensor]:
        """Run (or, grouped, hold) one step on ``x``.  Returns the step's loss,
        or ``None`` for a step held for a grouped replay (``group_steps > 1``):
        it runs with the group's last input or at :meth:`flush`."""
        self._ran = []                 # losses of every step this call runs, in order
        try:
            loss = self._call(x, mid)
        finally:
            ran, self._ran = self._ran, None
        if self.watchdog is not None and ran:
            self.watchdog.record()
        from .. import ops
        if ops.GRID_BARRIER_USED:
            ops.check_grid_barrier()   # a replayed BN-applying forward whose barrier gave up raises here
        if not ran and loss is not None:
            ran = [loss]
        if ran:
            self._last_losses = ran
        return loss

    def _call(self, x, mid):
        if self.state == 'pending':
            self._capture(x)
            if self.state == 'graph':
                self._replay(mid)
                return self.loss
        if self.state == 'graph':
            if self._static_mode:
                if self.group_steps > 1 and mid is None and self._same_layout(x):
                    self._held.append((x, x._version))
                    if len(self._held) < self.group_steps:
                        return None
                    held, self._held = self._held, []
                    self._check_held(held)
                    xs = [h[0] for h in held]
                    ent = self._group_entry(xs)
                    if ent is not None:
                        ent[0].replay()
                        self._ran.extend(ent[2])
                        return ent[2][-1]
                    self._held = held
                    loss = self.flush()
                    self._ran[-1] = loss       # the call's result itself needs no copy
                    return loss
                self.flush()                   # keep the steps in order
                loss = self._static_step(x, mid)
                self._ran.append(loss)
                return loss
            if x.shape != self.x.shape or x.dtype != self.x.dtype or x.device != self.x.device:
                return self._eager(x, mid)       # the graph is for the captured shape only (copy_ converts strides)
            if x.data_ptr() != self.x.data_ptr():
                self.x.copy_(x)
            self._replay(mid)
            return self.loss
        return self._eager(x, mid)
