"""Whole training steps as one HIP graph, data-parallel included.

A consumer step on the streamed batches (DCGAN discriminator, keypoint CNN)
is ~100 small kernels: eager PyTorch spends as long dispatching them as the
GPU spends running them (profiles/consumer_step.md: 1.07 ms eager vs 0.81 ms
graphed).  :class:`CapturedStep` captures forward, backward, the gradient
all-reduce and the optimizer update once and replays the graph per batch.

``DistributedDataParallel`` cannot live inside a captured graph (its reducer
hooks run host-side bookkeeping per step), so the data-parallel reduction is
done here explicitly: the gradients are flattened into buckets of at most
``bucket_mb`` and each bucket is one RCCL all-reduce enqueued on the capture
stream -- a captured collective replays with the graph like any kernel.  A
few large buckets suit xGMI's point-to-point ring (per-link bandwidth, fixed
per-collective latency) better than DDP's default 25 MB-but-many-hooks
pattern for a model this small (~0.7 M parameters = one bucket).

The reference trains on the CPU-collated batches in eager PyTorch
(examples/densityopt/densityopt.py:257-331) and has no data parallelism.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

__all__ = ['allreduce_gradients', 'CapturedStep']


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


class CapturedStep:
    """``step(x) -> loss`` for a fixed input shape, replayed from one HIP graph.

    Params
    ------
    model, optimizer: the optimizer must be created with ``capturable=True``
        (its step counters then live on the GPU).
    loss_fn: ``loss_fn(model, x) -> scalar loss`` (forward + loss; may use
        autocast -- pass ``cache_enabled=False`` so replays recast live weights).
    allreduce: average gradients over the default process group inside the
        graph (data parallel without DDP); ``'always'`` also on a 1-rank group.
    warmup: eager steps on a side stream before capture (allocator, MIOpen
        algorithm search, optimizer state).
    graph: False runs the same step eagerly (fallback / comparison).

    ``state`` is ``'graph'`` after a successful capture, ``'eager'`` otherwise.
    """

    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer,
                 loss_fn: Callable[[torch.nn.Module, torch.Tensor], torch.Tensor], allreduce: bool = True,
                 warmup: int = 3, graph: bool = True, group=None, bucket_mb: float = 64.0):
        self.model, self.opt, self.loss_fn = model, optimizer, loss_fn
        self.allreduce, self.warmup, self.group, self.bucket_mb = allreduce, warmup, group, bucket_mb
        self.state = 'pending' if graph else 'eager'
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.x = None
        self.loss = None
        self.collectives = 0
        self.error = None

    def _train(self, x):
        self.opt.zero_grad(set_to_none=True)
        loss = self.loss_fn(self.model, x)
        loss.backward()
        if self.allreduce:
            self.collectives = allreduce_gradients(self.model.parameters(), self.group, self.bucket_mb,
                                                   force=self.allreduce == 'always')
        self.opt.step()
        return loss.detach()

    def _capture(self, x):
        self.x = torch.empty_like(x)         # same strides (channels-last stays channels-last)
        self.x.copy_(x)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self._train(self.x)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        try:
            self.opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(g):
                self.loss = self._train(self.x)
            self.graph, self.state = g, 'graph'
        except RuntimeError as e:          # keep the run alive; callers report which mode ran
            self.error = str(e)
            self.state = 'eager'

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if self.state == 'pending':
            self._capture(x)
            if self.state == 'graph':
                self.graph.replay()
                return self.loss
        if self.state == 'graph':
            if x.data_ptr() != self.x.data_ptr():
                self.x.copy_(x)
            self.graph.replay()
            return self.loss
        return self._train(x)
