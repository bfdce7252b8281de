"""Persistent flat gradient buckets for data-parallel training steps.

``DistributedDataParallel`` cannot live inside a captured HIP graph (its
reducer does host-side bookkeeping per step), and packing gradients into a
fresh flat buffer per step (``torch.cat``), all-reducing it, dividing and
copying it back (``_foreach_copy_``) costs ~20 small kernels per step --
measured as a 45 % tax on the DCGAN consumer step even on one GPU
(profiles/r3/dp_tax.md).

:class:`GradBuckets` instead allocates the gradients ONCE as views into a few
flat buffers (one per dtype/device, at most ``bucket_mb`` each):

* every ``p.grad`` is permanently a view of its bucket, with ``p``'s own
  strides (channels-last conv weights stay channels-last);
* the gfx950 backward kernels (``blendtorch.ops``: MFMA weight gradient, fused
  BatchNorm, fused head) write the first gradient of a step straight into the
  view (``ops._grad_dest``): no AccumulateGrad kernel, no copy;
* the all-reduce runs in place on the flat bucket, directly on the compute
  stream (:class:`~blendtorch.parallel.comm.DeviceComm`), and the ``1/world``
  average folds into ``ops.FusedAdam(grad_scale=...)``: no ``div_`` kernel;
* views are 256-byte aligned so the optimizer's 16-byte vector loads apply.

Buckets are laid out in reverse parameter order (the order backward produces
gradients), so with several buckets the first one is complete earliest, and
:meth:`GradBuckets.arm` enqueues each bucket's all-reduce as soon as every
gradient in it has been written: the gfx950 backward kernels report each
bucket-view gradient they complete (``ops._GRAD_DONE``), and the collective
goes onto the compute stream right there, ahead of the rest of the backward
-- in a captured step, a node of the same linear queue before the first
layers' weight gradients (``n_buckets=2`` splits the DCGAN's 2.8 MB after the
last two layers).

Reference loop being data-paralleled: examples/densityopt/densityopt.py:257-331
(the reference itself trains single-process).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

__all__ = ['GradBuckets']

_ALIGN_BYTES = 256


def _dense(t):
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


class GradBuckets:
    """Flat persistent gradient storage for ``params``.

    Params
    ------
    params: parameters (those with ``requires_grad``) of one or more models.
    bucket_mb: maximum bucket size; a single parameter larger than this gets a
        bucket of its own.
    """

    def __init__(self, params: Sequence[torch.nn.Parameter], bucket_mb: float = 256.0, n_buckets: int = 0,
                 first_fraction: float = 0.7, second_sinks: bool = False):
        # second_sinks: a mirror of every bucket for a second gradient contribution per
        # step (two backward passes before one update, as densityopt's real / sim
        # halves): the backward kernels write it there and ops.FusedAdam adds it in
        # its update kernel -- without it autograd adds each second gradient into
        # .grad with one launch per parameter.  Only for optimizers that read it
        # (FusedAdam); the all-reduce covers the mirrors that were written.
        self.second_sinks = bool(second_sinks)
        self.buckets2: List[torch.Tensor] = []
        ps = [p for p in params if p.requires_grad]
        seen = set()
        self.params: List[torch.nn.Parameter] = []
        for p in ps:
            if id(p) not in seen:
                seen.add(id(p))
                self.params.append(p)
        for p in self.params:
            if not _dense(p):
                raise ValueError(f'GradBuckets: parameter {tuple(p.shape)} is not dense (contiguous / channels-last)')
        limit = max(1, int(bucket_mb * (1 << 20)))
        cut = None
        if n_buckets == 2:
            # two buckets: the first (the last layers' gradients, written first in
            # backward) ends once it holds first_fraction of the bytes, the second
            # takes the rest
            total = sum(p.numel() * p.element_size() for p in self.params)
            acc, cut = 0, set()
            for p in reversed(self.params):
                acc += p.numel() * p.element_size()
                cut.add(id(p))
                if acc >= first_fraction * total:
                    break
            limit = 1 << 62
        # group by (device, dtype), reverse order: the last layers' gradients come first in backward
        groups: Dict[tuple, List[torch.nn.Parameter]] = {}
        for p in reversed(self.params):
            groups.setdefault((p.device, p.dtype), []).append(p)
        self.buckets: List[torch.Tensor] = []
        self._members: List[List[torch.nn.Parameter]] = []
        for (dev, dt), members in groups.items():
            esz = torch.tensor([], dtype=dt).element_size()
            align = max(1, _ALIGN_BYTES // esz)
            cur, offs, size = [], [], 0
            for p in members:
                n = p.numel()
                if cur and ((size + n) * esz > limit or (cut is not None and id(cur[-1]) in cut
                                                         and id(p) not in cut)):
                    self._make(dev, dt, cur, offs, size)
                    cur, offs, size = [], [], 0
                offs.append(size)
                cur.append(p)
                size += -(-n // align) * align
            if cur:
                self._make(dev, dt, cur, offs, size)
        self.zero_()

    def _make(self, dev, dt, members, offs, size):
        flat = torch.zeros(size, dtype=dt, device=dev)
        flat2 = torch.zeros(size, dtype=dt, device=dev) if self.second_sinks else None
        for p, off in zip(members, offs):
            view = flat.as_strided(p.shape, p.stride(), off)
            p.grad = view
            p._bt_grad_sink = view
            if flat2 is not None:
                p._bt_grad_sink2 = flat2.as_strided(p.shape, p.stride(), off)
        self.buckets.append(flat)
        if flat2 is not None:
            self.buckets2.append(flat2)
        self._members.append(list(members))

    @property
    def numel(self) -> int:
        return sum(b.numel() for b in self.buckets)

    def attached(self) -> bool:
        """True while every parameter's ``.grad`` is still its bucket view."""
        return all(getattr(p, '_bt_grad_sink', None) is not None and p.grad is p._bt_grad_sink
                   for p in self.params)

    def zero_(self, memset: bool = True):
        """Start a step: the next gradient of each parameter overwrites its view.
        ``memset`` also clears the buckets (needed when some parameter's
        gradient comes from a kernel without a bucket sink, or not at all)."""
        if not self.attached():
            raise RuntimeError('GradBuckets: a parameter\'s .grad was replaced (zero_grad(set_to_none=True)?); '
                               'bucketed gradients must stay attached')
        if memset:
            for b in self.buckets + self.buckets2:
                b.zero_()
        for p in self.params:
            p._bt_grad_fresh = True
            if self.second_sinks:
                p._bt_grad_fresh2 = True
                p._bt_grad_second = False

    def arm_second(self):
        """Before a step's second backward pass (second_sinks): its gradients go to
        the second views again.  Host flags only -- a pass captured into a graph
        records where it writes, so call it before every capture of the second
        pass (densityopt captures one sim-half graph per static input tensor)."""
        if not self.second_sinks:
            return
        for p in self.params:
            p._bt_grad_fresh2 = True

    # -- all-reduce as soon as a bucket is complete ---------------------------------
    def arm(self, comm, op: str = 'sum'):
        """Before ONE backward pass: enqueue each bucket's all-reduce the
        moment its last gradient is reported written (``ops._GRAD_DONE``);
        :meth:`finish` (after the backward) reduces the rest.  Every gradient
        must come from exactly one contribution in this backward: a second one
        into an already reduced bucket raises."""
        from .. import ops
        if not self.attached():
            raise RuntimeError('GradBuckets: gradients were detached from their buckets')
        self._comm, self._op = comm, op
        self._where = {id(p): i for i, m in enumerate(self._members) for p in m}
        self._left = [{id(p) for p in m} for m in self._members]
        self._issued = [False] * len(self.buckets)
        self.order = []
        ops._GRAD_DONE = self._on_done
        ops._GRAD_LATE = self._on_late

    def _issue(self, i):
        from .. import ops
        self._issued[i] = True
        # (bucket, weight-gradient launches enqueued before its all-reduce): where it went
        self.order.append((i, ops.KERNEL_CALLS.get('conv_wgrad', 0)))
        b = self.buckets[i]
        if b.is_cuda:
            # weight gradients run on a side stream (ops.set_side_wgrad): a bucket
            # completed from the main stream also waits for the side stream's
            # launches; one completed from the side stream reduces there, behind them
            side = ops._SIDE_STREAMS.get(b.device) if b.device in ops._SIDE_PENDING else None
            cur = torch.cuda.current_stream(b.device)
            if side is not None and cur != side:
                cur.wait_stream(side)
        self._comm.all_reduce_(b, self._op)

    def _on_done(self, p):
        i = self._where.get(id(p))
        if i is None or self._issued[i]:
            return
        self._left[i].discard(id(p))
        if not self._left[i]:
            self._issue(i)

    def _on_late(self, p):
        i = self._where.get(id(p))
        if i is not None and self._issued[i]:
            raise RuntimeError('GradBuckets: a gradient arrived after its bucket was all-reduced '
                               '(several contributions per step need finish-time reduction: no arm())')

    def finish(self) -> int:
        """After the backward: reduce the buckets not reduced yet (gradients
        that never reported, or none at all); disarm.  Returns the number of
        collectives of the step."""
        from .. import ops
        ops._GRAD_DONE = ops._GRAD_LATE = None
        for i, done in enumerate(self._issued):
            if not done:
                self._issue(i)
        return len(self.buckets)

    def disarm(self):
        from .. import ops
        ops._GRAD_DONE = ops._GRAD_LATE = None

    def all_reduce(self, comm, op: str = 'sum') -> int:
        """Reduce every bucket in place over ``comm``
        (:class:`~blendtorch.parallel.comm.DeviceComm`).  Capturable when the
        communicator is native.  Returns the number of collectives issued."""
        if not self.attached():
            raise RuntimeError('GradBuckets: gradients were detached from their buckets')
        n = 0
        for i, b in enumerate(self.buckets):
            comm.all_reduce_(b, op)
            n += 1
            if self.buckets2 and any(getattr(p, '_bt_grad_second', False) for p in self._members[i]):
                comm.all_reduce_(self.buckets2[i], op)
                n += 1
        return n

    def detach(self):
        """Remove the buckets: parameters get ordinary gradients again."""
        for p in self.params:
            if getattr(p, '_bt_grad_sink', None) is not None:
                if p.grad is p._bt_grad_sink:
                    p.grad = p.grad.clone()
                del p._bt_grad_sink
            for a in ('_bt_grad_fresh', '_bt_grad_fresh2', '_bt_grad_second', '_bt_grad_sink2'):
                if hasattr(p, a):
                    delattr(p, a)
        self.buckets, self._members, self.buckets2 = [], [], []

    def __repr__(self):
        return (f'GradBuckets({len(self.params)} params, {len(self.buckets)} buckets, '
                f'{self.numel} elements)')
