"""Collectives enqueued on the compute stream: RCCL called directly.

``torch.distributed`` (backend ``nccl`` = RCCL) runs every collective on the
process group's own internal stream and joins it to the caller's stream with
events.  For the tiny, latency-bound collectives of this framework -- one
gradient bucket per training step, a few KB of simulation parameters, one
image shard per peer -- that join is the cost: eagerly each cross-stream wait
costs tens to hundreds of microseconds of host time on ROCm 7
(profiles/r2/hip_api_cost.json), and captured in a HIP graph it turns the
step into a fork/join DAG that replays node by node (profiles/r3/dp_tax.md).

:class:`DeviceComm` takes the communicator torch already built for a process
group (``ProcessGroupNCCL._comm_ptr()``) and enqueues ``ncclAllReduce`` /
``ncclBroadcast`` / grouped ``ncclSend``/``ncclRecv`` straight onto the
current HIP stream through the ``_hip`` extension (csrc/gpu/comm.cpp):

* no cross-stream events: an eager step pays one RCCL enqueue;
* capturable: inside ``torch.cuda.graph`` the collective becomes a node of the
  same linear queue as the step's kernels;
* the communicator is the process group's own (default) or, with
  ``dedicated=True``, one of its own (a ``dist.new_group``).  Measured on one
  MI355X with a 1-rank group (profiles/r3/pg_ab.md): the graphed training
  step's in-graph all-reduce costs 1.6 % on a dedicated communicator and 20 %
  on the shared one -- so the training step (:class:`~.step.CapturedStep`,
  densityopt) uses a dedicated one; streaming with no per-step collective
  loses 25 % to a second communicator existing at all -- so loaders share.
  Sharing is safe because both users serialise on the compute stream: a
  blocking c10d collective first waits for the caller's stream and the
  caller's stream then waits for it, so every rank sees one order of
  operations on the communicator.  Keep c10d calls on that group blocking
  (``async_op=False``) while a shared :class:`DeviceComm` uses it.

With gloo (CPU rehearsals) or without the extension every method falls back
to the equivalent ``torch.distributed`` call, so the same training code runs
in the CPU test suite.

The reference has no collectives; this backs the
data-parallel step (:class:`~blendtorch.parallel.grads.GradBuckets`), the
densityopt parameter broadcast and the scatter loader.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

__all__ = ['DeviceComm']

# nccl.h ncclDataType_t / ncclRedOp_t (stable across RCCL 2.x)
_DT = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
       torch.float64: 8, torch.bfloat16: 9, torch.bool: 1}
_OPS = {'sum': 0, 'prod': 1, 'max': 2, 'min': 3, 'avg': 4}
_C10D_OPS = {'sum': dist.ReduceOp.SUM, 'prod': dist.ReduceOp.PRODUCT, 'max': dist.ReduceOp.MAX,
             'min': dist.ReduceOp.MIN}


def _nonblocking():
    v = os.environ.get('TORCH_NCCL_USE_COMM_NONBLOCKING', '0').strip().lower()
    return v not in ('', '0', 'false', 'no', 'off')


def _rccl_path():
    return os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl.so')


class DeviceComm:
    """Collectives on the caller's stream over the process group's communicator (or, with
    ``dedicated=True``, a communicator of its own).

    Collective to construct: every rank of ``group`` (default: the whole
    world) must create it, in the same order relative to other collectives.

    ``native`` is True when RCCL is called directly (nccl backend, GPU
    tensors); otherwise methods go through ``torch.distributed``.
    ``force_native=False`` keeps the c10d path even on RCCL (comparison).
    """

    def __init__(self, group=None, device: Optional[torch.device] = None, dedicated: bool = False,
                 force_native: Optional[bool] = None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError('DeviceComm needs an initialised process group')
        base = group if group is not None else dist.group.WORLD
        self.backend = dist.get_backend(base)
        self.group = dist.new_group(ranks=dist.get_process_group_ranks(base), backend=self.backend) \
            if dedicated else base
        self.world = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        self.device = torch.device(device) if device is not None else (
            torch.device('cuda', torch.cuda.current_device()) if self.backend == 'nccl' else torch.device('cpu'))
        self._ext = None
        self._comm = 0
        self._backend_obj = None
        want = self.backend == 'nccl' if force_native is None else bool(force_native)
        if want and force_native is None and _nonblocking():
            # a nonblocking communicator returns ncclInProgress from enqueue calls,
            # which the direct path does not poll: keep the c10d path then
            want = False
        if want and self.backend == 'nccl':
            self._attach()
        elif want:
            raise RuntimeError(f'DeviceComm(force_native=True) needs the nccl backend, not {self.backend}')

    # -- setup ------------------------------------------------------------------
    def _attach(self):
        from .. import ops
        ext = ops.hip_ext()
        ext.rccl_load(_rccl_path())
        # make torch build (and connect) this group's communicator, then borrow it
        t = torch.zeros(1, device=self.device)
        dist.all_reduce(t, group=self.group)
        torch.cuda.synchronize(self.device)
        be = self.group._get_backend(self.device)
        comm = int(be._comm_ptr())
        if not comm:
            raise RuntimeError('DeviceComm: the process group has no RCCL communicator for this device')
        n, r = ext.rccl_count(comm), ext.rccl_rank(comm)
        if (n, r) != (self.world, self.rank):
            raise RuntimeError(f'DeviceComm: communicator is rank {r} of {n}, process group says '
                               f'{self.rank} of {self.world}')
        self._ext, self._comm = ext, comm
        # the borrowed communicator lives as long as this backend object (and
        # the process group it belongs to): keep a reference, and check the
        # group is still registered before every direct call (_live)
        self._backend_obj = be

    def _live(self):
        """Raise instead of calling RCCL through a communicator whose process
        group was destroyed (``dist.destroy_process_group``): the borrowed
        pointer would dangle."""
        ok = dist.is_initialized()
        if ok:
            try:
                from torch.distributed import distributed_c10d as c10d
                ok = self.group in c10d._world.pg_map
            except (AttributeError, ImportError):   # private registry moved: trust is_initialized
                pass
        if not ok:
            self._comm, self._ext, self._backend_obj = 0, None, None
            raise RuntimeError('DeviceComm: its process group was destroyed; the RCCL communicator is gone')

    def close(self):
        """Drop the borrowed communicator (before destroying the process group)."""
        self._comm, self._ext, self._backend_obj = 0, None, None

    @property
    def native(self) -> bool:
        return self._comm != 0

    def _stream(self, t):
        return torch.cuda.current_stream(t.device).cuda_stream

    def _check(self, t):
        self._live()
        if not t.is_cuda or t.device != self.device:
            raise ValueError(f'DeviceComm: tensor on {t.device}, communicator on {self.device}')
        if not t.is_contiguous():
            raise ValueError('DeviceComm: tensors must be contiguous')
        if t.dtype not in _DT:
            raise ValueError(f'DeviceComm: unsupported dtype {t.dtype}')

    def async_error(self) -> str:
        """RCCL's asynchronous error state of the communicator ('' when healthy)."""
        return self._ext.rccl_async_error(self._comm) if self.native else ''

    # -- collectives --------------------------------------------------------------
    def all_reduce_(self, t: torch.Tensor, op: str = 'sum') -> torch.Tensor:
        """In-place all-reduce of ``t`` (``op``: sum / prod / max / min / avg)."""
        if self.native:
            self._check(t)
            self._ext.rccl_all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], _OPS[op], self._comm,
                                      self._stream(t))
            return t
        buf = self._host(t)
        if op == 'avg':
            dist.all_reduce(buf, group=self.group)
            buf.div_(self.world)
        else:
            dist.all_reduce(buf, op=_C10D_OPS[op], group=self.group)
        return self._back(t, buf)

    def _host(self, t):
        # gloo rehearsals may hand GPU tensors: stage them through the host
        return t.cpu() if (t.is_cuda and self.backend != 'nccl') else t

    @staticmethod
    def _back(t, buf):
        if buf is not t:
            t.copy_(buf)
        return t

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        """In-place broadcast from group rank ``src``."""
        if self.native:
            self._check(t)
            self._ext.rccl_broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], int(src), self._comm,
                                     self._stream(t))
            return t
        buf = self._host(t)
        dist.broadcast(buf, dist.get_global_rank(self.group, src), group=self.group)
        return self._back(t, buf)

    def p2p(self, ops: Sequence[Tuple[bool, torch.Tensor, int]]):
        """One group of point-to-point transfers: ``(is_send, tensor, peer)``
        with group-rank peers.  All transfers of the group progress together
        (every xGMI link of a root busy at once)."""
        if not ops:
            return
        if self.native:
            spec = []
            for is_send, t, peer in ops:
                self._check(t)
                spec.append((1 if is_send else 0, t.data_ptr(), t.numel(), _DT[t.dtype], int(peer)))
            self._ext.rccl_p2p(spec, self._comm, self._stream(ops[0][1]))
            return
        bufs = [self._host(t) for _, t, _ in ops]
        p2p = [dist.P2POp(dist.isend if s else dist.irecv, b, dist.get_global_rank(self.group, peer), self.group)
               for (s, _, peer), b in zip(ops, bufs)]
        for w in dist.batch_isend_irecv(p2p):
            w.wait()
        for (s, t, _), b in zip(ops, bufs):
            if not s:
                self._back(t, b)

    # -- start-up self-check ------------------------------------------------------
    def selfcheck(self, nbytes: int = 1 << 20, timeout_s: float = 60.0) -> dict:
        """Exercise the paths a multi-GPU run depends on before it starts:

        1. a point-to-point ring (send ``nbytes`` to rank+1, receive from
           rank-1) -- the xGMI P2P path scatter mode uses, which an all-reduce
           alone does not prove;
        2. an all-reduce of device tensors (sum of rank+1 == w(w+1)/2);
        3. (native RCCL) the same all-reduce captured in a HIP graph between
           two kernels and replayed twice -- the form the data-parallel
           training step replays every step.

        Each stage is waited for with a host-side timeout; a hang or a wrong
        value raises ``RuntimeError`` naming this rank, the peer(s) and RCCL's
        asynchronous error state.  Returns timings (ms) per stage."""
        import time
        w, r = self.world, self.rank
        nxt, prv = (r + 1) % w, (r - 1) % w
        dev = self.device if self.native or self.backend == 'nccl' else torch.device('cpu')
        n = max(1, nbytes // 4)
        out = {}

        def wait(stage, peers):
            if dev.type != 'cuda':
                return
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            t_end = time.monotonic() + timeout_s
            while not ev.query():
                if time.monotonic() > t_end:
                    raise RuntimeError(f'rank {r}/{w}: RCCL self-check stage {stage!r} (peers {peers}) did not '
                                       f'complete within {timeout_s:.0f} s; async error: '
                                       f'{self.async_error() or "none"}')
                time.sleep(1e-3)

        t0 = time.perf_counter()
        send = torch.full((n,), float(r), device=dev)
        recv = torch.full((n,), -1.0, device=dev)
        if w > 1:
            self.p2p([(True, send, nxt), (False, recv, prv)])
        else:
            recv.copy_(send)
        wait('p2p ring', {'send_to': nxt, 'recv_from': prv})
        bad = int((recv != float(prv)).sum())
        if bad:
            raise RuntimeError(f'rank {r}/{w}: RCCL P2P ring delivered {bad} wrong values from rank {prv} '
                               f'(expected {float(prv)}, got {float(recv[0])})')
        out['p2p_ms'] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        t = torch.full((1024,), float(r + 1), device=dev)
        self.all_reduce_(t)
        wait('all_reduce', 'all')
        want = w * (w + 1) / 2
        if not bool((t == want).all()):
            raise RuntimeError(f'rank {r}/{w}: RCCL all-reduce gave {float(t[0])}, expected {want}')
        out['all_reduce_ms'] = (time.perf_counter() - t0) * 1e3
        out['native'] = self.native
        mode = os.environ.get('BT_SELFCHECK_GRAPH', 'temp')   # temp (default) | same | 0 (diagnostics)
        if self.native and mode != '0':
            if mode == 'same':
                out['graph_all_reduce_ms'] = self._selfcheck_graph(wait)
            else:
                # on a temporary communicator over the same ranks, destroyed afterwards: a
                # graph-captured collective on the training step's own communicator left it
                # ~25 % slower for the rest of the run (15.2k vs 20.9k img/s on the 1-rank
                # disc step, profiles/r6/b2/disc_pg1_*.jsonl)
                sub = dist.new_group(ranks=dist.get_process_group_ranks(self.group), backend='nccl')
                tmp = DeviceComm(group=sub, device=self.device)
                try:
                    out['graph_all_reduce_ms'] = tmp._selfcheck_graph(wait)
                finally:
                    tmp.close()
                    torch.cuda.synchronize(self.device)
                    dist.destroy_process_group(sub)
        return out

    def _selfcheck_graph(self, wait) -> float:
        """Stage 3: the collective as :class:`~.step.CapturedStep` runs it at
        world > 1 -- ``ncclAllReduce`` captured into a HIP graph with kernels
        around it, replayed twice.  A capture that RCCL rejects, a replay that
        hangs, or a wrong sum raises here, before any training step depends on it."""
        import time
        w, r = self.world, self.rank
        t0 = time.perf_counter()
        dev = self.device
        t = torch.empty((1024,), device=dev)
        acc = torch.zeros((1024,), device=dev)
        g = torch.cuda.CUDAGraph()
        try:
            # torch's shared default capture stream (the one CapturedStep's graphs use
            # too): a stream of its own here would be one more HIP stream for the
            # runtime to spread over its few hardware queues for the rest of the run
            with torch.cuda.device(dev), torch.cuda.graph(g, capture_error_mode='thread_local'):
                t.fill_(float(r + 1))
                self.all_reduce_(t)
                acc.add_(t)
        except RuntimeError as e:
            raise RuntimeError(f'rank {r}/{w}: capturing ncclAllReduce into a HIP graph failed ({e}); async '
                               f'error: {self.async_error() or "none"}') from e
        for _ in range(2):
            g.replay()
        wait('graph all_reduce (captured, 2 replays)', 'all')
        want = 2.0 * w * (w + 1) / 2
        if not bool((acc == want).all()):
            raise RuntimeError(f'rank {r}/{w}: graph-captured RCCL all-reduce gave {float(acc[0])} after 2 replays, '
                               f'expected {want}')
        del g
        return (time.perf_counter() - t0) * 1e3
