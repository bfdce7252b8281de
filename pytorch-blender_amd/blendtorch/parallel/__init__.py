"""Multi-GPU data distribution over RCCL/xGMI (one process per GPU).

The reference has no collectives at all: its only
scale-out axis is producer processes feeding DataLoader workers.  On an
MI355X node every GPU is a rank (``torch.distributed`` with backend
``"nccl"`` = RCCL) and rendered batches reach each GPU one of two ways:

* **shard mode** (default, :func:`shard_addresses`): each rank owns a
  disjoint subset of the producers and streams its own frames straight into
  its own HBM -- no GPU-GPU traffic on the hot path, weak scaling by
  construction;
* **pool mode** (:func:`pool_addresses`): every rank launches its producers
  but connects to all of them; PUSH round-robin balances frames across the
  GPUs, which is the reference's fan-out semantics at node scale;
* **scatter mode** (:class:`ScatterLoader`): a root rank receives
  ``world x B`` undecoded u8 frames and hands each rank its B-image shard
  plus packed metadata bytes in one grouped send/recv round
  (``batch_isend_irecv``: the root drives all its xGMI links concurrently --
  point-to-point links, so a ring would be the wrong shape here); each rank
  decodes its own shard.

Plus the small collectives the examples need: :func:`broadcast_tensor`
(duplex simulation parameters), :func:`all_gather_stats` (per-rank
throughput), and process-group setup helpers.
"""
from __future__ import annotations

import datetime
import os
from typing import Dict, Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist

from .comm import DeviceComm  # noqa: E402
from .grads import GradBuckets  # noqa: E402
from .topology import parse_cpulist, plan_rank_cpus, plan_rank_resources  # noqa: E402

__all__ = ['init_distributed', 'rank_world', 'shard_addresses', 'pool_addresses', 'partition_cpus', 'plan_rank_cpus',
           'parse_cpulist',
           'scatter_batch', 'broadcast_tensor', 'all_gather_stats', 'ScatterLoader', 'barrier', 'pack_meta',
           'unpack_meta', 'DeviceComm', 'GradBuckets', 'plan_rank_resources']


def rank_world():
    """(rank, world_size, local_rank) from the process group or the environment."""
    if dist.is_available() and dist.is_initialized():
        r, w = dist.get_rank(), dist.get_world_size()
    else:
        r, w = int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1))
    return r, w, int(os.environ.get('LOCAL_RANK', r))


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600):
    """Initialise the default process group from torchrun's environment.

    Backend ``nccl`` (RCCL) when GPUs are visible, else ``gloo``.  Sets the
    current HIP device to LOCAL_RANK.  No-op for WORLD_SIZE == 1 unless a
    backend is forced.  Returns (rank, world, device).
    """
    rank, world, local = rank_world()
    use_gpu = torch.cuda.is_available()
    # local % count: several ranks may share a GPU when rehearsing with gloo
    device = torch.device('cuda', local % max(1, torch.cuda.device_count())) if use_gpu else torch.device('cpu')
    if use_gpu:
        torch.cuda.set_device(device)
    backend = backend or os.environ.get('BLENDTORCH_DIST_BACKEND') or None   # e.g. gloo to rehearse ranks on one GPU
    if (world > 1 or backend is not None) and not dist.is_initialized():
        backend = backend or ('nccl' if use_gpu else 'gloo')
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == 'nccl':
            kw['device_id'] = device
        dist.init_process_group(**kw)
        rank, world = dist.get_rank(), dist.get_world_size()
    return rank, world, device


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def pool_addresses(local_addresses: Sequence[str]) -> List[str]:
    """Pool mode: every rank's producer addresses, gathered on every rank.

    A loader that connects to the whole pool gets the reference's M producers
    x W consumers topology across GPUs (examples/datagen/Readme.md:168-177):
    each producer's PUSH socket round-robins frames over all connected ranks,
    so a slower rank simply receives fewer frames, and a dead producer only
    thins the pool.  Same-host shared-memory frames stay zero-copy: any rank
    can map a producer's ring and hand the slot back.
    """
    local = list(local_addresses)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, local)
    return [a for part in gathered for a in part]


def shard_addresses(addresses: Sequence[str], rank: int, world: int) -> List[str]:
    """Round-robin disjoint subset of producer addresses for ``rank``.

    Every address belongs to exactly one rank; with fewer addresses than
    ranks, ranks share (``addresses[rank % n]``) so nobody starves.
    """
    addresses = list(addresses)
    if not addresses:
        return []
    if len(addresses) < world:
        return [addresses[rank % len(addresses)]]
    return addresses[rank::world]


def partition_cpus(cpus: Sequence[int], local_rank: int, local_world: int) -> List[int]:
    """Contiguous slice of the node's CPUs for one local rank (producer pinning)."""
    cpus = list(cpus)
    share = max(1, len(cpus) // max(1, local_world))
    mine = cpus[local_rank * share:(local_rank + 1) * share]
    return mine or cpus


def scatter_batch(full: Optional[torch.Tensor], shard_shape: Sequence[int], dtype: torch.dtype,
                  device: torch.device, src: int = 0) -> torch.Tensor:
    """Scatter ``full`` (``[world*B, ...]`` on ``src``) so rank r gets rows
    ``[r*B, (r+1)*B)``.  One grouped P2P round: the root posts all sends at
    once so every xGMI link carries its shard concurrently."""
    rank, world, _ = rank_world()
    out = torch.empty(tuple(shard_shape), dtype=dtype, device=device)
    if world == 1:
        out.copy_(full)
        return out
    B = shard_shape[0]
    if rank == src:
        assert full is not None and full.shape[0] == world * B
        ops = []
        for r in range(world):
            if r == src:
                out.copy_(full[r * B:(r + 1) * B])
            else:
                ops.append(dist.P2POp(dist.isend, full[r * B:(r + 1) * B].contiguous(), r))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    else:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, out, src)]):
            w.wait()
    return out


def broadcast_tensor(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    """In-place broadcast (e.g. densityopt's simulation parameters)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src)
    return t


def all_gather_stats(stats: Dict[str, float], device: Optional[torch.device] = None) -> List[Dict[str, float]]:
    """Gather a flat dict of numbers from every rank (same keys everywhere)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [dict(stats)]
    keys = sorted(stats)
    dev = device or (torch.device('cuda', torch.cuda.current_device())
                     if dist.get_backend() == 'nccl' else torch.device('cpu'))
    t = torch.tensor([float(stats[k]) for k in keys], dtype=torch.float64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [dict(zip(keys, o.tolist())) for o in out]


_META_DTYPES = {}


def _meta_schema(batch, n, image_key):
    """Split a collated batch's metadata into fixed-size tensor keys (sent as
    raw bytes in the image round) and everything else (object keys)."""
    tensors, objects = [], []
    for k, v in batch.items():
        if k == image_key:
            continue
        if isinstance(v, torch.Tensor) and v.dim() >= 1 and v.shape[0] == n and not v.is_complex():
            tensors.append((k, str(v.dtype).replace('torch.', ''), tuple(v.shape[1:])))
        else:
            objects.append(k)
    return tensors, objects


def _meta_row_bytes(schema):
    row = 0
    for _, dt, shp in schema:
        per = torch.tensor([], dtype=getattr(torch, dt)).element_size()
        for d in shp:
            per *= int(d)
        row += per
    return row


def pack_meta(batch, schema, n, out=None):
    """Per-item bytes of every tensor key, concatenated: u8 [n, M] (CPU).

    Every key must still match the agreed ``schema`` (dtype and per-item
    shape): the peers' receive buffers were sized from it, and a row of a
    different width would corrupt or hang the point-to-point round.
    ``out``: an [n, M] u8 CPU tensor (e.g. pinned) to write into."""
    cols = []
    for k, dt, shape in schema:
        v = batch[k]
        if not isinstance(v, torch.Tensor) or str(v.dtype).replace('torch.', '') != dt \
                or tuple(v.shape[1:]) != tuple(shape) or v.shape[0] != n:
            got = (tuple(v.shape), str(v.dtype)) if isinstance(v, torch.Tensor) else type(v).__name__
            raise ValueError(f'scatter metadata {k!r} changed: agreed ({dt}, [{n}, *{tuple(shape)}]), got {got}')
        v = v.detach().to('cpu').contiguous()
        cols.append(v.reshape(n, -1).view(torch.uint8).reshape(n, -1))
    row = sum(c.shape[1] for c in cols)
    if row != _meta_row_bytes(schema):
        raise ValueError(f'scatter metadata row is {row} bytes, the agreed schema says {_meta_row_bytes(schema)}')
    if out is None:
        if not cols:
            return torch.zeros((n, 0), dtype=torch.uint8)
        return torch.cat(cols, dim=1).contiguous()
    if tuple(out.shape) != (n, row):
        raise ValueError(f'pack_meta: out is {tuple(out.shape)}, need {(n, row)}')
    off = 0
    for c in cols:
        out[:, off:off + c.shape[1]].copy_(c)
        off += c.shape[1]
    return out


def unpack_meta(packed, schema):
    """Inverse of :func:`pack_meta` (views into ``packed``; any device)."""
    out, off = {}, 0
    n = packed.shape[0]
    for k, dt, shape in schema:
        dtype = getattr(torch, dt)
        per = int(torch.tensor([], dtype=dtype).element_size())
        for d in shape:
            per *= int(d)
        col = packed[:, off:off + per].contiguous()
        out[k] = col.view(dtype).reshape((n,) + tuple(shape))
        off += per
    return out


class ScatterLoader:
    """Scatter-mode distribution (north-star config 3): ONE root rank receives
    ``world * B`` frames per step and every rank gets its B-frame shard.

    What crosses xGMI is the undecoded u8 pixels (3-4 B/px instead of 12 B/px
    of fp32 planes) plus every fixed-size metadata tensor (btid, frameid,
    keypoints ...) packed into one byte row per item -- both in ONE grouped
    point-to-point round: the root posts a send per peer at once, so each
    point-to-point xGMI link carries its shard concurrently (a ring would
    serialise them).  Every rank then runs the fused decode kernel on its own
    shard.  The metadata schema is agreed once (first step) and every later
    batch is checked against it; only keys that are not fixed-size tensors
    (rare) fall back to a per-step object scatter.

    No per-step host synchronisation on RCCL: the sends/receives are RCCL
    calls on the compute stream (:class:`~.comm.DeviceComm`), the peers'
    metadata rows are packed into a reused pinned buffer and copied to the
    device asynchronously (the root keeps its own rows as the collated host
    tensors, like shard mode; peers get device tensors), and receive buffers
    come from the caching allocator.  The decode kernel follows on the same
    stream.

    Params
    ------
    source: iterable of batch dicts on the root (ignored elsewhere): the image
        under ``image_key`` is u8 ``[world*B, H, W, C]`` channels-last (a
        :class:`~blendtorch.btt.gpu.DeviceLoader` with
        ``DecodeConfig.raw(...)``), metadata collated per item.
    batch_size: per-rank B.
    decode: :class:`~blendtorch.ops.DecodeConfig` applied to each shard (None:
        deliver the u8 shard).  CUDA shards run the gfx950 kernel, CPU shards
        (gloo rehearsals) the PyTorch reference -- bit-identical.
    device: where shards land and are decoded.
    num_batches: steps to deliver (all ranks must agree).
    comm: a :class:`~.comm.DeviceComm` (default: one is created on the world
        group when the first step runs -- collective).
    comm_device: device of the tensors handed to a non-native (gloo) group
        (default CPU for gloo, ``device`` otherwise).

    Reference semantics: the fan-out of PUSH/PULL round-robin across consumers
    (examples/datagen/Readme.md:168-177) and densityopt's partition of work
    over instances (examples/densityopt/densityopt.py:95-107).
    """

    def __init__(self, source: Optional[Iterable], batch_size: int, decode, device: torch.device,
                 num_batches: int, image_key: str = 'image', src: int = 0, comm_device=None, comm=None):
        self.source = source
        self.batch_size = int(batch_size)
        self.decode = decode
        self.device = torch.device(device)
        self.num_batches = int(num_batches)
        self.image_key = image_key
        self.src = src
        self.comm_device = comm_device
        self.comm = comm
        self._pinned = None
        self.stats = {'steps': 0, 'object_scatters': 0, 'bytes_sent': 0}

    def __len__(self):
        return self.num_batches

    def _comm_dev(self):
        if self.comm_device is not None:
            return torch.device(self.comm_device)
        if dist.is_available() and dist.is_initialized() and dist.get_backend() != 'nccl':
            return torch.device('cpu')
        return self.device

    def _decode(self, shard):
        if self.decode is None:
            return shard
        from .. import ops
        if shard.is_cuda:
            return ops.decode(shard, self.decode)
        return ops.reference_decode(shard, self.decode)

    def _pack(self, batch, schema, n, cdev):
        """Metadata rows on ``cdev``: packed into a reused (pinned) host
        buffer, then one asynchronous copy."""
        row = _meta_row_bytes(schema)
        if cdev.type != 'cuda':
            return pack_meta(batch, schema, n)
        if self._pinned is None or tuple(self._pinned[0].shape) != (n, row):
            # two host buffers used alternately: the async copy of step k may
            # still read one while step k+1 packs the other
            self._pinned = [torch.empty((n, row), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
            self._pin_ev = [None, None]
            self._pin_i = 0
        i = self._pin_i
        self._pin_i ^= 1
        if self._pin_ev[i] is not None:
            self._pin_ev[i].synchronize()      # the copy that read it two steps ago (long done)
        host = pack_meta(batch, schema, n, out=self._pinned[i])
        dev = torch.empty((n, row), dtype=torch.uint8, device=cdev)
        dev.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(cdev))
        self._pin_ev[i] = ev
        return dev

    def __iter__(self):
        rank, world, _ = rank_world()
        multi = world > 1 and dist.is_available() and dist.is_initialized()
        if multi and self.comm is None:
            from .comm import DeviceComm
            self.comm = DeviceComm(device=self.device if self.device.type == 'cuda' else None)
        comm = self.comm
        it = iter(self.source) if rank == self.src else None
        B = self.batch_size
        cdev = self.device if (comm is not None and comm.native) else self._comm_dev()
        header = None          # (H, W, C, tensor schema, object keys), agreed on the first step
        for _ in range(self.num_batches):
            batch = next(it) if rank == self.src else None
            if header is None:
                if rank == self.src:
                    img0 = batch[self.image_key]
                    if img0.dtype != torch.uint8 or img0.dim() != 4 or img0.shape[0] != world * B:
                        raise ValueError(f'scatter source must deliver u8 [{world * B},H,W,C] images, got '
                                         f'{img0.dtype} {tuple(img0.shape)}')
                    header = (tuple(img0.shape[1:]),) + _meta_schema(batch, world * B, self.image_key)
                if multi:
                    box = [header]
                    dist.broadcast_object_list(box, src=self.src)
                    header = box[0]
                row_bytes = _meta_row_bytes(header[1])
            shape, schema, objects = header
            if rank == self.src:
                full = batch[self.image_key]
                if tuple(full.shape) != (world * B,) + tuple(shape) or full.dtype != torch.uint8:
                    raise ValueError(f'scatter source changed its image shape: {tuple(full.shape)}')
                if full.device != cdev:
                    full = full.to(cdev)
                img = full[self.src * B:(self.src + 1) * B]
                if multi:
                    # only the peers' metadata rows travel (packed, pinned, async H2D);
                    # the root keeps its own rows as the collated host tensors
                    meta = self._pack(batch, schema, world * B, cdev)
                    ops_ = []
                    for r in range(world):
                        if r != self.src:
                            ops_.append((True, full[r * B:(r + 1) * B], r))
                            ops_.append((True, meta[r * B:(r + 1) * B], r))
                    comm.p2p(ops_)
                    self.stats['bytes_sent'] += (world - 1) * B * (full[0].numel() + row_bytes)
                own = {k: batch[k][self.src * B:(self.src + 1) * B] for k, _, _ in schema}
            else:
                img = torch.empty((B,) + tuple(shape), dtype=torch.uint8, device=cdev)
                mrow = torch.empty((B, row_bytes), dtype=torch.uint8, device=cdev)
                comm.p2p([(False, img, self.src), (False, mrow, self.src)])
                own = unpack_meta(mrow, schema)
            if img.device != self.device:
                img = img.to(self.device, non_blocking=True)
            out = {self.image_key: self._decode(img)}
            out.update(own)
            if objects:
                # keys that are not fixed-size tensors: the slow path, per step
                self.stats['object_scatters'] += 1
                parts = None
                if rank == self.src:
                    parts = [{k: _slice_obj(batch[k], r * B, (r + 1) * B) for k in objects} for r in range(world)]
                if multi:
                    box = [None]
                    dist.scatter_object_list(box, parts, src=self.src)
                    out.update(box[0])
                else:
                    out.update(parts[0])
            self.stats['steps'] += 1
            yield out
        if it is not None and hasattr(it, 'close'):
            it.close()      # finish the root's loader so its stats are final


def _slice_obj(v, a, b):
    try:
        return v[a:b]
    except TypeError:
        return v
