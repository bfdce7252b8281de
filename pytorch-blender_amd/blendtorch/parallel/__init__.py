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
  ``world x B`` frames and hands each rank its B-image shard with one
  grouped send/recv round (``batch_isend_irecv``: the root drives all its
  xGMI links concurrently -- point-to-point links, so a ring would be the
  wrong shape here), metadata follows as one small object scatter.

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

from .topology import parse_cpulist, plan_rank_cpus  # noqa: E402

__all__ = ['init_distributed', 'rank_world', 'shard_addresses', 'pool_addresses', 'partition_cpus', 'plan_rank_cpus',
           'parse_cpulist',
           'scatter_batch', 'broadcast_tensor', 'all_gather_stats', 'ScatterLoader', 'barrier']


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


class ScatterLoader:
    """Scatter-mode distribution: the root rank streams ``world*B`` items per
    step with a :class:`blendtorch.btt.gpu.DeviceLoader` (or any iterable of
    batch dicts) and every rank receives its ``B``-item shard in HBM.

    Params
    ------
    source: iterable of dict batches on the root (ignored elsewhere); the
        image tensor must have leading dim ``world * B``.
    batch_size: per-rank B.
    shape, dtype: per-item image shape / dtype (identical on all ranks).
    num_batches: steps to deliver (all ranks must agree).
    """

    def __init__(self, source: Optional[Iterable], batch_size: int, shape: Sequence[int], dtype: torch.dtype,
                 device: torch.device, num_batches: int, image_key: str = 'image', src: int = 0):
        self.source = source
        self.batch_size = batch_size
        self.shape = tuple(shape)
        self.dtype = dtype
        self.device = device
        self.num_batches = num_batches
        self.image_key = image_key
        self.src = src

    def __len__(self):
        return self.num_batches

    def __iter__(self):
        rank, world, _ = rank_world()
        it = iter(self.source) if rank == self.src else None
        B = self.batch_size
        for _ in range(self.num_batches):
            full, metas = None, None
            if rank == self.src:
                batch = next(it)
                full = batch[self.image_key]
                metas = [{k: (v[r * B:(r + 1) * B] if hasattr(v, '__getitem__') and not isinstance(v, str) else v)
                          for k, v in batch.items() if k != self.image_key} for r in range(world)]
            img = scatter_batch(full, (B,) + self.shape, self.dtype, self.device, self.src)
            meta = {}
            if world > 1:
                box = [None]
                dist.scatter_object_list(box, metas if rank == self.src else None, src=self.src)
                meta = box[0]
            elif metas:
                meta = metas[0]
            yield {self.image_key: img, **meta}
