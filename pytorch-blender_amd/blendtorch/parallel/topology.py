"""Node topology for producer placement: which host CPUs sit next to which GPU.

On an 8x MI355X node the GPUs hang off two (or more) host NUMA domains. The
producers of one rank write every frame into host memory, and that rank's GPU
reads it back over its own PCIe link (the zero-copy decode path). The frames
should therefore live in DRAM attached to the GPU's root complex, written by
cores on the same socket. Crossing sockets doubles the host-memory traffic on
the inter-socket link and costs PCIe read bandwidth.

:func:`plan_rank_cpus` resolves each local rank's GPU to its PCI device
(``hipDeviceGetPCIBusId``), reads ``/sys/bus/pci/devices/<bdf>/local_cpulist``,
and splits every NUMA-local CPU set evenly between the ranks that share it.
When the topology is unknown (no sysfs, no GPU, an empty intersection with
the allowed CPUs) it falls back to a contiguous partition of the allowed CPUs.

The reference has no such notion: its producers are whatever processes the OS
schedules (pkg_pytorch/blendtorch/btt/launcher.py:137-161).
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

SYSFS_PCI = Path('/sys/bus/pci/devices')

__all__ = ['parse_cpulist', 'gpu_pci_bus_id', 'pci_local_cpus', 'plan_rank_cpus', 'plan_rank_resources']


def parse_cpulist(text: str) -> List[int]:
    """``'0-3,8,10-11'`` -> ``[0, 1, 2, 3, 8, 10, 11]`` (sysfs cpulist format)."""
    out: List[int] = []
    for part in text.strip().split(','):
        part = part.strip()
        if not part:
            continue
        if '-' in part:
            a, b = part.split('-', 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_pci_bus_id(index: int) -> Optional[str]:
    """PCI address (``dddd:bb:dd.f``, lower case) of HIP device ``index``, or
    None if the HIP extension / device is unavailable."""
    try:
        from .. import ops
        ext = ops.hip_ext()
        n = ext.device_count()
        return ext.pci_bus_id(int(index) % n).lower() if n > 0 else None
    except Exception:
        return None


def pci_local_cpus(bus_id: str, sysfs: Path = SYSFS_PCI) -> Optional[List[int]]:
    """CPUs local to a PCI device (its NUMA node), from sysfs."""
    try:
        return parse_cpulist((Path(sysfs) / bus_id / 'local_cpulist').read_text())
    except (OSError, ValueError):
        return None


def _contiguous(cpus: Sequence[int], i: int, n: int) -> List[int]:
    cpus = list(cpus)
    share = max(1, len(cpus) // max(1, n))
    return cpus[i * share:(i + 1) * share] or cpus


def plan_rank_cpus(local_rank: int, local_world: int, allowed: Sequence[int],
                   bus_ids: Optional[Sequence[Optional[str]]] = None, sysfs: Path = SYSFS_PCI) -> Dict[str, object]:
    """CPU slice for ``local_rank``'s producers.

    Params
    ------
    allowed: CPUs this job may use (affinity mask, trimmed to the cgroup quota).
    bus_ids: PCI address per local rank (default: queried from HIP for
        devices ``0..local_world-1``).

    Returns ``{'cpus': [...], 'numa_local': bool, 'domain': [...]}``. ``cpus``
    is this rank's exclusive slice. ``domain`` is the whole GPU-local set
    (intersected with ``allowed``), which suits a soft affinity when
    per-core pinning is not wanted. ``numa_local`` says whether the topology
    was resolved.
    """
    allowed = sorted(set(int(c) for c in allowed))
    if bus_ids is None:
        bus_ids = [gpu_pci_bus_id(r) for r in range(local_world)]
    allowed_set = set(allowed)
    domains = []
    for bid in bus_ids:
        local = pci_local_cpus(bid, sysfs) if bid else None
        dom = [c for c in (local or []) if c in allowed_set]
        domains.append(tuple(dom) if dom else None)
    if len(domains) != local_world or any(d is None for d in domains):
        return {'cpus': _contiguous(allowed, local_rank, local_world), 'numa_local': False, 'domain': allowed}
    mine = domains[local_rank]
    sharers = [r for r in range(local_world) if domains[r] == mine]
    j = sharers.index(local_rank)
    return {'cpus': _contiguous(mine, j, len(sharers)), 'numa_local': True, 'domain': list(mine)}


def current_allowed_cpus() -> List[int]:
    return sorted(os.sched_getaffinity(0))


# Measured CPU cost per delivered 640x480 RGBA frame on the headline path
# (bench.py, cubesim producers -> shm ring -> zero-copy decode, one MI355X;
# profiles/r4/cpu_per_frame.md: 62-67 us in the producers -- render with
# per-row dirty spans, 45 us of it -- and 19-21 us in the consumer process
# with the host-ordered loader hand-off; round 3 measured 100 + 44).
# bench.py reports the current values as ``cpu.us_per_frame`` on every run.
PRODUCER_US_PER_FRAME = 65.0
CONSUMER_US_PER_FRAME = 20.0
HEADLINE_FRAME_BYTES = 640 * 480 * 4
# Per-message part of those costs (pickle/descriptor, socket, scan, batch
# bookkeeping: independent of the pixel count); the rest scales with the
# frame's bytes.  Estimates, not measurements: for other frame sizes pass the
# measured ``cpu.us_per_frame`` of a bench run as producer_us / consumer_us.
PRODUCER_FIXED_US = 10.0
CONSUMER_FIXED_US = 10.0
# host->device read ceiling of one MI355X PCIe link (profiles/direct_host_read.md)
LINK_GBYTES_PER_S = 51.5


def frame_costs_us(frame_bytes: int = HEADLINE_FRAME_BYTES) -> Tuple[float, float]:
    """(producer, consumer) CPU microseconds per frame of ``frame_bytes``:
    the headline frame's measured costs, the per-message part fixed and the
    rest scaled by the frame size (exact at 640x480 RGBA)."""
    k = max(0, int(frame_bytes)) / HEADLINE_FRAME_BYTES
    return (PRODUCER_FIXED_US + (PRODUCER_US_PER_FRAME - PRODUCER_FIXED_US) * k,
            CONSUMER_FIXED_US + (CONSUMER_US_PER_FRAME - CONSUMER_FIXED_US) * k)


def producers_for_share(share: float, frame_bytes: int = HEADLINE_FRAME_BYTES,
                        producer_us: Optional[float] = None, consumer_us: Optional[float] = None,
                        link_gbytes: float = LINK_GBYTES_PER_S, cap: int = 8) -> int:
    """Producer processes one rank should run on ``share`` CPUs: the frame
    rate the rank can sustain is the smaller of its PCIe link's and its CPU
    share's (every frame costs ``producer_us`` in some producer and
    ``consumer_us`` in the rank's own process; default :func:`frame_costs_us`
    for this frame size); the producers need ``rate * producer_us`` cores of
    it, rounded up.  When the link is the bound a 1.5x margin keeps producers
    ahead of it (backpressure absorbs the surplus); when the CPU is, more
    producers would only steal the consumer's cores."""
    p_def, c_def = frame_costs_us(frame_bytes)
    producer_us = p_def if producer_us is None else float(producer_us)
    consumer_us = c_def if consumer_us is None else float(consumer_us)
    link_rate = link_gbytes * 1e9 / max(1, frame_bytes)
    cpu_rate = max(0.0, share) * 1e6 / (producer_us + consumer_us)
    rate = min(link_rate, cpu_rate)
    need = rate * producer_us / 1e6
    n = need * 1.5 if link_rate <= cpu_rate else need
    return int(max(1, min(cap, -(-n // 1))))


def plan_rank_resources(rank: int, local_rank: int, local_world: int, world: int, allowed: Sequence[int],
                        budget: int, pin: bool, producers: int = 0, dist_mode: str = 'shard', shm_slots: int = 48,
                        shm_free_bytes: Optional[int] = None, frame_bytes: int = 640 * 480 * 4,
                        named_sockets: int = 1, port_base: int = 21000, port_stride: int = 64,
                        bus_ids: Optional[Sequence[Optional[str]]] = None, sysfs: Path = SYSFS_PCI,
                        pid: Optional[int] = None, producer_us: Optional[float] = None,
                        consumer_us: Optional[float] = None) -> Dict[str, object]:
    """Everything one rank of ``bench.py`` claims on the node, decided without
    talking to the other ranks (so every rank computes the same, disjoint plan):

    * ``cpus``/``domain``/``numa_local``: :func:`plan_rank_cpus` over the CPUs
      the job may keep busy (``allowed`` trimmed to the cgroup ``budget`` when
      per-core pinning isolates anything, i.e. ``pin``);
    * ``producers``: producer processes this rank launches -- ``producers`` if
      given, else what the measured per-frame CPU costs justify on the rank's
      CPU share (:func:`producers_for_share`: 5 on 16 CPUs, where the PCIe
      link is the bound; 2 on the 2 CPUs a rank gets when 8 ranks share a
      16-CPU quota, where the CPU is).  Scatter mode spreads 8 producers over
      all ranks (the root's PCIe link is the bound);
    * ``affinity``: per-producer CPU lists (single cores when pinning, the
      GPU's NUMA domain otherwise, or None);
    * ``start_port``: ``port_base + rank * port_stride`` (the launcher takes
      ``producers`` consecutive ports per named socket), or a pid-derived base
      for a single rank so concurrent jobs rarely collide;
    * ``shm_slots``: ring slots per producer that fit 60 % of the free
      ``/dev/shm`` shared by every local rank's producers (0 = inline frames
      when fewer than 8 would fit).
    """
    plan = plan_rank_cpus(local_rank, local_world, list(allowed)[:budget] if pin else allowed, bus_ids, sysfs)
    share = max(1, budget // max(1, local_world))
    nprod = producers or producers_for_share(budget / max(1, local_world), frame_bytes, producer_us, consumer_us)
    if dist_mode == 'scatter' and not producers:
        nprod = max(1, -(-8 // max(1, world)))
    mine = plan['cpus']
    if pin:
        affinity = [[mine[i % len(mine)]] for i in range(nprod)]
    elif plan['numa_local']:
        affinity = [plan['domain']] * nprod
    else:
        affinity = None
    if world == 1:
        start_port = 20000 + ((os.getpid() if pid is None else pid) % 200) * 50
    else:
        start_port = port_base + rank * port_stride
    span = nprod * max(1, named_sockets)
    if span > port_stride and world > 1:
        raise ValueError(f'{nprod} producers x {named_sockets} sockets exceed the {port_stride}-port block per rank')
    slots = int(shm_slots)
    if slots > 0 and shm_free_bytes is not None:
        fit = int(0.6 * shm_free_bytes / max(1, frame_bytes * nprod * max(1, local_world)))
        slots = min(slots, fit) if fit >= 8 else 0
    return {'cpus': mine, 'domain': plan['domain'], 'numa_local': plan['numa_local'], 'share': share,
            'producers': nprod, 'affinity': affinity, 'start_port': start_port, 'port_span': span,
            'shm_slots': slots}
