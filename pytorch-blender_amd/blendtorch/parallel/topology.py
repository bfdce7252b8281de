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
from typing import Dict, List, Optional, Sequence

SYSFS_PCI = Path('/sys/bus/pci/devices')

__all__ = ['parse_cpulist', 'gpu_pci_bus_id', 'pci_local_cpus', 'plan_rank_cpus']


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
