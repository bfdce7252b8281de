"""Self-launch of one process per GPU (``python bench.py --gpus N``).

The driver may start a program either as N torchrun ranks (``WORLD_SIZE`` set
in the environment) or as a single process asked for N GPUs.  In the second
case the parent must become a pure supervisor: it may not touch the GPU (a
process that initialised HIP must never be replaced by another program on
this pool, and the children need the devices to themselves), so it

1. counts the visible devices in a throw-away child (``torch.cuda.device_count``
   honours ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``),
2. picks a free rendezvous port on 127.0.0.1,
3. starts N children with torchrun's environment contract (``RANK``,
   ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR``,
   ``MASTER_PORT``), each in its own session so a whole rank (and the
   producer processes it launched) can be torn down as a group,
4. relays their output (children share the parent's stdout, so rank 0's
   JSON line reaches the caller unchanged; each rank's stderr is relayed
   line by line and its tail kept),
5. returns the worst exit code.  If one rank fails the others are stopped
   after ``grace_s`` (a rank blocked in a collective on a dead peer would
   otherwise hang until the RCCL timeout), and
6. prints, for every rank that failed, its exit status and the last lines
   of its stderr in one block -- with 8 ranks interleaving their logs, the
   failing rank's traceback is otherwise hard to find.

The reference has no GPU ranks at all; its only scale axis is the number of
Blender instances a single consumer process launches
(pkg_pytorch/blendtorch/btt/launcher.py:104-157, benchmarks/benchmark.py:8).
"""
from __future__ import annotations

import collections
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence

__all__ = ['visible_gpu_count', 'free_port', 'rank_env', 'spawn_ranks', 'worst_rc', 'failure_report']


def visible_gpu_count(timeout_s: float = 300.0) -> int:
    """Number of HIP devices a child process would see (0 when none / no torch).

    Runs in a separate interpreter so the calling process never initialises
    the GPU runtime (the first ``import torch`` on a fresh box can take a
    minute or two, hence the generous timeout)."""
    code = 'import torch; print(torch.cuda.device_count() if torch.cuda.is_available() else 0)'
    try:
        r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=timeout_s)
    except (OSError, subprocess.TimeoutExpired):
        return 0
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def free_port(host: str = '127.0.0.1') -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None,
             addr: str = '127.0.0.1') -> Dict[str, str]:
    """Environment of one single-node rank (torchrun's variable names)."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK='0', NODE_RANK='0', MASTER_ADDR=addr, MASTER_PORT=str(port))
    # dmabuf IPC is the only mode this host driver supports (RCCL / tensor sharing)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return env


def worst_rc(codes: Sequence[Optional[int]]) -> int:
    """Exit status for the job: the first failing rank's code (signals map to
    128+sig like a shell does), 0 only if every rank succeeded."""
    worst = 0
    for c in codes:
        if c is None:
            c = 1
        if c < 0:
            c = 128 - c
        if c != 0 and worst == 0:
            worst = c
    return worst


def _kill_group(p: subprocess.Popen, sig: int):
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _relay(stream, sink, tail: collections.deque):
    """Copy a rank's stderr to ours line by line, keeping its last lines."""
    for raw in iter(stream.readline, b''):
        tail.append(raw.decode('utf-8', 'replace').rstrip('\n'))
        try:
            sink.write(raw)
            sink.flush()
        except (OSError, ValueError):
            pass
    stream.close()


def failure_report(codes: Sequence[Optional[int]], tails: Sequence[Sequence[str]], first: Optional[int] = None) -> str:
    """Text block naming every failed rank with the tail of its stderr
    (the rank that failed first is marked: later ones were usually stopped)."""
    out = []
    for r, (c, tail) in enumerate(zip(codes, tails)):
        if c in (0, None):
            continue
        sig = f' (signal {-c})' if c < 0 else ''
        mark = ' [failed first]' if r == first else ''
        out.append(f'[launch] rank {r} exited with {c}{sig}{mark}; last {len(tail)} stderr lines:')
        out.extend(f'[launch]   rank {r}| {line}' for line in tail)
    return '\n'.join(out)


def spawn_ranks(cmd: Sequence[str], world: int, port: Optional[int] = None, grace_s: float = 30.0,
                timeout_s: Optional[float] = None, env: Optional[Dict[str, str]] = None,
                poll_s: float = 0.1, tail_lines: int = 25, report=None):
    """Run ``cmd`` as ``world`` ranks on this node and wait for all of them.

    Returns ``(codes, rc)``: the per-rank exit codes and the job's exit status
    (the code of the rank that failed FIRST -- ranks stopped afterwards report
    SIGTERM, which would hide the cause -- or 124 on ``timeout_s``).  When a rank exits non-zero (or
    ``timeout_s`` passes) the remaining ranks receive SIGTERM, then SIGKILL
    ``grace_s`` later; every rank runs in its own session and is signalled as
    a process group.  Each rank's stderr is relayed to ours; the last
    ``tail_lines`` of every failed rank are printed together at the end
    (to ``report``, default ``sys.stderr``)."""
    port = port or free_port()
    procs = [subprocess.Popen(list(cmd), env=rank_env(r, world, port, env), start_new_session=True,
                              stderr=subprocess.PIPE)
             for r in range(world)]
    tails = [collections.deque(maxlen=tail_lines) for _ in range(world)]
    sink = getattr(sys.stderr, 'buffer', None) or sys.stderr
    relays = [threading.Thread(target=_relay, args=(p.stderr, sink, t), daemon=True) for p, t in zip(procs, tails)]
    for t in relays:
        t.start()
    codes: List[Optional[int]] = [None] * world
    t0 = time.monotonic()
    term_at = None
    rc = 0
    first = None
    try:
        while any(c is None for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    codes[i] = p.poll()
                    if codes[i] not in (None, 0) and rc == 0:
                        rc = worst_rc([codes[i]])
                        first = i
            failed = rc != 0
            late = timeout_s is not None and time.monotonic() - t0 > timeout_s
            if late and rc == 0:
                rc = 124
            if (failed or late) and term_at is None and any(c is None for c in codes):
                term_at = time.monotonic()
                for i, p in enumerate(procs):
                    if codes[i] is None:
                        _kill_group(p, signal.SIGTERM)
            if term_at is not None and time.monotonic() - term_at > grace_s:
                for i, p in enumerate(procs):
                    if codes[i] is None:
                        _kill_group(p, signal.SIGKILL)
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            _kill_group(p, signal.SIGTERM)
        for p in procs:
            try:
                p.wait(grace_s)
            except subprocess.TimeoutExpired:
                _kill_group(p, signal.SIGKILL)
        raise
    for t in relays:
        t.join(5)
    if rc:
        text = failure_report(codes, [list(t) for t in tails], first)
        if rc == 124 and first is None:
            text = f'[launch] timed out after {timeout_s} s\n' + text
        print(text, file=report or sys.stderr, flush=True)
    return codes, rc
