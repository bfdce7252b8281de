"""Launch and tear down producer instances (Blender or headless stand-ins).

Reference: pkg_pytorch/blendtorch/btt/launcher.py:15-197.  The command-line
contract handed to every instance is identical:

    <exe> [scene] [--background] --python-use-system-env --python <script> --
        -btid <i> -btseed <seed+i> -btsockets NAME=proto://addr:port ... <instance args>

Addresses are allocated socket-major: for each named socket, ``num_instances``
consecutive ports starting at ``start_port`` (``:104-107``); seeds are
``seed + i`` with a random base when ``seed`` is None (``:109-112``).

Differences (deliberate):

* ``producer=`` runs a headless producer instead of Blender: a native
  stand-in by name (``'cubesim'``, ``'cartpolesim'``, ``'supershapesim'``),
  ``'python'`` (run ``script`` with this interpreter), or any executable path.
  The launch arguments are the same, so scripts/stand-ins are interchangeable.
* Each instance gets its own process group (the reference built the
  ``setsid`` kwargs but never passed them, ``:124-132``), so ``__exit__``
  tears down whole process trees.
* ``cpu_affinity`` pins instance i to a CPU set -- producers are CPU-bound
  and per-GPU ranks partition the node's cores.
* ``respawn=True`` restarts instances that die (the reference never
  respawns; PUSH/PULL simply rebalances over the survivors).
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np

from .finder import discover_blender
from .launch_info import LaunchInfo
from .utils import get_primary_ip

logger = logging.getLogger('blendtorch')

NATIVE_PRODUCERS = ('cubesim', 'cartpolesim', 'supershapesim')


def producer_path(name):
    """Absolute path of a bundled native producer executable."""
    p = Path(__file__).resolve().parent.parent / 'bin' / name
    if not p.exists():
        raise FileNotFoundError(f'native producer {name!r} not built ({p}); run `python -m blendtorch._build`')
    return p


class BlenderLauncher:
    """Context manager that launches ``num_instances`` producer processes.

    Params mirror the reference (scene, script, num_instances, named_sockets,
    start_port, bind_addr, instance_args, proto, blend_path, seed, background)
    plus ``producer``, ``cpu_affinity``, ``respawn``, ``env``, ``shm_slots``
    and ``stdout``/``stderr`` (passed to Popen).

    ``shm_slots > 0`` opts every instance into the same-host shared-memory
    frame ring (``BLENDTORCH_SHM_SLOTS`` in the children's environment: a
    scene script's ``btb.DataPublisher`` and the native producers pick it
    up without code changes).  Only for consumers on this host.
    ``shm_codec='tile16'`` (``BLENDTORCH_SHM_CODEC``) additionally sends the
    ring frames as key-frame deltas (only changed 16x16 tiles).

    Attributes
    ----------
    launch_info: LaunchInfo
        Available inside the ``with`` block.
    """

    def __init__(self, scene=None, script=None, num_instances=1, named_sockets=None, start_port=11000,
                 bind_addr='127.0.0.1', instance_args=None, proto='tcp', blend_path=None, seed=None,
                 background=False, producer=None, cpu_affinity=None, respawn=False, env=None, stdout=None,
                 stderr=None, shm_slots=0, shm_codec=None):
        assert num_instances > 0
        self.num_instances = num_instances
        self.start_port = start_port
        self.bind_addr = bind_addr
        self.proto = proto
        self.scene = scene
        self.script = script
        self.blend_path = blend_path
        self.named_sockets = list(named_sockets) if named_sockets else []
        self.seed = seed
        self.background = background
        self.instance_args = instance_args if instance_args is not None else [[] for _ in range(num_instances)]
        assert len(self.instance_args) == num_instances
        self.producer = producer
        self.cpu_affinity = cpu_affinity
        if cpu_affinity is not None:
            assert len(cpu_affinity) == num_instances
        self.respawn = respawn
        self.env = dict(env or {})
        if shm_slots:
            self.env['BLENDTORCH_SHM_SLOTS'] = int(shm_slots)
        if shm_codec:
            self.env['BLENDTORCH_SHM_CODEC'] = str(shm_codec)
        self.stdout = stdout
        self.stderr = stderr

        if producer is None:
            self.blender_info = discover_blender(self.blend_path)
            if self.blender_info is None:
                logger.warning('Launching Blender failed;')
                raise ValueError('Blender not found or misconfigured.')
            logger.info(f'Blender found {self.blender_info["path"]} version '
                        f'{self.blender_info["major"]}.{self.blender_info["minor"]}')
        else:
            self.blender_info = None
            if producer not in NATIVE_PRODUCERS and producer != 'python':
                if not Path(producer).exists():
                    raise ValueError(f'producer executable {producer!r} not found')
        self.launch_info = None
        self._cmds = None
        self._monitor = None
        self._monitor_stop = threading.Event()
        self.respawn_count = 0

    # -- command construction ------------------------------------------------
    def _address_generator(self, proto, bind_addr, start_port):
        if bind_addr == 'primaryip':
            bind_addr = get_primary_ip()
        port = start_port
        while True:
            if proto == 'ipc':
                yield f'ipc:///tmp/blendtorch-{os.getpid()}-{port}'
            else:
                yield f'{proto}://{bind_addr}:{port}'
            port += 1

    def _base_cmd(self):
        if self.producer is None:
            cmd = [str(self.blender_info['path'])]
            if self.scene is not None and len(str(self.scene)) > 0:
                cmd.append(str(self.scene))
            if self.background:
                cmd.append('--background')
            cmd += ['--python-use-system-env', '--python', str(self.script)]
            return cmd
        if self.producer == 'python':
            return [sys.executable, str(self.script)]
        if self.producer in NATIVE_PRODUCERS:
            return [str(producer_path(self.producer))]
        return [str(self.producer)]

    def _spawn(self, idx):
        cmd = self._cmds[idx]
        cpus = self.cpu_affinity[idx] if self.cpu_affinity is not None else None

        def preexec():  # runs in the child between fork and exec
            os.setsid()
            if cpus:
                try:
                    os.sched_setaffinity(0, set(cpus))
                except OSError:
                    pass

        env = os.environ.copy()
        if self.env:
            env.update({k: str(v) for k, v in self.env.items()})
        pkg_root = str(Path(__file__).resolve().parent.parent.parent)
        env['PYTHONPATH'] = pkg_root + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
        kwargs = {'preexec_fn': preexec} if os.name == 'posix' else \
            {'creationflags': subprocess.CREATE_NEW_PROCESS_GROUP}
        p = subprocess.Popen(cmd, shell=False, stdin=None, stdout=self.stdout, stderr=self.stderr, env=env, **kwargs)
        logger.info(f'Started instance: {cmd}')
        return p

    # -- context manager -------------------------------------------------------
    def __enter__(self):
        assert self.launch_info is None, 'Already launched.'
        addresses = {}
        gen = self._address_generator(self.proto, self.bind_addr, self.start_port)
        for s in self.named_sockets:
            addresses[s] = [next(gen) for _ in range(self.num_instances)]

        seed = self.seed
        if seed is None:
            seed = np.random.randint(np.iinfo(np.int32).max - self.num_instances)
        seeds = [seed + i for i in range(self.num_instances)]

        base = self._base_cmd()
        self._cmds = []
        for idx in range(self.num_instances):
            args = ['-btid', str(idx), '-btseed', str(seeds[idx]), '-btsockets']
            args += [f'{k}={v[idx]}' for k, v in addresses.items()]
            args += [str(a) for a in self.instance_args[idx]]
            self._cmds.append(base + ['--'] + args)
        processes = [self._spawn(i) for i in range(self.num_instances)]
        self.launch_info = LaunchInfo(addresses, [' '.join(c) for c in self._cmds], processes=processes)
        if self.respawn:
            self._monitor_stop.clear()
            self._monitor = threading.Thread(target=self._monitor_loop, daemon=True)
            self._monitor.start()
        return self

    def _monitor_loop(self):
        while not self._monitor_stop.wait(0.25):
            self.respawn_dead()

    def respawn_dead(self):
        """Restart every instance that has exited; returns how many."""
        if self.launch_info is None:
            return 0
        n = 0
        for i, p in enumerate(self.launch_info.processes):
            if p.poll() is not None:
                logger.warning(f'instance {i} exited with {p.returncode}; respawning')
                from ..transport.shm import cleanup_pid
                cleanup_pid(p.pid)   # its shm ring (consumers keep their mappings until they let go)
                self.launch_info.processes[i] = self._spawn(i)
                n += 1
        self.respawn_count += n
        return n

    def assert_alive(self):
        """Assert that every launched process is still running."""
        if self.launch_info is None:
            return
        codes = self._poll()
        assert all(c is None for c in codes), f'Alive test failed. Exit codes {codes}'

    def wait(self):
        """Block until every launched process has exited."""
        for p in self.launch_info.processes:
            p.wait()

    def __exit__(self, exc_type, exc_value, exc_traceback):
        self._monitor_stop.set()
        if self._monitor is not None:
            self._monitor.join()
            self._monitor = None
        procs = self.launch_info.processes
        for p in procs:
            if p.poll() is None:
                try:
                    if os.name == 'posix':
                        os.killpg(p.pid, signal.SIGTERM)
                    else:
                        p.terminate()
                except (ProcessLookupError, PermissionError):
                    pass
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL) if os.name == 'posix' else p.kill()
                except (ProcessLookupError, PermissionError):
                    pass
                p.wait()
        assert all(c is not None for c in self._poll()), 'Not all Blender instances closed.'
        from ..transport.shm import cleanup_pid
        for p in procs:   # shared-memory rings of killed producers
            cleanup_pid(p.pid)
        self.launch_info = None
        logger.info('Blender instances closed')

    def _poll(self):
        return [p.poll() for p in self.launch_info.processes]
