#!/usr/bin/env python
"""Config 5: cart-pole RemoteEnv step rate with E parallel envs, observations
staged in HBM and a batched policy on the GPU.

Reference claim: "2000 Hz easily achieved" for one env without image transfer
(Readme.md:95).  Each step: the E envs get their actions (one fan-out of
REQ sends), reply after simulating one frame (one fan-in), observations are
packed into a pinned buffer and copied to the device in one transfer, the
P-controller policy (examples/control/cartpole.py:17-36) runs on the device.

    python benchmarks/bench_rl.py [--envs 8] [--steps 5000] [--device cuda|cpu]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / 'pytorch-blender_amd'))

import torch

from blendtorch import btt
from blendtorch.btt.env import VectorRemoteEnv
from blendtorch.models import CartpolePolicy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=8)
    ap.add_argument('--steps', type=int, default=5000)
    ap.add_argument('--warmup', type=int, default=200)
    ap.add_argument('--device', default='cuda' if torch.cuda.is_available() else 'cpu')
    ap.add_argument('--start-port', type=int, default=24000)
    ap.add_argument('--render-every', type=int, default=0)
    ap.add_argument('--python-client', action='store_true', help='use the pure-Python REQ clients')
    ap.add_argument('--proto', choices=['tcp', 'ipc'], default='tcp', help='tcp (as the reference) or ipc (same host)')
    ap.add_argument('--io-threads', type=int, default=0, help='native client IO threads (0: one per 4 envs)')
    a = ap.parse_args()
    dev = torch.device(a.device)
    args = dict(producer='cartpolesim', num_instances=a.envs, named_sockets=['GYM'], start_port=a.start_port, proto=a.proto,
                seed=7, instance_args=[['--render-every', str(a.render_every)]] * a.envs)
    with btt.BlenderLauncher(**args) as bl:
        venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'], device=dev, native=not a.python_client,
                               io_threads=a.io_threads)
        policy = CartpolePolicy().to(dev)
        obs, _ = venv.reset()
        episodes = 0

        def step(obs):
            nonlocal episodes
            act = policy(obs)
            obs, rew, done, infos = venv.step(act)
            if bool(done.any()):
                # reset only the finished envs (one concurrent round)
                idx = torch.nonzero(done).flatten().tolist()
                o, _ = venv.reset(which=idx)
                obs[idx] = o.to(obs.device)
                episodes += len(idx)
            return obs

        for _ in range(a.warmup):
            obs = step(obs)
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            obs = step(obs)
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        venv.close()
    print(json.dumps({'metric': 'cartpole env steps/s (aggregate)', 'value': round(a.envs * a.steps / dt, 1),
                      'unit': 'steps/s', 'envs': a.envs, 'steps': a.steps, 'per_env_hz': round(a.steps / dt, 1),
                      'ms_per_step': round(dt / a.steps * 1e3, 4), 'device': str(dev), 'episodes': episodes,
                      'client': 'python' if a.python_client else 'native', 'proto': a.proto, 'io_threads': a.io_threads,
                      'baseline': '2000 Hz (1 env, reference Readme.md:95)'}))


if __name__ == '__main__':
    main()
