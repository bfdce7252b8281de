#!/usr/bin/env python
"""Cart-pole P-controller driving a remote environment (reference:
examples/control/cartpole.py).  The env runs in Blender (cartpole.blend) when
available, else in the native `cartpolesim` stand-in; the gym-style wrapper
is cartpole_gym.envs.CartpoleEnv (registered as blendtorch-cartpole-v0 when
gym is installed).

    python cartpole.py [--steps 2000] [--real-time]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'pytorch-blender_amd'))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import cartpole_gym  # noqa: E402,F401  (registers blendtorch-cartpole-v0)
from blendtorch import btt  # noqa: E402

KAPPA = 30


def control(obs):
    # P controller on the error x_pole - x_cart
    xcart, xpole, _ = obs
    return (xpole - xcart) * KAPPA


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--real-time', action='store_true')
    a = ap.parse_args()
    env = btt.env.make('blendtorch-cartpole-v0', real_time=a.real_time)
    obs = env.reset()
    episodes, length, lengths = 0, 0, []
    for _ in range(a.steps):
        obs, reward, done, info = env.step(control(obs))
        length += 1
        if done:
            obs = env.reset()
            episodes += 1
            lengths.append(length)
            length = 0
    env.close()
    print(f'{a.steps} steps, {episodes} episodes, mean episode length '
          f'{(sum(lengths) / len(lengths)) if lengths else length:.1f}')


if __name__ == '__main__':
    main()
