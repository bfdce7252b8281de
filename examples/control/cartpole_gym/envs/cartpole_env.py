"""Gym-style cart-pole env backed by a remote simulation.

Reference: examples/control/cartpole_gym/envs/cartpole_env.py (which ignores
its ``render_every`` argument and always passes 10; here it is honoured).
With Blender available the env runs cartpole.blend.py inside Blender; else the
native cartpolesim stand-in serves the same protocol."""
from pathlib import Path

import numpy as np

from blendtorch import btt

try:
    from gym import spaces
except ImportError:  # spaces are informational only
    spaces = None


class CartpoleEnv(btt.env.OpenAIRemoteEnv):
    def __init__(self, render_every=10, real_time=False, launcher_args=None):
        super().__init__(version='0.0.1')
        here = Path(__file__).parent
        if btt.discover_blender() is not None:
            self.launch(scene=here / 'cartpole.blend', script=here / 'cartpole.blend.py',
                        real_time=real_time, render_every=render_every, launcher_args=launcher_args)
        else:
            self.launch(scene='', script='', producer='cartpolesim', real_time=real_time,
                        render_every=render_every, launcher_args=launcher_args)
        if spaces is not None:
            self.action_space = spaces.Box(np.float32(-100), np.float32(100), shape=(1,))
            self.observation_space = spaces.Box(np.float32(-10), np.float32(10), shape=(1,))
