"""Registers blendtorch-cartpole-v0 (reference: examples/control/cartpole_gym/
__init__.py:3-6).  ``btt.env.register`` also registers with gym when gym is
installed, so both ``gym.make`` and ``btt.env.make`` work."""
from blendtorch import btt

btt.env.register('blendtorch-cartpole-v0', 'cartpole_gym.envs:CartpoleEnv')
