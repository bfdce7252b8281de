"""Gym-style environments of the cart-pole example.

``CartpoleEnv`` wraps the remote cart-pole simulation (Blender's
cartpole.blend, or the native ``cartpolesim`` stand-in) behind the
old-gym ``reset``/``step``/``render`` interface."""
from .cartpole_env import CartpoleEnv

__all__ = ['CartpoleEnv']
