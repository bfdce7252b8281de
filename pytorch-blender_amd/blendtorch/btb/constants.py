"""Blender-side defaults (reference: pkg_blender/blendtorch/btb/constants.py:4)."""

#: Default socket timeout of the Blender side, in milliseconds.
DEFAULT_TIMEOUTMS = 5000
