"""PyTorch-side defaults (reference: pkg_pytorch/blendtorch/btt/constants.py:4)."""

#: Default socket timeout of the PyTorch side, in milliseconds.
DEFAULT_TIMEOUTMS = 10000
