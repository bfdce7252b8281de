"""Multicast callbacks (reference: pkg_blender/blendtorch/btb/signal.py:3-53).

    >>> sig = Signal()
    >>> h = sig.add(print, 'value:')
    >>> sig.invoke(3)
    value: 3
    >>> sig.remove(h)
"""
from functools import partial


class Signal:
    """Ordered list of callbacks invoked together."""

    def __init__(self):
        self.slots = []

    def add(self, fn, *args, **kwargs):
        """Register ``fn`` with bound leading args/kwargs; returns a handle."""
        handle = partial(fn, *args, **kwargs)
        self.slots.append(handle)
        return handle

    def remove(self, handle):
        """Unregister a handle returned by :meth:`add`."""
        self.slots.remove(handle)

    def invoke(self, *args, **kwargs):
        """Call every registered callback (in registration order)."""
        for s in list(self.slots):
            s(*args, **kwargs)
