"""Message transport selection.

``zmq`` resolves to blendtorch's native ZMTP engine (:mod:`.native_zmq`) by
default.  ``BLENDTORCH_TRANSPORT=pyzmq`` selects a real pyzmq installation
instead (useful inside a stock Blender that ships pyzmq); both speak the same
ZMTP wire protocol, so the two sides of a connection may differ.
"""
import os


def _resolve():
    choice = os.environ.get('BLENDTORCH_TRANSPORT', 'native').lower()
    if choice == 'pyzmq':
        import zmq as _zmq  # noqa: F401  (real pyzmq)
        return _zmq
    try:
        from . import native_zmq
        return native_zmq
    except ImportError:
        if choice == 'native':
            try:
                import zmq as _zmq
                return _zmq
            except ImportError:
                pass
        raise


zmq = _resolve()

__all__ = ['zmq']
