"""pyzmq-compatible API over blendtorch's native ZMTP engine.

The reference drives every message through pyzmq (see SURVEY.md §2.6 for the
17 call sites).  pyzmq/libzmq are not part of this stack, so this module offers
the subset of the pyzmq surface the btt/btb packages (and user code written
against them) need: ``Context``, ``Socket`` (``setsockopt``, ``bind``,
``connect``, ``send*/recv*`` incl. ``*_pyobj``, ``poll``, ``close``),
``Poller``, the error classes (``Again``, ``ZMQError``) and the constants.
Wire format is ZMTP/3.0, so these sockets interoperate with libzmq peers.

Differences from pyzmq worth knowing:
* all Contexts of a process share one native IO thread (a forked child gets
  its own; sockets inherited across fork are parked, never used);
* ``recv_pyobj`` decodes simple dict/ndarray messages with the native
  zero-copy codec (ndarray values are writable views on the received frame);
  anything else falls back to :func:`pickle.loads`.  Set
  ``BLENDTORCH_FAST_UNPICKLE=0`` to always use :mod:`pickle`.
"""
from __future__ import annotations

import atexit
import json
import os
import pickle
import threading
import weakref

from .. import _native

# --- constants (numeric values identical to libzmq / pyzmq) -----------------
PAIR, PUB, SUB, REQ, REP, DEALER, ROUTER, PULL, PUSH = range(9)
IDENTITY = ROUTING_ID = 5
RCVMORE = 13
TYPE = 16
LINGER = 17
RECONNECT_IVL = 18
SNDHWM = 23
RCVHWM = 24
HWM = 201  # pseudo option: sets both
RCVTIMEO = 27
SNDTIMEO = 28
LAST_ENDPOINT = 32
IMMEDIATE = 39
REQ_CORRELATE = 52
REQ_RELAXED = 53
# blendtorch extensions
BT_SNDBUF_KB = 1001
BT_RCVBUF_KB = 1002
BT_ALLOC_THRESHOLD = 1003

NOBLOCK = DONTWAIT = 1
SNDMORE = 2
POLLIN = 1
POLLOUT = 2

EINTR = 4
EAGAIN = 11
EINVAL = 22
EFSM = 156384763
ETERM = 156384765

DEFAULT_PROTOCOL = pickle.DEFAULT_PROTOCOL

_FAST_UNPICKLE = os.environ.get('BLENDTORCH_FAST_UNPICKLE', '1') != '0'


class ZMQBaseError(Exception):
    pass


class ZMQError(ZMQBaseError):
    def __init__(self, errno=None, msg=None):
        self.errno = errno
        self.strerror = msg or ''
        super().__init__(msg)

    def __str__(self):
        return self.strerror


class Again(ZMQError):
    pass


class ContextTerminated(ZMQError):
    pass


class InterruptedSystemCall(ZMQError, InterruptedError):
    pass


class _ErrorNamespace:
    ZMQBaseError = ZMQBaseError
    ZMQError = ZMQError
    Again = Again
    ContextTerminated = ContextTerminated
    InterruptedSystemCall = InterruptedSystemCall


error = _ErrorNamespace()


def _translate(e):
    code = getattr(e, 'errno', None)
    if code == EAGAIN:
        return Again(code, 'Resource temporarily unavailable')
    if code == ETERM:
        return ContextTerminated(code, str(e))
    if code == EINTR:
        return InterruptedSystemCall(code, str(e))
    return ZMQError(code, str(e))


def _call(fn, *args):
    try:
        return fn(*args)
    except _native.NativeError as e:
        raise _translate(e) from None


class Frame:
    """A received message part (zero-copy view on the native buffer)."""

    __slots__ = ('_f', 'more')

    def __init__(self, f, more=False):
        self._f = f
        self.more = more

    @property
    def bytes(self):
        return self._f.bytes

    @property
    def buffer(self):
        return memoryview(self._f)

    def __len__(self):
        return len(self._f)

    def __bytes__(self):
        return self._f.bytes


_live_sockets = weakref.WeakSet()
_live_lock = threading.Lock()


class Socket:
    def __init__(self, context, socket_type):
        self.context = context
        self._sock = _call(context._native.socket, socket_type)
        self.socket_type = socket_type
        self._closed = False
        self._send_parts = []
        self._recv_parts = []
        self._rcvmore = False
        with _live_lock:
            _live_sockets.add(self)
        context._sockets.add(self)

    # -- options ---------------------------------------------------------
    def setsockopt(self, opt, value):
        if opt == HWM:
            self.setsockopt(SNDHWM, value)
            self.setsockopt(RCVHWM, value)
            return
        if isinstance(value, (bytes, str)):
            v = value.encode() if isinstance(value, str) else value
            _call(self._sock.setsockopt_bytes, opt, v)
        else:
            _call(self._sock.setsockopt, opt, int(value))

    set = setsockopt

    def getsockopt(self, opt):
        if opt == RCVMORE:
            return int(self._rcvmore)
        if opt in (LAST_ENDPOINT, IDENTITY):
            return _call(self._sock.getsockopt_string, opt).encode()
        return _call(self._sock.getsockopt, opt)

    get = getsockopt

    def setsockopt_string(self, opt, value, encoding='utf-8'):
        self.setsockopt(opt, value.encode(encoding))

    def getsockopt_string(self, opt, encoding='utf-8'):
        return self.getsockopt(opt).decode(encoding)

    def _opt_property(opt):  # noqa: N805
        return property(lambda self: self.getsockopt(opt), lambda self, v: self.setsockopt(opt, v))

    linger = _opt_property(LINGER)
    sndhwm = _opt_property(SNDHWM)
    rcvhwm = _opt_property(RCVHWM)
    sndtimeo = _opt_property(SNDTIMEO)
    rcvtimeo = _opt_property(RCVTIMEO)
    immediate = _opt_property(IMMEDIATE)
    hwm = property(lambda self: self.getsockopt(SNDHWM), lambda self, v: self.setsockopt(HWM, v))
    last_endpoint = property(lambda self: self.getsockopt(LAST_ENDPOINT))

    @property
    def type(self):
        return self.socket_type

    # -- topology --------------------------------------------------------
    def bind(self, addr):
        return _call(self._sock.bind, addr)

    def bind_to_random_port(self, addr, min_port=49152, max_port=65536, max_tries=100):
        ep = self.bind(f'{addr}:*')
        return int(ep.rsplit(':', 1)[1])

    def connect(self, addr):
        _call(self._sock.connect, addr)

    def unbind(self, addr):
        _call(self._sock.unbind, addr)

    def disconnect(self, addr):
        _call(self._sock.disconnect, addr)

    # -- send ------------------------------------------------------------
    def send(self, data, flags=0, copy=True, track=False, **kwargs):
        if isinstance(data, str):
            raise TypeError('str objects cannot be sent; use send_string')
        if isinstance(data, Frame):
            data = data._f
        self._send_parts.append(data)
        if flags & SNDMORE:
            return None
        parts, self._send_parts = self._send_parts, []
        try:
            _call(self._sock.send_multipart, parts, flags & ~SNDMORE)
        except Exception:
            raise
        return None

    def send_multipart(self, msg_parts, flags=0, copy=True, track=False, **kwargs):
        parts = [p._f if isinstance(p, Frame) else p for p in msg_parts]
        _call(self._sock.send_multipart, parts, flags)

    def send_pyobj(self, obj, flags=0, protocol=DEFAULT_PROTOCOL, **kwargs):
        return self.send(pickle.dumps(obj, protocol), flags)

    def send_string(self, u, flags=0, copy=True, encoding='utf-8', **kwargs):
        return self.send(u.encode(encoding), flags)

    def send_json(self, obj, flags=0, **kwargs):
        return self.send(json.dumps(obj).encode('utf-8'), flags)

    # -- recv ------------------------------------------------------------
    def _next_frame(self, flags):
        if not self._recv_parts:
            parts = _call(self._sock.recv_multipart, flags)
            self._recv_parts = list(parts)
        f = self._recv_parts.pop(0)
        self._rcvmore = bool(self._recv_parts)
        return f

    def recv(self, flags=0, copy=True, track=False):
        f = self._next_frame(flags)
        if copy:
            return f.bytes
        return Frame(f, self._rcvmore)

    def recv_multipart(self, flags=0, copy=True, track=False):
        if self._recv_parts:
            parts, self._recv_parts = self._recv_parts, []
        else:
            parts = _call(self._sock.recv_multipart, flags)
        self._rcvmore = False
        if copy:
            return [p.bytes for p in parts]
        return [Frame(p, p.more) for p in parts]

    def recv_pyobj(self, flags=0):
        f = self._next_frame(flags)
        return loads(f)

    def recv_string(self, flags=0, encoding='utf-8'):
        return self.recv(flags).decode(encoding)

    def recv_json(self, flags=0, **kwargs):
        return json.loads(self.recv(flags).decode('utf-8'))

    # -- misc ------------------------------------------------------------
    def poll(self, timeout=None, flags=POLLIN):
        t = -1 if timeout is None else int(timeout)
        return _call(_native.poll, [(self._sock, flags)], t)[0]

    @property
    def closed(self):
        return self._closed

    def close(self, linger=None):
        if self._closed:
            return
        self._closed = True
        lg = -2 if linger is None else int(linger)
        try:
            self._sock.close(lg)
        except Exception:
            pass

    def stats(self):
        return self._sock.stats()

    def num_peers(self):
        return self._sock.num_peers()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            if not self._closed:
                self.close()
        except Exception:
            pass


def loads(frame):
    """Unpickle a received frame (zero-copy fast path when possible)."""
    if _FAST_UNPICKLE:
        try:
            return _native.fast_loads(frame)
        except ValueError:
            pass
    return pickle.loads(memoryview(frame))


# --- fork safety -------------------------------------------------------------
# The native engine runs an IO thread per context; threads do not survive
# fork().  DataLoader workers fork, so every process lazily gets its own
# native context, and sockets inherited from the parent are parked (never
# closed or destroyed in the child: their context's IO thread does not exist
# there, and the parent still owns the connections).
_proc_ctx = None
_proc_pid = None
_inherited = []


def _process_context():
    global _proc_ctx, _proc_pid
    pid = os.getpid()
    if _proc_pid != pid:
        _proc_ctx = _native.global_context() if _proc_pid is None and pid == _MAIN_PID else _native.Context()
        _proc_pid = pid
    return _proc_ctx


def _after_fork_in_child():
    global _live_sockets, _proc_pid
    with _live_lock:
        _inherited.extend(_live_sockets)
        _live_sockets = weakref.WeakSet()
    _proc_pid = -1


_MAIN_PID = os.getpid()
if hasattr(os, 'register_at_fork'):
    os.register_at_fork(after_in_child=_after_fork_in_child)


class Context:
    _instance = None

    def __init__(self, io_threads=1, **kwargs):
        self._native = _process_context()
        self._sockets = weakref.WeakSet()
        self.closed = False

    @classmethod
    def instance(cls, io_threads=1):
        if cls._instance is None or cls._instance._pid != os.getpid():
            cls._instance = cls(io_threads)
        return cls._instance

    @property
    def _pid(self):
        return _proc_pid

    def socket(self, socket_type, **kwargs):
        if self.closed:
            raise ContextTerminated(ETERM, 'Context was terminated')
        return Socket(self, socket_type)

    def term(self):
        for s in list(self._sockets):
            s.close()
        self.closed = True

    def destroy(self, linger=None):
        for s in list(self._sockets):
            s.close(linger)
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.term()


class Poller:
    def __init__(self):
        self.sockets = []

    def register(self, socket, flags=POLLIN | POLLOUT):
        for i, (s, _) in enumerate(self.sockets):
            if s is socket:
                if flags:
                    self.sockets[i] = (socket, flags)
                else:
                    del self.sockets[i]
                return
        if flags:
            self.sockets.append((socket, flags))

    modify = register

    def unregister(self, socket):
        self.sockets = [(s, f) for s, f in self.sockets if s is not socket]

    def poll(self, timeout=None):
        if not self.sockets:
            return []
        t = -1 if timeout is None else int(timeout)
        # sockets with already-buffered multipart frames are readable
        res = _call(_native.poll, [(s._sock, f) for s, f in self.sockets], t)
        out = []
        for (s, f), r in zip(self.sockets, res):
            if s._recv_parts and (f & POLLIN):
                r |= POLLIN
            if r:
                out.append((s, r))
        return out


def _close_all_at_exit():
    # Honour each socket's LINGER so queued messages are flushed before exit,
    # the way libzmq's context termination does.
    with _live_lock:
        socks = list(_live_sockets)
    for s in socks:
        try:
            s.close()
        except Exception:
            pass


atexit.register(_close_all_at_exit)

zmq_version = lambda: 'blendtorch-native-zmtp3.0'  # noqa: E731
pyzmq_version = zmq_version
