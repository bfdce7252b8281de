"""Independent wire-level oracles for the native ZMTP/3.x engine.

No libzmq / pyzmq exists in this environment, so interoperability is pinned
against a hand-written peer that speaks the wire format straight from the
ZMTP 3.0/3.1 RFCs (23/ZMTP, 37/ZMTP): 64-byte greeting, READY command with
metadata properties, 1-byte flags (MORE=1, LONG=2, COMMAND=4) with a 1- or
8-byte big-endian size.  It covers every direction the reference deploys:

* Blender's pyzmq PUSH -> our PULL (pkg_blender/blendtorch/btb/publisher.py:21-28):
  single, multipart (MORE) and long frames, greetings delivered in fragments
  (libzmq sends the 10-byte signature first) and as version 3.1;
* a REQ / DEALER peer -> our REP: the envelope is echoed byte-exact
  (pkg_blender/blendtorch/btb/env.py:209-252);
* our REQ with REQ_RELAXED + REQ_CORRELATE -> a REP peer: every request is
  [4-byte request id, empty delimiter, body], stale replies are dropped
  (pkg_pytorch/blendtorch/btt/env.py:34-45);
* PAIR both ways (btb/btt duplex.py);
* hostile peers (zero-size commands, 64-bit sizes) must not take the
  process down;
* pickles written by CPython with protocols 2/4/5 and the numpy-1.x module
  path ``numpy.core.multiarray`` (what Blender's bundled numpy writes).
"""
import pickle
import socket
import struct
import threading
import time

import numpy as np
import pytest

from blendtorch import _native
from blendtorch.transport import zmq

MORE, LONG, COMMAND = 0x01, 0x02, 0x04


def _recvn(s, n):
    b = b''
    while len(b) < n:
        chunk = s.recv(n - len(b))
        if not chunk:
            raise ConnectionError('peer closed')
        b += chunk
    return b


class RawPeer:
    """A ZMTP 3.x peer written from the RFC, independent of the engine under test."""

    def __init__(self, sock):
        self.s = sock
        self.s.settimeout(5.0)
        self.peer_props = None

    @classmethod
    def connect(cls, port):
        return cls(socket.create_connection(('127.0.0.1', port)))

    def greet(self, minor=0, fragmented=False):
        sig = b'\xff' + b'\x00' * 8 + b'\x7f'
        rest = bytes([3, minor]) + b'NULL'.ljust(20, b'\x00') + b'\x00' + b'\x00' * 31
        assert len(sig + rest) == 64
        if fragmented:
            # libzmq: signature first, then the version once it saw the peer's
            # signature, then the rest -- here additionally split mid-field
            self.s.sendall(sig)
            time.sleep(0.02)
            for chunk in (rest[:1], rest[1:2], rest[2:7], rest[7:30], rest[30:]):
                self.s.sendall(chunk)
                time.sleep(0.01)
        else:
            self.s.sendall(sig + rest)
        g = _recvn(self.s, 64)
        assert g[0] == 0xFF and g[9] == 0x7F, g[:10]
        assert g[10] == 3                     # major version 3
        assert g[12:16] == b'NULL' and g[16:32] == b'\x00' * 16
        assert g[32] == 0                     # as-server flag (NULL mechanism: 0)
        return g

    @staticmethod
    def props(**kv):
        out = b''
        for k, v in kv.items():
            k = k.replace('_', '-').encode()
            out += bytes([len(k)]) + k + struct.pack('>I', len(v)) + v
        return out

    def send_command(self, name, body, force_long=False):
        payload = bytes([len(name)]) + name + body
        if len(payload) > 255 or force_long:
            self.s.sendall(bytes([COMMAND | LONG]) + struct.pack('>Q', len(payload)) + payload)
        else:
            self.s.sendall(bytes([COMMAND, len(payload)]) + payload)

    def ready(self, sock_type, identity=None):
        kv = {'Socket_Type': sock_type}
        if identity is not None:
            kv['Identity'] = identity
        self.send_command(b'READY', self.props(**kv))
        flags, body = self.read_frame()
        assert flags & COMMAND and body[:6] == b'\x05READY'
        self.peer_props = self.parse_props(body[6:])
        return self.peer_props

    @staticmethod
    def parse_props(b):
        out, i = {}, 0
        while i < len(b):
            n = b[i]
            k = b[i + 1:i + 1 + n].decode()
            (vl,) = struct.unpack('>I', b[i + 1 + n:i + 5 + n])
            out[k] = b[i + 5 + n:i + 5 + n + vl]
            i += 5 + n + vl
        return out

    def handshake(self, sock_type, minor=0, fragmented=False, identity=None):
        self.greet(minor, fragmented)
        return self.ready(sock_type, identity)

    def send_frame(self, body, more=False, force_long=False):
        f = MORE if more else 0
        if len(body) > 255 or force_long:
            self.s.sendall(bytes([f | LONG]) + struct.pack('>Q', len(body)) + body)
        else:
            self.s.sendall(bytes([f, len(body)]) + body)

    def send_msg(self, frames, force_long=False):
        for i, fr in enumerate(frames):
            self.send_frame(fr, more=i + 1 < len(frames), force_long=force_long)

    def read_frame(self):
        flags = _recvn(self.s, 1)[0]
        if flags & LONG:
            (size,) = struct.unpack('>Q', _recvn(self.s, 8))
        else:
            size = _recvn(self.s, 1)[0]
        return flags, _recvn(self.s, size)

    def read_msg(self):
        frames = []
        while True:
            flags, body = self.read_frame()
            if flags & COMMAND:
                continue                     # e.g. PING
            frames.append(body)
            if not flags & MORE:
                return frames

    def close(self):
        self.s.close()


class RawServer:
    """Listening side for native sockets that connect."""

    def __init__(self):
        self.l = socket.socket()
        self.l.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.l.bind(('127.0.0.1', 0))
        self.l.listen(4)
        self.l.settimeout(5.0)
        self.port = self.l.getsockname()[1]

    def accept(self):
        c, _ = self.l.accept()
        return RawPeer(c)

    def close(self):
        self.l.close()


def _native_sock(kind, timeout=3000):
    s = zmq.Context().socket(kind)
    s.setsockopt(zmq.RCVTIMEO, timeout)
    s.setsockopt(zmq.LINGER, 0)
    return s


# ---------------------------------------------------------------------------
# PUSH (raw, = Blender's pyzmq) -> PULL (native)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize('minor,fragmented', [(0, False), (1, False), (0, True), (1, True)])
def test_raw_push_into_native_pull(free_port, minor, fragmented):
    pull = _native_sock(zmq.PULL)
    pull.bind(f'tcp://127.0.0.1:{free_port}')
    peer = RawPeer.connect(free_port)
    props = peer.handshake(b'PUSH', minor=minor, fragmented=fragmented)
    assert props['Socket-Type'] == b'PULL'
    peer.send_msg([b'single'])
    assert pull.recv() == b'single'
    peer.send_msg([b'part1', b'', b'part3'])              # MORE-flag multipart, incl. an empty frame
    assert pull.recv_multipart() == [b'part1', b'', b'part3']
    small_long = bytes(range(100))
    peer.send_msg([small_long], force_long=True)          # 8-byte size on a small frame
    assert pull.recv() == small_long
    big = np.random.default_rng(0).integers(0, 256, 1228800, dtype=np.uint8).tobytes()   # one RGBA frame
    peer.send_msg([b'hdr', big])
    assert pull.recv_multipart() == [b'hdr', big]
    # a pickled producer dict exactly as pyzmq's send_pyobj frames it
    obj = {'btid': 1, 'image': np.zeros((4, 5, 3), np.uint8), 'frameid': 9}
    peer.send_msg([pickle.dumps(obj, protocol=4)])
    got = pull.recv_pyobj()
    assert got['btid'] == 1 and got['frameid'] == 9 and got['image'].shape == (4, 5, 3)
    peer.close()
    pull.close()


def test_native_push_greets_and_frames_like_libzmq(free_port):
    push = _native_sock(zmq.PUSH)
    push.bind(f'tcp://127.0.0.1:{free_port}')
    peer = RawPeer.connect(free_port)
    props = peer.handshake(b'PULL', minor=1)
    assert props['Socket-Type'] == b'PUSH'
    push.send_multipart([b'a', b'b' * 300])
    f1, b1 = peer.read_frame()
    f2, b2 = peer.read_frame()
    assert f1 == MORE and b1 == b'a'
    assert f2 == LONG and b2 == b'b' * 300
    peer.close()
    push.close()


# ---------------------------------------------------------------------------
# REQ / DEALER (raw) -> REP (native): envelope echoed byte-exact
# ---------------------------------------------------------------------------
def test_raw_req_into_native_rep_envelope(free_port):
    rep = _native_sock(zmq.REP)
    rep.bind(f'tcp://127.0.0.1:{free_port}')
    peer = RawPeer.connect(free_port)
    assert peer.handshake(b'REQ')['Socket-Type'] == b'REP'
    peer.send_msg([b'', pickle.dumps({'cmd': 'reset'})])
    assert rep.recv_pyobj() == {'cmd': 'reset'}
    rep.send(b'reply-1')
    assert peer.read_msg() == [b'', b'reply-1']
    peer.close()
    rep.close()


def test_raw_dealer_routing_envelope_echoed(free_port):
    """Frames before the empty delimiter are the routing envelope (e.g. a
    4-byte correlate id from a REQ_CORRELATE client, or proxy identities):
    REP must hand back exactly those bytes, in order, before the reply."""
    rep = _native_sock(zmq.REP)
    rep.bind(f'tcp://127.0.0.1:{free_port}')
    peer = RawPeer.connect(free_port)
    assert peer.handshake(b'DEALER')['Socket-Type'] == b'REP'
    env = [b'\x00\x01\x02\x03', b'hop-b']
    peer.send_msg(env + [b'', b'request'])
    assert rep.recv() == b'request'
    rep.send_multipart([b'r1', b'r2'])
    assert peer.read_msg() == env + [b'', b'r1', b'r2']
    # second request with another envelope: no state leaks from the first
    peer.send_msg([b'\xaa\xbb\xcc\xdd', b'', b'again'])
    assert rep.recv() == b'again'
    rep.send(b'ok')
    assert peer.read_msg() == [b'\xaa\xbb\xcc\xdd', b'', b'ok']
    peer.close()
    rep.close()


# ---------------------------------------------------------------------------
# REQ (native, RELAXED + CORRELATE) -> REP (raw)
# ---------------------------------------------------------------------------
def test_native_req_correlate_relaxed_wire():
    srv = RawServer()
    req = _native_sock(zmq.REQ, timeout=3000)
    req.setsockopt(zmq.REQ_RELAXED, 1)
    req.setsockopt(zmq.REQ_CORRELATE, 1)
    req.connect(f'tcp://127.0.0.1:{srv.port}')
    peer = srv.accept()
    assert peer.handshake(b'REP')['Socket-Type'] == b'REQ'

    req.send(b'first')
    m1 = peer.read_msg()
    assert len(m1) == 3 and len(m1[0]) == 4 and m1[1] == b'' and m1[2] == b'first'
    # RELAXED: a new request without waiting for the reply; a new id
    req.send(b'second')
    m2 = peer.read_msg()
    assert len(m2[0]) == 4 and m2[1] == b'' and m2[2] == b'second' and m2[0] != m1[0]
    # CORRELATE: the reply to the superseded request is dropped ...
    peer.send_msg([m1[0], b'', b'stale'])
    # ... and so is one with a forged id; only the current id gets through
    peer.send_msg([b'\xde\xad\xbe\xef', b'', b'forged'])
    peer.send_msg([m2[0], b'', b'fresh'])
    assert req.recv() == b'fresh'
    peer.close()
    req.close()
    srv.close()


def test_native_req_plain_envelope():
    """Without CORRELATE a REQ request is [empty delimiter, body] (RFC 28)."""
    srv = RawServer()
    req = _native_sock(zmq.REQ)
    req.connect(f'tcp://127.0.0.1:{srv.port}')
    peer = srv.accept()
    peer.handshake(b'REP')
    req.send(b'ping')
    assert peer.read_msg() == [b'', b'ping']
    peer.send_msg([b'', b'pong'])
    assert req.recv() == b'pong'
    peer.close()
    req.close()
    srv.close()


# ---------------------------------------------------------------------------
# PAIR both ways
# ---------------------------------------------------------------------------
def test_pair_native_bind_raw_connect(free_port):
    pair = _native_sock(zmq.PAIR)
    pair.bind(f'tcp://127.0.0.1:{free_port}')
    peer = RawPeer.connect(free_port)
    assert peer.handshake(b'PAIR')['Socket-Type'] == b'PAIR'
    peer.send_msg([pickle.dumps({'btid': None, 'msg': 'hi'}, protocol=4)])
    assert pair.recv_pyobj() == {'btid': None, 'msg': 'hi'}
    pair.send_multipart([b'x', b'y'])
    assert peer.read_msg() == [b'x', b'y']
    peer.close()
    pair.close()


def test_pair_raw_bind_native_connect():
    srv = RawServer()
    pair = _native_sock(zmq.PAIR)
    pair.connect(f'tcp://127.0.0.1:{srv.port}')
    peer = srv.accept()
    assert peer.handshake(b'PAIR', minor=1)['Socket-Type'] == b'PAIR'
    pair.send(b'from-native')
    assert peer.read_msg() == [b'from-native']
    peer.send_msg([b'from-raw'])
    assert pair.recv() == b'from-raw'
    peer.close()
    pair.close()
    srv.close()


def test_incompatible_socket_type_rejected(free_port):
    pull = _native_sock(zmq.PULL)
    pull.bind(f'tcp://127.0.0.1:{free_port}')
    peer = RawPeer.connect(free_port)
    peer.greet()
    peer.send_command(b'READY', RawPeer.props(Socket_Type=b'PULL'))   # PULL-PULL is invalid
    # the engine answers with its READY or an ERROR and then drops the connection
    got = b''
    try:
        while True:
            chunk = peer.s.recv(4096)
            if not chunk:
                break
            got += chunk
    except (ConnectionError, socket.timeout):
        pass
    assert b'READY' not in got[got.find(b'ERROR'):] if b'ERROR' in got else True
    peer.close()
    pull.close()


# ---------------------------------------------------------------------------
# hostile peers: malformed framing must close that connection only
# ---------------------------------------------------------------------------
@pytest.mark.parametrize('evil', ['zero_command', 'name_past_frame', 'huge_long_command', 'huge_data_frame'])
def test_hostile_frames_do_not_crash(free_port, evil):
    pull = _native_sock(zmq.PULL)
    pull.bind(f'tcp://127.0.0.1:{free_port}')
    bad = RawPeer.connect(free_port)
    bad.handshake(b'PUSH')
    if evil == 'zero_command':
        bad.s.sendall(bytes([COMMAND, 0]) + b'PING' * 8)
    elif evil == 'name_past_frame':
        bad.s.sendall(bytes([COMMAND, 3, 200]) + b'ab' + b'\x00' * 64)
    elif evil == 'huge_long_command':
        bad.s.sendall(bytes([COMMAND | LONG]) + struct.pack('>Q', 2 ** 64 - 5) + b'\x04PING' + b'\x00' * 32)
    else:
        bad.s.sendall(bytes([LONG]) + struct.pack('>Q', 2 ** 62) + b'\x00' * 64)
    # the engine drops the offender ...
    bad.s.settimeout(3.0)
    try:
        closed = bad.s.recv(1) == b''
    except (ConnectionError, socket.timeout):
        closed = True
    assert closed
    bad.close()
    # ... and keeps serving well-behaved peers
    good = RawPeer.connect(free_port)
    good.handshake(b'PUSH')
    good.send_msg([b'still-alive'])
    assert pull.recv() == b'still-alive'
    good.close()
    pull.close()


# ---------------------------------------------------------------------------
# pickles as other numpy / pickle versions write them
# ---------------------------------------------------------------------------
class _Numpy1Path:
    """Temporarily make CPython's pickler write numpy-1.x module paths."""

    def __enter__(self):
        import numpy._core.multiarray as ma
        import numpy._core.numeric as nu
        self.saved = [(ma._reconstruct, ma._reconstruct.__module__), (nu._frombuffer, nu._frombuffer.__module__)]
        ma._reconstruct.__module__ = 'numpy.core.multiarray'
        nu._frombuffer.__module__ = 'numpy.core.numeric'
        return self

    def __exit__(self, *a):
        for f, m in self.saved:
            f.__module__ = m


@pytest.mark.parametrize('protocol', [2, 3, 4, 5])
@pytest.mark.parametrize('numpy1', [False, True])
def test_native_loader_decodes_foreign_pickles(protocol, numpy1):
    import warnings
    img = np.random.default_rng(protocol).integers(0, 256, (48, 64, 4), dtype=np.uint8)
    obj = {'btid': 2, 'image': img, 'xy': np.random.rand(8, 2), 'frameid': 11}
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', DeprecationWarning)
        if numpy1:
            with _Numpy1Path():
                raw = pickle.dumps(obj, protocol=protocol)
            assert b'numpy.core.' in raw and b'numpy._core' not in raw
        else:
            raw = pickle.dumps(obj, protocol=protocol)
        if protocol == 2:
            pytest.importorskip('numpy')
        got = _native.fast_loads(raw)
    assert got['btid'] == 2 and got['frameid'] == 11
    assert np.array_equal(got['image'], img) and np.array_equal(got['xy'], obj['xy'])
    assert _native.pickle_describe(raw)   # the loader's scanner locates the payloads too


def _patched_shape(shape_ops):
    """A numpy pickle (protocol 2) of 6 bytes whose shape tuple is replaced."""
    raw = pickle.dumps(np.arange(6, dtype=np.uint8).reshape(2, 3), protocol=2)
    good = b'K\x02K\x03\x86'
    assert raw.count(good) == 1
    return raw.replace(good, shape_ops)


@pytest.mark.parametrize('shape_ops', [
    b'J\xfe\xff\xff\xffJ\xfd\xff\xff\xff\x86',                         # (-2, -3): product 6
    b'\x8a\x05\x00\x00\x00\x00\x01\x8a\x05\x00\x00\x00\x00\x01\x86',   # (2**32, 2**32): overflows int64 product
    b'\x8a\x09\x00\x00\x00\x00\x00\x00\x00\x00\x01K\x06\x86',          # (2**64, 6): long beyond int64
])
def test_fast_loads_rejects_hostile_shapes(shape_ops):
    raw = _patched_shape(shape_ops)
    with pytest.raises((ValueError, OverflowError)):
        _native.fast_loads(raw)


@pytest.mark.parametrize('op', [b'\x8e', b'\x8d', b'\x96'])   # BINBYTES8, BINUNICODE8, BYTEARRAY8
def test_fast_loads_rejects_wrapping_lengths(op):
    for n in (2 ** 64 - 1, 2 ** 64 - 8, 2 ** 63):
        raw = b'\x80\x05' + op + struct.pack('<Q', n) + b'abc.'
        with pytest.raises(ValueError):
            _native.fast_loads(raw)
