"""Native ZMTP/3.0 engine: wire bytes, socket patterns, options, and the
zero-copy pickle codec (differentially tested against CPython pickle)."""
import pickle
import socket
import struct
import threading
import time

import numpy as np
import pytest

from blendtorch import _native
from blendtorch.transport import zmq


def test_greeting_and_ready_bytes_rfc():
    g = _native.greeting_bytes(False)
    assert len(g) == 64
    assert g[0] == 0xFF and g[9] == 0x7F                 # signature
    assert g[10] == 3                                      # major version
    assert g[12:16] == b'NULL' and g[16:32] == b'\x00' * 16
    r = _native.ready_command(zmq.PUSH)
    # flags(COMMAND) size, name-len, "READY", property "Socket-Type" = "PUSH"
    assert r[0] & 0x04
    body = r[2:] if not (r[0] & 0x02) else r[9:]
    assert body[:6] == b'\x05READY'
    assert b'\x0bSocket-Type\x00\x00\x00\x04PUSH' in body


def _raw_peer_handshake(port, sock_type=b'PULL'):
    """Speak ZMTP by hand (independent oracle of the wire format)."""
    s = socket.create_connection(('127.0.0.1', port))
    greeting = b'\xff' + b'\x00' * 8 + b'\x7f' + bytes([3, 0]) + b'NULL' + b'\x00' * 16 + b'\x00' + b'\x00' * 31
    s.sendall(greeting)
    got = b''
    while len(got) < 64:
        got += s.recv(64 - len(got))
    assert got[0] == 0xFF and got[10] == 3
    prop = b'\x0bSocket-Type' + struct.pack('>I', len(sock_type)) + sock_type
    cmd = b'\x05READY' + prop
    s.sendall(bytes([0x04, len(cmd)]) + cmd)
    return s


def _read_frame(s):
    hdr = s.recv(1)
    flags = hdr[0]
    if flags & 0x02:
        size = struct.unpack('>Q', _recvn(s, 8))[0]
    else:
        size = _recvn(s, 1)[0]
    return flags, _recvn(s, size)


def _recvn(s, n):
    b = b''
    while len(b) < n:
        chunk = s.recv(n - len(b))
        assert chunk
        b += chunk
    return b


def test_wire_interop_with_handwritten_peer(free_port):
    ctx = zmq.Context()
    push = ctx.socket(zmq.PUSH)
    push.bind(f'tcp://127.0.0.1:{free_port}')
    s = _raw_peer_handshake(free_port)
    flags, body = _read_frame(s)            # peer's READY command
    assert flags & 0x04 and body.startswith(b'\x05READY') and b'PUSH' in body
    push.send(b'hello')
    big = bytes(range(256)) * 1000
    push.send(big)
    f1, b1 = _read_frame(s)
    f2, b2 = _read_frame(s)
    assert (f1, b1) == (0, b'hello')
    assert f2 & 0x02 and b2 == big             # long frame: 8-byte size
    s.close()
    push.close()


def test_push_pull_round_robin_and_fair_queue(free_port):
    ctx = zmq.Context()
    push = ctx.socket(zmq.PUSH)
    push.bind(f'tcp://127.0.0.1:{free_port}')
    pulls = [ctx.socket(zmq.PULL) for _ in range(2)]
    for p in pulls:
        p.connect(f'tcp://127.0.0.1:{free_port}')
    time.sleep(0.2)
    for i in range(10):
        push.send_pyobj(i)
    got = [[], []]
    for k, p in enumerate(pulls):
        while p.poll(300):
            got[k].append(p.recv_pyobj())
    assert sorted(got[0] + got[1]) == list(range(10))
    assert len(got[0]) == 5 and len(got[1]) == 5
    for s in pulls + [push]:
        s.close()


def test_sndhwm_backpressure_blocks_not_drops(free_port):
    ctx = zmq.Context()
    push = ctx.socket(zmq.PUSH)
    push.setsockopt(zmq.SNDHWM, 2)
    push.setsockopt(zmq.IMMEDIATE, 1)
    push.bind(f'tcp://127.0.0.1:{free_port}')
    # IMMEDIATE: no peer -> a non-blocking send fails instead of queueing
    with pytest.raises(zmq.Again):
        push.send(b'x', zmq.NOBLOCK)
    pull = ctx.socket(zmq.PULL)
    pull.setsockopt(zmq.RCVHWM, 2)
    pull.connect(f'tcp://127.0.0.1:{free_port}')
    time.sleep(0.2)
    sent = 0
    payload = b'y' * (4 << 20)      # 4 MB: kernel buffers cannot absorb many
    t0 = time.time()
    while time.time() - t0 < 2.0:
        try:
            push.send(payload, zmq.NOBLOCK)
            sent += 1
        except zmq.Again:
            break
    assert sent < 50                  # sender was blocked by HWM
    n = 0
    while pull.poll(500):
        pull.recv()
        n += 1
    assert n == sent                  # nothing was dropped
    push.close()
    pull.close()


def test_req_rep_relaxed_correlate(free_port):
    ctx = zmq.Context()
    rep = ctx.socket(zmq.REP)
    rep.bind(f'tcp://127.0.0.1:{free_port}')
    req = ctx.socket(zmq.REQ)
    req.setsockopt(zmq.REQ_RELAXED, 1)
    req.setsockopt(zmq.REQ_CORRELATE, 1)
    req.setsockopt(zmq.RCVTIMEO, 2000)
    req.connect(f'tcp://127.0.0.1:{free_port}')
    req.send_pyobj({'cmd': 'a'})
    assert rep.recv_pyobj() == {'cmd': 'a'}
    # RELAXED: a new request may be sent before the reply arrived
    req.send_pyobj({'cmd': 'b'})
    rep.send_pyobj('reply-a')          # stale reply to the first request
    assert rep.recv_pyobj() == {'cmd': 'b'}
    rep.send_pyobj('reply-b')
    assert req.recv_pyobj() == 'reply-b'   # CORRELATE drops the stale one
    req.close()
    rep.close()


def test_rcvtimeo_raises_again(free_port):
    ctx = zmq.Context()
    pull = ctx.socket(zmq.PULL)
    pull.setsockopt(zmq.RCVTIMEO, 100)
    pull.bind(f'tcp://127.0.0.1:{free_port}')
    t0 = time.time()
    with pytest.raises(zmq.Again):
        pull.recv()
    assert 0.05 < time.time() - t0 < 2
    pull.close()


def test_pair_and_ipc(tmp_path):
    ctx = zmq.Context()
    a = ctx.socket(zmq.PAIR)
    a.bind(f'ipc://{tmp_path}/sock')
    b = ctx.socket(zmq.PAIR)
    b.connect(f'ipc://{tmp_path}/sock')
    b.send_pyobj({'x': 1})
    assert a.recv_pyobj() == {'x': 1}
    a.send_multipart([b'p1', b'p2'])
    assert b.recv_multipart() == [b'p1', b'p2']
    a.close()
    b.close()


def test_linger_flushes_on_close(free_port):
    ctx = zmq.Context()
    push = ctx.socket(zmq.PUSH)
    push.setsockopt(zmq.LINGER, 2000)
    push.bind(f'tcp://127.0.0.1:{free_port}')
    pull = ctx.socket(zmq.PULL)
    pull.connect(f'tcp://127.0.0.1:{free_port}')
    time.sleep(0.1)
    for i in range(20):
        push.send(b'z' * 100000)
    push.close()                        # blocks until flushed (<= linger)
    n = 0
    while pull.poll(500):
        pull.recv()
        n += 1
    assert n == 20
    pull.close()


PAYLOADS = [
    {'btid': 3, 'image': np.random.randint(0, 255, (48, 64, 3), np.uint8), 'xy': np.random.rand(8, 2),
     'frameid': 7},
    {'a': None, 'b': True, 'c': 1.5, 'd': 'text', 'e': b'bytes', 'f': [1, 2, (3, 4)], 'g': {'nested': 1}},
    {'big': 2 ** 40, 'neg': -5, 'f32': np.float32(2.5), 'i64': np.int64(9), 'arr': np.arange(10, dtype=np.int64)},
    {'fortran': np.asfortranarray(np.random.rand(3, 4)), 'empty': np.zeros((0, 3), np.float32)},
    {'flipped': np.flipud(np.arange(12, dtype=np.uint8).reshape(4, 3))},
]


def _eq(a, b):
    if isinstance(a, np.ndarray):
        return isinstance(b, np.ndarray) and a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_eq(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return type(a) == type(b) and len(a) == len(b) and all(_eq(x, y) for x, y in zip(a, b))
    return a == b and type(a) == type(b)


@pytest.mark.parametrize('protocol', [3, 4, 5])
@pytest.mark.parametrize('idx', range(len(PAYLOADS)))
def test_fast_loads_matches_pickle(protocol, idx):
    raw = pickle.dumps(PAYLOADS[idx], protocol=protocol)
    ref = pickle.loads(raw)
    try:
        got = _native.fast_loads(raw)
    except ValueError:
        pytest.skip('construct outside the fast path (falls back to pickle)')
    assert _eq(ref, got)


def test_native_writer_roundtrip():
    d = {'btid': 1, 'image': np.random.randint(0, 255, (10, 12, 4), np.uint8), 'xy': np.random.rand(8, 2),
         'frameid': 300, 'name': 'x', 'ok': True, 'none': None, 'f': 0.25}
    for proto in (3, 4, 5):
        raw = _native.dumps_array_dict(d, proto)
        assert _eq(pickle.loads(raw), d)


def test_hypothesis_dict_roundtrip():
    hyp = pytest.importorskip('hypothesis')
    from hypothesis import given, settings, strategies as st
    values = st.one_of(st.none(), st.booleans(), st.integers(-2 ** 62, 2 ** 62), st.floats(allow_nan=False),
                       st.text(max_size=20), st.binary(max_size=50))
    dicts = st.dictionaries(st.text(min_size=1, max_size=8), values, max_size=6)

    @settings(max_examples=200, deadline=None)
    @given(dicts, st.sampled_from([3, 4, 5]))
    def check(d, proto):
        raw = pickle.dumps(d, protocol=proto)
        try:
            got = _native.fast_loads(raw)
        except ValueError:
            return
        assert _eq(pickle.loads(raw), got)
    check()


@pytest.mark.parametrize('n', [5, 200, 256, 4099, 921600])
@pytest.mark.parametrize('align', [16, 64])
def test_writer_aligned_payload(n, align):
    """Writer.ndarray(align=...) pads with pickle no-ops so the payload starts
    at an aligned offset; pickle, numpy and the native scanner read the same
    value as without padding."""
    import pickle as _pickle
    from blendtorch import _native
    rng = np.random.default_rng(n)
    for key in ('k', 'key-xyz', 'a' * 37):
        img = rng.integers(0, 256, size=n, dtype=np.uint8)
        d = {'btid': 1, key: 2.5, 'image': img, 'xy': np.arange(16.0).reshape(8, 2)}
        b = _native.dumps_array_dict(d, 4, align)
        off = b.find(img.tobytes())
        assert off > 0 and off % align == 0
        for r in (_pickle.loads(b), _native.fast_loads(b)):
            assert np.array_equal(r['image'], img) and r[key] == 2.5 and np.array_equal(r['xy'], d['xy'])


def test_recv_round_fair_across_uneven_sockets(tmp_path):
    """The GPU loader's fan-in policy (csrc/gpu/loader.cpp run(): one
    Socket::recv_round per pass, at most ONE message per producer pipe across
    all IO sockets).  5 backpressured producers spread over 4 PULL sockets as
    the loader spreads them ({p0,p4}, {p1}, {p2}, {p3}): every producer's share
    stays within +-10 % of 1/5 over >= 2000 messages (the reference's contract:
    examples/datagen/Readme.md:177, workers interleave producers fairly).
    Draining a socket at a time would give p1..p3 twice p0's and p4's share."""
    P, K = 5, 4
    ctx = zmq.Context()
    addrs = [f'ipc://{tmp_path}/p{i}' for i in range(P)]
    stop = threading.Event()
    sent = [0] * P

    def produce(i, s):
        while not stop.is_set():
            try:
                s.send(bytes([i]) * 256, zmq.NOBLOCK)
                sent[i] += 1
            except zmq.Again:
                time.sleep(0.0002)

    pushes = []
    for a in addrs:
        s = ctx.socket(zmq.PUSH)
        s.setsockopt(zmq.SNDHWM, 4)
        s.setsockopt(zmq.LINGER, 0)
        s.bind(a)
        pushes.append(s)
    pulls = []
    for _ in range(K):
        s = ctx.socket(zmq.PULL)
        s.setsockopt(zmq.RCVHWM, 4)
        s.setsockopt(zmq.LINGER, 0)
        pulls.append(s)
    for i, a in enumerate(addrs):
        pulls[i % K].connect(a)
    threads = [threading.Thread(target=produce, args=(i, pushes[i]), daemon=True) for i in range(P)]
    for t in threads:
        t.start()
    try:
        deadline = time.time() + 10
        while min(sent) < 50 and time.time() < deadline:   # every pipe backlogged
            time.sleep(0.01)
        counts = [0] * P
        rounds = 0
        while sum(counts) < 2500 and time.time() < deadline + 30:
            got = _native.recv_round([p._sock for p in pulls])
            rounds += 1
            ids = [bytes(parts[0])[0] for parts in got]
            assert len(ids) == len(set(ids)), ids      # one message per producer per round
            for i in ids:
                counts[i] += 1
            time.sleep(0.0005)            # a consumer slower than its producers
        total = sum(counts)
        assert total >= 2000, counts
        shares = [c / total for c in counts]
        assert all(abs(s - 1 / P) <= 0.1 / P for s in shares), (counts, rounds)
    finally:
        stop.set()
        for t in threads:
            t.join(2)
        for s in pulls + pushes:
            s.close(0)
