"""Shared-memory ring ownership: the lease never takes a frame from a
consumer that claimed it, stale descriptors are dropped (not raised), and a
tile16 key frame replaced mid-stream stays readable until every frame that
names it is gone (shmring lease, set_key_frame)."""
import os
import threading
import time

import numpy as np
import pytest

from blendtorch import btt
from blendtorch.btb.publisher import DataPublisher
from blendtorch.transport import shm, zmq


def _ring(nslots=2, nbytes=64, lease_s=0.1):
    name = f'blendtorch-{os.getpid()}-test-{time.monotonic_ns()}'
    return shm.ShmRing(name, nslots, nbytes, lease_s=lease_s)


def _desc(ring, put):
    slot, off, h, w, c, gen = put
    return (ring.name, slot, off, h, w, c, 'image', gen)


def test_lease_reclaims_only_unclaimed_slots():
    ring = _ring()
    try:
        a = _desc(ring, ring.put(np.full((4, 16), 1, np.uint8)))
        b = _desc(ring, ring.put(np.full((4, 16), 2, np.uint8)))
        assert shm.claim(a)                       # consumer holds A (e.g. paused mid-epoch)
        t0 = time.time()
        slot = ring.acquire(timeout_s=2.0)         # producer starves, then reclaims
        assert time.time() - t0 >= 0.1
        assert slot == b[1] and ring.reclaimed == 1  # the unclaimed one, never A
        # B's descriptor is stale now: dropped, not raised
        before = shm.stats['stale']
        assert shm.resolve({shm.KEY: b}) is None
        assert shm.stats['stale'] == before + 1
        with pytest.raises(shm.TornFrame):
            shm.resolve({shm.KEY: b}, strict=True)
        # A's pixels are intact and its slot goes back on release
        seg = shm._open(a[0])
        assert (seg.slot_array(a[1], (4, 16)) == 1).all()
        shm.release(a)
        assert int(seg.states[a[1]]) & 3 == shm.FREE
    finally:
        ring.close()


def test_held_slot_reclaimed_only_after_dead_consumer_factor():
    ring = _ring(nslots=1, lease_s=0.02)
    try:
        a = _desc(ring, ring.put(np.zeros((2, 8), np.uint8)))
        assert shm.claim(a)
        with pytest.raises(TimeoutError):          # 5x the lease: still ours
            ring.acquire(timeout_s=0.1)
        assert ring.reclaimed == 0
        slot = ring.acquire(timeout_s=5.0)          # > 20x the lease: the consumer is presumed dead
        assert slot == a[1] and ring.reclaimed == 1
    finally:
        ring.close()


def test_slot_cas_is_atomic_native():
    from blendtorch import _native
    w = np.zeros(4, np.uint32)
    assert _native.slot_cas(w, 2, 0, 7) and w[2] == 7
    assert not _native.slot_cas(w, 2, 0, 9) and w[2] == 7
    with pytest.raises(TypeError):
        _native.slot_cas(np.zeros(4, np.int64), 0, 0, 1)   # no silent cast copy
    with pytest.raises(IndexError):
        _native.slot_cas(w, 4, 0, 1)


def test_dataset_survives_consumer_pause_past_lease(free_port):
    """A CPU consumer that stops taking frames for longer than the producer's
    lease: frames it already claimed are intact, queued descriptors whose
    slots were reclaimed are dropped, and the stream keeps its length."""
    addr = f'tcp://127.0.0.1:{free_port}'
    pub = DataPublisher(addr, btid=0, shm_slots=3, shm_lease_s=0.05, send_hwm=2)
    stop = threading.Event()

    def produce():
        i = 0
        while not stop.is_set():
            try:
                pub.publish(image=np.full((8, 8, 3), i % 251, np.uint8), frameid=i)
            except Exception:
                return
            i += 1

    th = threading.Thread(target=produce, daemon=True)
    th.start()
    try:
        ds = btt.RemoteIterableDataset([addr], max_items=40, timeoutms=10000, queue_size=2)
        got = []
        for k, item in enumerate(ds):
            if k == 5:
                time.sleep(0.6)              # 12x the lease
            img = item['image']
            assert (img == item['frameid'] % 251).all()   # pixels belong to their metadata
            got.append(item['frameid'])
        assert len(got) == 40
        assert got == sorted(got)
    finally:
        stop.set()
        pub.close()
        th.join(5)


def test_set_key_frame_mid_stream_cpu(free_port):
    """Frames published against key K1 are still queued when the producer
    switches to K2: they must decode against K1 (its segment stays alive),
    and K1 is unlinked once they have all been handed back."""
    h, w = 32, 48
    k1 = np.full((h, w, 3), 10, np.uint8)
    k2 = np.full((h, w, 3), 200, np.uint8)
    frames = []
    for i in range(8):
        f = (k1 if i < 4 else k2).copy()
        f[(i * 3) % 16:(i * 3) % 16 + 8, 16:32] = 50 + i
        frames.append(f)
    addr = f'tcp://127.0.0.1:{free_port}'
    pub = DataPublisher(addr, btid=1, shm_slots=16, shm_codec='tile16', send_hwm=20)
    pull = zmq.Context().socket(zmq.PULL)
    pull.setsockopt(zmq.RCVHWM, 20)
    pull.connect(addr)
    time.sleep(0.2)
    try:
        pub.set_key_frame(k1)
        for f in frames[:4]:
            pub.publish(image=f)
        old_key = pub._key_ring.name
        pub.set_key_frame(k2)
        assert os.path.exists('/dev/shm/' + old_key)      # 4 frames still name it
        for f in frames[4:]:
            pub.publish(image=f)
        for i in range(8):
            assert pull.poll(5000)
            msg = shm.resolve(pull.recv_pyobj())
            assert np.array_equal(msg['image'], frames[i]), i
        pub.publish(image=frames[0])                       # next publish reaps retired keys
        assert not os.path.exists('/dev/shm/' + old_key)
        assert pub._retired_keys == []
    finally:
        pull.close()
        pub.close()


def test_libatomic_cas_fallback_is_atomic_cas():
    """Without the native module (Blender's Python) slot words still change
    by a real compare-and-swap (libatomic through ctypes)."""
    import numpy as np
    from blendtorch.transport import shm
    cas = shm._libatomic_cas()
    assert cas is not None
    words = np.zeros(4, dtype=np.uint32)
    words[2] = (7 << 2) | shm.PUBLISHED
    assert not cas(words, 2, (7 << 2) | shm.FREE, 1)           # wrong expectation: untouched
    assert words[2] == (7 << 2) | shm.PUBLISHED
    assert cas(words, 2, (7 << 2) | shm.PUBLISHED, (7 << 2) | shm.HELD)
    assert words[2] == (7 << 2) | shm.HELD and words[1] == 0 and words[3] == 0


def test_cas_through_ctypes_path_with_native_forced_off(monkeypatch):
    """``shm._cas`` with the native module forced off goes through libatomic's
    out-of-line ``__atomic_compare_exchange_4(ptr, expected*, desired,
    success_order, failure_order)``; threads racing CAS-increments on one
    word (ctypes drops the GIL around the call) lose no update."""
    import threading
    import numpy as np
    from blendtorch.transport import shm
    monkeypatch.setattr(shm, '_native_cas', None)
    monkeypatch.setattr(shm, '_ctypes_cas', shm._libatomic_cas())
    assert shm._ctypes_cas is not None
    words = np.zeros(2, dtype=np.uint32)
    assert shm._cas(words, 1, 0, 5) and words[1] == 5
    assert not shm._cas(words, 1, 0, 9) and words[1] == 5
    n_threads, per = 4, 2000

    def bump():
        for _ in range(per):
            while True:
                cur = int(words[0])
                if shm._cas(words, 0, cur, cur + 1):
                    break

    ts = [threading.Thread(target=bump) for _ in range(n_threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert int(words[0]) == n_threads * per and int(words[1]) == 5
