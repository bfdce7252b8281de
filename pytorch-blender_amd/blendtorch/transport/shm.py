"""Python side of the same-host shared-memory frame slots (csrc/transport/shmring.h).

Producers on the consumer's host may place image payloads in a POSIX
shared-memory ring and send only a descriptor ``'_btshm': (segment, slot,
byte_offset, H, W, C, key, generation[, codec])`` in the message dict; a 9th
element ``('tile16', key_segment, key_generation)`` marks a key-frame delta
frame (csrc/codec/tiledelta.h), which :func:`resolve` rebuilds.  The GPU loader DMAs the
slot in place; CPU consumers call :func:`resolve`, which copies the image into
the dict under ``key`` and hands the slot back.  :class:`ShmRing` is the
producer side for Python publishers (``btb.DataPublisher(shm_slots=N)``).

Segment layout (shared with C++): header {u64 magic, u32 version, u32 nslots,
u64 slot_bytes, u64 data_offset}, u32 word per slot (generation << 2 |
state; states 0 free, 1 writing, 2 published, 3 held), slots at data_offset
(4 KiB aligned).  Descriptors carry the generation: a consumer claims the slot
(CAS (gen, published) -> (gen, held)), copies, and hands it back (CAS (gen,
held) -> (gen, free)).  A producer starved for its lease reclaims only
published (unclaimed) slots, so a paused consumer never has a frame taken
from under it; a descriptor whose slot was reclaimed while it sat in a queue
is stale and is dropped (:func:`resolve` returns None).
"""
from __future__ import annotations

import mmap
import os
import struct
import time

import numpy as np

MAGIC = 0x6d68735f7462746e
_HDR = struct.Struct('<QIIQQ')
FREE, WRITING, PUBLISHED, HELD = 0, 1, 2, 3
HELD_LEASE_FACTOR = 20    # csrc/transport/shmring.h kHeldLeaseFactor
KEY = '_btshm'

try:   # atomic slot words (CPython build of the native module; absent inside Blender's Python)
    from .._native import slot_cas as _native_cas
except ImportError:  # pragma: no cover - exercised only without the native build
    _native_cas = None


def _libatomic_cas():
    """A lock-free 32-bit compare-and-swap from the GCC runtime's libatomic,
    through ctypes -- for Pythons without the native module (Blender's own):
    the producer's lease reclaim must not overwrite a slot a consumer has just
    claimed (PUBLISHED -> HELD) between a read and a store."""
    import ctypes
    import ctypes.util
    for name in ('libatomic.so.1', ctypes.util.find_library('atomic')):
        if not name:
            continue
        try:
            fn = ctypes.CDLL(name).__atomic_compare_exchange_4
        except (OSError, AttributeError):
            continue
        fn.restype = ctypes.c_bool
        # the out-of-line libatomic entry point is (ptr, expected*, desired,
        # success_order, failure_order) -- no 'weak' argument (that one exists
        # only in the compiler builtin)
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]

        def cas(states, i, expected, desired, _fn=fn, _c=ctypes):
            exp = _c.c_uint32(int(expected))
            addr = states.ctypes.data + 4 * int(i)
            return bool(_fn(addr, _c.addressof(exp), int(desired) & 0xFFFFFFFF, 5, 5))   # seq_cst, seq_cst
        return cas
    return None


_ctypes_cas = _libatomic_cas() if _native_cas is None else None


def _cas(states, i, expected, desired):
    """Compare-and-swap slot word ``i``: the native module's atomic, else
    libatomic's through ctypes; only without either a plain check-then-store
    (then a consumer's claim racing a producer's lease reclaim can be
    overwritten -- the loader reports that batch as torn)."""
    if _native_cas is not None:
        return _native_cas(states, int(i), int(expected), int(desired))
    if _ctypes_cas is not None:
        return _ctypes_cas(states, i, expected, desired)
    if int(states[i]) != expected:
        return False
    states[i] = desired
    return True

_views = {}
_views_pid = None


def _path(name):
    return '/dev/shm/' + name.lstrip('/')


class _Segment:
    def __init__(self, name, fd, mm, owner):
        self.name = name
        self.fd = fd
        self.mm = mm
        self.owner = owner
        magic, version, nslots, slot_bytes, data_offset = _HDR.unpack_from(mm, 0)
        if magic != MAGIC and not owner:
            raise ValueError(f'{name} is not a blendtorch shm segment')
        self.nslots, self.slot_bytes, self.data_offset = nslots, slot_bytes, data_offset
        self.states = np.frombuffer(mm, dtype=np.uint32, count=nslots, offset=_HDR.size)
        self.ino = os.fstat(fd).st_ino

    def slot_array(self, i, shape, dtype=np.uint8):
        off = self.data_offset + i * self.slot_bytes
        return np.frombuffer(self.mm, dtype=dtype, count=int(np.prod(shape)), offset=off).reshape(shape)

    def close(self):
        self.states = None
        try:
            self.mm.close()
        except BufferError:  # numpy views still alive; the mapping dies with them
            pass
        os.close(self.fd)
        if self.owner:
            try:
                os.unlink(_path(self.name))
            except FileNotFoundError:
                pass


def _open(name):
    global _views, _views_pid
    if _views_pid != os.getpid():   # fresh cache after fork
        _views, _views_pid = {}, os.getpid()
    seg = _views.get(name)
    if seg is not None:
        # a producer may have closed the segment and created a new one under
        # the same name: the cached mapping would show the old, unlinked file.
        # A file that is merely gone (unlinked, e.g. a retired key frame) is
        # still readable through the cached mapping.
        try:
            stale = os.stat(_path(name)).st_ino != seg.ino
        except FileNotFoundError:
            stale = False
        if stale:
            del _views[name]
            seg = None
    if seg is None:
        fd = os.open(_path(name), os.O_RDWR)
        size = os.fstat(fd).st_size
        seg = _Segment(name, fd, mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE), False)
        _views[name] = seg
    return seg


class TornFrame(RuntimeError):
    """The producer reclaimed the slot while it was being read."""


stats = {'stale': 0, 'torn': 0}   # descriptors dropped by resolve() in this process


def _word(gen, state):
    return ((int(gen) & 0x3fffffff) << 2) | state


TILE = 16   # csrc/codec/tiledelta.h kTile


def _expand_tiled(seg, off, h, w, c, codec):
    """Rebuild a key-frame delta frame (csrc/codec/tiledelta.h): the key frame
    from the producer's key segment, overwritten by the slot's payload tiles."""
    kind, key_name = codec[0], codec[1]
    if kind != 'tile16':
        raise ValueError(f'unknown shm codec {kind!r}')
    ty, tx = h // TILE, w // TILE
    nt = ty * tx
    n = int(np.frombuffer(seg.mm, dtype=np.uint32, count=1, offset=off)[0])
    pos = np.frombuffer(seg.mm, dtype=np.uint32, count=n, offset=off + 4).astype(np.int64)
    pay_off = off + (((nt + 1) * 4 + 255) & ~255)
    if n > nt or (n and int(pos.max()) >= nt):
        raise ValueError(f'malformed tile16 frame in {seg.name}')
    kseg = _open(key_name)
    img = np.frombuffer(kseg.mm, dtype=np.uint8, count=h * w * c, offset=kseg.data_offset).copy()
    if n:
        tiles = np.frombuffer(seg.mm, dtype=np.uint8, count=n * TILE * TILE * c, offset=pay_off)
        view = img.reshape(ty, TILE, tx, TILE, c)
        view[pos // tx, :, pos % tx] = tiles.reshape(n, TILE, TILE, c)
    return img


def release(desc):
    """Hand a descriptor's slot back without reading it (dropped messages)."""
    name, slot, off, h, w, c, key, gen = desc[:8]
    try:
        seg = _open(name)
    except FileNotFoundError:
        return            # producer gone: nothing to hand back
    if not _cas(seg.states, slot, _word(gen, HELD), _word(gen, FREE)):
        _cas(seg.states, slot, _word(gen, PUBLISHED), _word(gen, FREE))


def claim(desc):
    """Take a descriptor's slot (PUBLISHED -> HELD); False if it is stale."""
    name, slot, off, h, w, c, key, gen = desc[:8]
    return _cas(_open(name).states, slot, _word(gen, PUBLISHED), _word(gen, HELD))


def resolve(obj, strict=False):
    """Materialise a shared-memory image into ``obj`` (in place) and free its slot.

    Returns ``obj``, or None when the descriptor is stale (its producer
    reclaimed the slot while the message sat in a queue) or the slot was taken
    back during the copy -- the caller drops such a message rather than
    deliver another frame's pixels under its metadata.  ``strict=True``
    raises :class:`TornFrame` instead."""
    if not isinstance(obj, dict) or KEY not in obj:
        return obj
    desc = obj.pop(KEY)
    name, slot, off, h, w, c, key, gen = desc[:8]
    seg = _open(name)
    if not _cas(seg.states, slot, _word(gen, PUBLISHED), _word(gen, HELD)):
        stats['stale'] += 1
        if strict:
            raise TornFrame(f'shm slot {name}:{slot} was reclaimed before it was read')
        return None
    try:
        if len(desc) > 8 and desc[8]:
            img = _expand_tiled(seg, off, h, w, c, desc[8])
        else:
            n = h * w * c
            img = np.frombuffer(seg.mm, dtype=np.uint8, count=n, offset=off).copy()
    finally:
        ok = _cas(seg.states, slot, _word(gen, HELD), _word(gen, FREE))
    if not ok:
        stats['torn'] += 1
        if strict:
            raise TornFrame(f'shm slot {name}:{slot} was reclaimed while it was read')
        return None
    obj[key] = img.reshape((h, w, c) if c > 1 else (h, w))
    return obj


class ShmRing:
    """Producer-side ring (single writer).  ``acquire`` blocks while every slot
    is still with a consumer -- the same backpressure as a full SNDHWM."""

    def __init__(self, name, nslots, slot_bytes, lease_s=30.0):
        self.lease_s = lease_s
        slot_bytes = (slot_bytes + 4095) // 4096 * 4096
        data_offset = (_HDR.size + 4 * nslots + 4095) // 4096 * 4096
        size = data_offset + nslots * slot_bytes
        fd = os.open(_path(name), os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
        try:
            os.ftruncate(fd, size)
            # reserve the pages now: a too-small /dev/shm fails here (ENOSPC)
            # instead of SIGBUS on the first slot write (as shmring.cpp does)
            os.posix_fallocate(fd, 0, size)
        except OSError:
            os.close(fd)
            os.unlink(_path(name))
            raise
        mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        _HDR.pack_into(mm, 0, 0, 1, nslots, slot_bytes, data_offset)
        self.seg = _Segment(name, fd, mm, True)
        self.seg.states[:] = FREE
        _HDR.pack_into(mm, 0, MAGIC, 1, nslots, slot_bytes, data_offset)
        self._next = 0
        self._published_at = {}
        self.reclaimed = 0

    @property
    def name(self):
        return self.seg.name

    def acquire(self, timeout_s=None, lease_s=None):
        """Claim a free slot for writing.  ``lease_s`` (default: the ring's
        ``lease_s``, 30 s) bounds how long the producer waits before taking
        back the oldest slot no consumer has claimed."""
        if lease_s is None:
            lease_s = self.lease_s
        t0 = time.time()
        n = self.seg.nslots
        while True:
            for k in range(n):
                i = (self._next + k) % n
                w = int(self.seg.states[i])
                if w & 3 == FREE:
                    self.seg.states[i] = (w & ~3) | WRITING
                    self._next = (i + 1) % n
                    return i
            waited = time.time() - t0
            if timeout_s is not None and waited > timeout_s:
                raise TimeoutError('no free shared-memory slot')
            if lease_s is not None and waited > lease_s:
                # reclaim the oldest unclaimed slot (its message was dropped);
                # claimed (held) ones only after a far longer stall (dead consumer)
                ok = (PUBLISHED, HELD) if waited > lease_s * HELD_LEASE_FACTOR else (PUBLISHED,)
                cand = [i for i in range(n) if int(self.seg.states[i]) & 3 in ok]
                if cand:
                    i = min(cand, key=lambda j: self._published_at.get(j, 0.0))
                    w = int(self.seg.states[i])
                    if w & 3 in ok and _cas(self.seg.states, i, w, (w & ~3) | WRITING):
                        self.reclaimed += 1
                        return i
            time.sleep(0.0002)

    def put(self, image):
        """Copy ``image`` (u8 HxW[xC]) into a free slot; returns the descriptor
        fields (slot, byte offset, H, W, C, generation)."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.nbytes > self.seg.slot_bytes:
            raise ValueError('image larger than the ring slot')
        i = self.acquire()
        h, w = img.shape[:2]
        c = img.shape[2] if img.ndim == 3 else 1
        self.seg.slot_array(i, img.shape)[...] = img
        gen = ((int(self.seg.states[i]) >> 2) + 1) & 0x3fffffff
        self._published_at[i] = time.time()
        self.seg.states[i] = _word(gen, PUBLISHED)
        return i, self.seg.data_offset + i * self.seg.slot_bytes, h, w, c, gen

    def put_tile16(self, image, key):
        """Write ``image`` into a free slot as a key-frame delta against ``key``
        (same shape; csrc/codec/tiledelta.h layout: tile count, tile positions,
        payload tiles of 16 rows x 16*C bytes).  Needs H and W multiples of 16
        and slots of :func:`tile16_max_bytes`.  Returns the same fields as
        :meth:`put` plus the number of payload tiles."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape[:2]
        c = img.shape[2] if img.ndim == 3 else 1
        ty, tx = h // TILE, w // TILE
        nt = ty * tx
        f = img.reshape(ty, TILE, tx, TILE, c)
        changed = (f != key.reshape(ty, TILE, tx, TILE, c)).any(axis=(1, 3, 4))     # [ty, tx]
        pos = np.flatnonzero(changed).astype(np.uint32)
        n = len(pos)
        pay = tile16_payload_offset(h, w)
        if pay + n * TILE * TILE * c > self.seg.slot_bytes:
            raise ValueError('tile16 frame larger than the ring slot')
        i = self.acquire()
        off = self.seg.data_offset + i * self.seg.slot_bytes
        hdr = np.frombuffer(self.seg.mm, dtype=np.uint32, count=1 + nt, offset=off)
        hdr[0] = n
        hdr[1:1 + n] = pos
        if n:
            dst = np.frombuffer(self.seg.mm, dtype=np.uint8, count=n * TILE * TILE * c, offset=off + pay)
            dst.reshape(n, TILE, TILE, c)[...] = f.transpose(0, 2, 1, 3, 4)[changed]
        gen = ((int(self.seg.states[i]) >> 2) + 1) & 0x3fffffff
        self._published_at[i] = time.time()
        self.seg.states[i] = _word(gen, PUBLISHED)
        return i, off, h, w, c, gen, n

    def close(self):
        self.seg.close()


def tile16_supported(shape):
    return len(shape) in (2, 3) and shape[0] % TILE == 0 and shape[1] % TILE == 0 and shape[0] > 0 and shape[1] > 0


def tile16_payload_offset(h, w):
    """Byte offset of the first payload tile (count + positions, 256-B aligned)."""
    return (((h // TILE) * (w // TILE) + 1) * 4 + 255) & ~255


def tile16_max_bytes(h, w, c):
    return tile16_payload_offset(h, w) + (h // TILE) * (w // TILE) * TILE * TILE * c


def cleanup_pid(pid):
    """Remove segments a (dead) producer process left behind."""
    prefix = f'blendtorch-{pid}-'
    try:
        for f in os.listdir('/dev/shm'):
            if f.startswith(prefix):
                try:
                    os.unlink('/dev/shm/' + f)
                except OSError:
                    pass
    except OSError:
        pass
