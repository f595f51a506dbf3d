"""Gecko shape obfuscation -- ``extras/obfs/gecko.go`` + ``gecko_frame.go`` on MI355X.

Gecko sits on top of a Salamander packet connection.  QUIC long-header
(handshake) packets are split into 2..8 chunks, each sent as its own frame
``0x80 | msgID | idx<<4|total | padLen | pad | chunk`` padded so the wire
datagram lands in ``[min_pkt, max_pkt]``; short-header packets pass through.

=============================================  ==============================================
reference (Go)                                 here
=============================================  ==============================================
``GeckoOptions`` (gecko.go:28-32)              ``GeckoOptions``
``WrapPacketConnGecko`` (gecko.go:34-55)       ``wrap_packet_conn_gecko(sock, opts)``
``newGeckoPacketConn`` (gecko.go:83-95)        ``GeckoPacketConn(inner, min_pkt, max_pkt)``
``WriteTo`` / ``writeFragmented`` (:99-129)    ``write_to(p, addr)``
``ReadFrom`` / ``acceptChunk`` (:157-250)      ``read_from(bufsize)`` / ``accept_chunk``
``gcLoop`` / ``gcExpired`` (:254-275)          background thread / ``gc_expired(now)``
``evictOldestLocked`` (:291-307)               ``evict_oldest_locked()``
``encodeFrame`` / ``decodeFrame``              ``encode_frame`` / ``decode_frame`` (C ABI)
``randomPadLen`` / ``randIntn`` (:131-153)     ``random_pad_len`` / ``rand_intn``
(new) one device pass over many frames         ``plan_fragments`` + ``encode_batch`` (GPU)
(new) device parse of received datagrams       ``parse_batch`` (GPU)
=============================================  ==============================================

The frame codec and the device batch calls go through ``include/hyobfs_gecko.h``
(``libhyobfs.so``); reassembly state stays on the host, as in the reference.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check

FLAG_FRAGMENT = 0x80
HEADER_LEN = 5
MIN_FRAGMENT_CHUNKS = 2
MAX_FRAGMENT_CHUNKS = 8
REASSEMBLY_TTL = 8.0          # seconds
MAX_REASSEMBLY = 4096
MAX_PER_SOURCE = 8
BUFFER_SIZE = 2048
DEFAULT_MIN_PACKET = 512
DEFAULT_MAX_PACKET = 1200
SALT_LEN = 8

ERR_TRUNCATED = -20
ERR_INVALID = -21
PASS, FRAGMENT, EMPTY = 0, 1, -22


class FrameTruncatedError(ValueError):
    """errFrameTruncated (gecko_frame.go:19)."""


class FrameInvalidError(ValueError):
    """errFrameInvalid (gecko_frame.go:20)."""


class GeckoError(ValueError):
    """Construction errors of WrapPacketConnGecko (gecko.go:35-47)."""


class UnsupportedError(OSError):
    """errors.ErrUnsupported: the inner conn is not UDP-like (gecko.go:320-341)."""


class HyobfsGeckoHeader(ctypes.Structure):
    _fields_ = [("pad_len", ctypes.c_uint16), ("msg_id", ctypes.c_uint8), ("chunk_idx", ctypes.c_uint8),
                ("total_chunks", ctypes.c_uint8), ("reserved_", ctypes.c_uint8 * 3)]


class HyobfsGeckoBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("msg", ctypes.c_void_p), ("frames", ctypes.c_void_p),
                ("salts", ctypes.c_void_p), ("pad_key", ctypes.c_uint8 * 32), ("pad_nonce", ctypes.c_uint8 * 12),
                ("reserved_", ctypes.c_uint32), ("out", ctypes.c_void_p),
                ("out_off", ctypes.c_void_p), ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_uint64),
                ("out_cap", ctypes.c_uint64)]


# struct hyobfs_gecko_frame / hyobfs_gecko_parsed as numpy records (16 bytes each)
FRAME_DTYPE = np.dtype([("chunk_off", "<u8"), ("chunk_len", "<u4"), ("pad_len", "<u2"), ("msg_id", "u1"),
                        ("idx_total", "u1")])
PARSED_DTYPE = np.dtype([("status", "<i4"), ("pad_len", "<u2"), ("msg_id", "u1"), ("idx_total", "u1"),
                         ("payload_off", "<u4"), ("payload_len", "<u4")])
assert FRAME_DTYPE.itemsize == 16 and PARSED_DTYPE.itemsize == 16


def _glib(lib=None):
    lib = lib or _lib.load()
    if not getattr(lib, "_gecko_declared", False):
        vp, sz, u64, i32, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32
        hp = ctypes.POINTER(HyobfsGeckoHeader)
        for name, res, args in (
                ("hyobfs_gecko_encode_frame", ctypes.c_int64, [hp, vp, sz, vp, sz]),
                ("hyobfs_gecko_decode_frame", i32, [vp, sz, hp, ctypes.POINTER(sz)]),
                ("hyobfs_gecko_pad_len", u32, [i32, i32, u32, u32]),
                ("hyobfs_gecko_workspace_size", u64, [u64]),
                ("hyobfs_gecko_encode_batch", i32, [vp, ctypes.POINTER(HyobfsGeckoBatch), vp]),
                ("hyobfs_gecko_parse_batch", i32, [vp, vp, vp, u64, vp, vp]),
                ("hyobfs_gecko_random_pad_key", i32, [vp, vp])):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        lib._gecko_declared = True
    return lib


@dataclass(frozen=True)
class FrameHeader:
    """frameHeader (gecko_frame.go:30-35)."""
    pad_len: int
    msg_id: int
    chunk_idx: int
    total_chunks: int


def encode_frame(h: FrameHeader, payload: bytes, cap: int | None = None) -> bytes:
    """encodeFrame (gecko_frame.go:39-61): header, pad_len random bytes, payload."""
    payload = bytes(payload)
    need = HEADER_LEN + h.pad_len + len(payload)
    cap = need if cap is None else cap
    out = ctypes.create_string_buffer(max(cap, 1))
    ch = HyobfsGeckoHeader(pad_len=h.pad_len, msg_id=h.msg_id & 0xFF, chunk_idx=h.chunk_idx & 0xFF,
                           total_chunks=h.total_chunks & 0xFF)
    r = _glib().hyobfs_gecko_encode_frame(ctypes.byref(ch), payload, len(payload), out, cap)
    if r == ERR_INVALID:
        raise FrameInvalidError("gecko frame invalid")
    if r == ERR_TRUNCATED:
        raise FrameTruncatedError("gecko frame truncated")
    check(int(r) if r < 0 else 0, "encode_frame")
    return out.raw[:r]


def decode_frame(buf: bytes) -> tuple[FrameHeader, bytes]:
    """decodeFrame (gecko_frame.go:65-86): (header, payload)."""
    buf = bytes(buf)
    h = HyobfsGeckoHeader()
    off = ctypes.c_size_t()
    r = _glib().hyobfs_gecko_decode_frame(buf, len(buf), ctypes.byref(h), ctypes.byref(off))
    if r == ERR_INVALID:
        raise FrameInvalidError("gecko frame invalid")
    if r == ERR_TRUNCATED:
        raise FrameTruncatedError("gecko frame truncated")
    check(r, "decode_frame")
    return FrameHeader(h.pad_len, h.msg_id, h.chunk_idx, h.total_chunks), buf[off.value:]


def rand_intn(n: int) -> int:
    """randIntn (gecko.go:145-153): uniform in [0, n) from 4 random bytes, big-endian, mod n."""
    if n <= 1:
        return 0
    return int.from_bytes(os.urandom(4), "big") % n


def random_fragment_chunks() -> int:
    """randomFragmentChunks (gecko.go:140-142)."""
    return MIN_FRAGMENT_CHUNKS + rand_intn(MAX_FRAGMENT_CHUNKS - MIN_FRAGMENT_CHUNKS + 1)


def random_pad_len(min_pkt: int, max_pkt: int, chunk_len: int) -> int:
    """randomPadLen (gecko.go:131-138), through the C ABI with 4 random bytes."""
    return int(_glib().hyobfs_gecko_pad_len(min_pkt, max_pkt, chunk_len, int.from_bytes(os.urandom(4), "big")))


def chunk_bounds(msg_len: int, chunks: int) -> list[tuple[int, int]]:
    """writeFragmented's chunking (gecko.go:109-118): len/chunks each, the last takes the rest."""
    size = msg_len // chunks
    return [(i * size, msg_len if i == chunks - 1 else (i + 1) * size) for i in range(chunks)]


@dataclass
class GeckoOptions:
    """GeckoOptions (gecko.go:28-32)."""
    password: bytes = b""
    min_packet_size: int = 0
    max_packet_size: int = 0


def _validate(opts: GeckoOptions) -> tuple[int, int]:
    if not opts.password:
        raise GeckoError("gecko: password is required")
    lo = opts.min_packet_size or DEFAULT_MIN_PACKET
    hi = opts.max_packet_size or DEFAULT_MAX_PACKET
    if lo <= 0 or lo > hi or hi > BUFFER_SIZE:
        raise GeckoError("gecko: invalid min/max packet size")
    return lo, hi


@dataclass
class _Entry:
    chunks: list
    received: int
    total: int
    deadline: float


class GeckoPacketConn:
    """geckoPacketConn (gecko.go:69-95) over an inner packet conn with
    ``write_to(p, addr)`` / ``read_from(bufsize) -> (payload, addr)`` / ``close()``."""

    def __init__(self, inner, min_pkt: int = DEFAULT_MIN_PACKET, max_pkt: int = DEFAULT_MAX_PACKET):
        self.inner = inner
        self.min_pkt, self.max_pkt = min_pkt, max_pkt
        self._msg_id = 0
        self._msg_lock = threading.Lock()
        self._read_lock = threading.Lock()
        self.mu = threading.Lock()
        self.reassembly: dict[tuple[str, int], _Entry] = {}
        self.per_source: dict[str, int] = {}
        self._closed = threading.Event()
        self._gc = threading.Thread(target=self._gc_loop, daemon=True)
        self._gc.start()

    # ---------------------------------------------------------------- send
    def write_to(self, p, addr) -> int:
        """WriteTo (gecko.go:99-110)."""
        p = bytes(p)
        if len(p) == 0:
            return 0
        if p[0] & 0x80:
            return self._write_fragmented(p, addr)
        return self.inner.write_to(p, addr)

    def _next_msg_id(self) -> int:
        with self._msg_lock:
            self._msg_id = (self._msg_id + 1) & 0xFFFFFFFF
            return self._msg_id & 0xFF

    def _write_fragmented(self, p: bytes, addr) -> int:
        """writeFragmented (gecko.go:112-129)."""
        chunks = random_fragment_chunks()
        msg_id = self._next_msg_id()
        for i, (s, e) in enumerate(chunk_bounds(len(p), chunks)):
            chunk = p[s:e]
            pad = random_pad_len(self.min_pkt, self.max_pkt, len(chunk))
            frame = encode_frame(FrameHeader(pad, msg_id, i, chunks), chunk)
            self.inner.write_to(frame, addr)
        return len(p)

    # ------------------------------------------------------------- receive
    def read_from(self, bufsize: int = BUFFER_SIZE):
        """ReadFrom (gecko.go:157-193): returns (payload, addr)."""
        with self._read_lock:
            while True:
                buf, addr = self.inner.read_from(BUFFER_SIZE)
                if len(buf) <= 0:
                    continue
                if not buf[0] & 0x80:
                    return bytes(buf[:bufsize]), addr
                try:
                    h, payload = decode_frame(buf)
                except (FrameTruncatedError, FrameInvalidError):
                    continue   # malformed frame: dropped silently
                out = self.accept_chunk(addr, h, payload)
                if out is None:
                    continue
                return out[:bufsize], addr

    def accept_chunk(self, addr, h: FrameHeader, payload: bytes):
        """acceptChunk (gecko.go:195-250): the reassembled message, or None."""
        key = (str(addr), h.msg_id)
        with self.mu:
            e = self.reassembly.get(key)
            if e is None:
                if self.per_source.get(key[0], 0) >= MAX_PER_SOURCE:
                    return None
                if len(self.reassembly) >= MAX_REASSEMBLY:
                    self.evict_oldest_locked()
                e = _Entry([None] * h.total_chunks, 0, h.total_chunks, time.monotonic() + REASSEMBLY_TTL)
                self.reassembly[key] = e
                self.per_source[key[0]] = self.per_source.get(key[0], 0) + 1
            elif e.total != h.total_chunks:
                return None   # inconsistent chunk count
            if h.chunk_idx >= len(e.chunks) or e.chunks[h.chunk_idx] is not None:
                return None   # bad index or duplicate
            e.chunks[h.chunk_idx] = bytes(payload)
            e.received += 1
            if e.received < e.total:
                return None
            out = b"".join(e.chunks)
            self.drop_entry_locked(key)
            return out

    # --------------------------------------------------------- maintenance
    def _gc_loop(self) -> None:
        while not self._closed.wait(REASSEMBLY_TTL / 2):
            self.gc_expired(time.monotonic())

    def gc_expired(self, now: float) -> None:
        """gcExpired (gecko.go:265-275); ``now`` on the time.monotonic() clock."""
        with self.mu:
            for k in [k for k, e in self.reassembly.items() if now > e.deadline]:
                self.drop_entry_locked(k)

    def drop_entry_locked(self, k) -> None:
        if self.reassembly.pop(k, None) is None:
            return
        n = self.per_source.get(k[0], 0) - 1
        if n <= 0:
            self.per_source.pop(k[0], None)
        else:
            self.per_source[k[0]] = n

    def evict_oldest_locked(self) -> None:
        """evictOldestLocked (gecko.go:291-307): drop the entry with the earliest deadline."""
        if self.reassembly:
            k = min(self.reassembly, key=lambda k: self.reassembly[k].deadline)
            self.drop_entry_locked(k)

    # ---------------------------------------------------------- boilerplate
    def close(self) -> None:
        self._closed.set()
        if self.inner is not None:
            self.inner.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def local_addr(self):
        return self.inner.local_addr()

    def _udp(self, name):
        f = getattr(self.inner, name, None)
        if f is None:
            raise UnsupportedError("unsupported operation")
        return f

    def fileno(self) -> int:
        return self._udp("fileno")()

    def set_read_buffer(self, nbytes: int) -> None:
        self._udp("set_read_buffer")(nbytes)

    def set_write_buffer(self, nbytes: int) -> None:
        self._udp("set_write_buffer")(nbytes)


def wrap_packet_conn_gecko(sock, opts: GeckoOptions, device: int = 0) -> GeckoPacketConn:
    """WrapPacketConnGecko (gecko.go:34-55): options checked before any device work."""
    lo, hi = _validate(opts)
    from .conn import wrap_packet_conn_salamander
    inner = wrap_packet_conn_salamander(sock, opts.password, device)
    return GeckoPacketConn(inner, lo, hi)


# ------------------------------------------------------------- device batches
def plan_fragments(msg_lens, min_pkt: int = DEFAULT_MIN_PACKET, max_pkt: int = DEFAULT_MAX_PACKET,
                   first_msg_id: int = 1, rand32=None):
    """Frames for a batch of long-header messages laid back to back in one buffer,
    as writeFragmented would send them (gecko.go:112-129).

    rand32(k) -> k uniform uint32 values (default: os.urandom).  Returns
    (frames: FRAME_DTYPE array, out_off: uint64 array of packed wire offsets, total wire bytes)."""
    if rand32 is None:
        def rand32(k):
            return np.frombuffer(os.urandom(4 * k), ">u4").astype(np.uint64)
    lib = _glib()
    frames = []
    off = 0
    for m, L in enumerate(msg_lens):
        r = rand32(1 + MAX_FRAGMENT_CHUNKS)
        chunks = MIN_FRAGMENT_CHUNKS + int(r[0] % (MAX_FRAGMENT_CHUNKS - MIN_FRAGMENT_CHUNKS + 1))
        mid = (first_msg_id + m) & 0xFF
        for i, (s, e) in enumerate(chunk_bounds(int(L), chunks)):
            pad = int(lib.hyobfs_gecko_pad_len(min_pkt, max_pkt, e - s, int(r[1 + i])))
            frames.append((off + s, e - s, pad, mid, (i << 4) | chunks))
        off += int(L)
    fr = np.array(frames, dtype=FRAME_DTYPE)
    widths = SALT_LEN + HEADER_LEN + fr["pad_len"].astype(np.uint64) + fr["chunk_len"].astype(np.uint64)
    out_off = np.zeros(len(fr), np.uint64)
    if len(fr):
        np.cumsum(widths[:-1], out=out_off[1:])
    return fr, out_off, int(widths.sum())


def workspace_size(n: int) -> int:
    return int(_glib().hyobfs_gecko_workspace_size(n))


def random_pad_key() -> tuple[bytes, bytes]:
    """A fresh (key, nonce) for the padding keystream from the OS (hyobfs_gecko_random_pad_key,
    getrandom: the source of the reference's crypto/rand)."""
    key, nonce = ctypes.create_string_buffer(32), ctypes.create_string_buffer(12)
    check(_glib().hyobfs_gecko_random_pad_key(key, nonce), "random_pad_key")
    return key.raw, nonce.raw


def encode_batch(obfuscator, *, msg, frames, salts, out, out_off, pad_key: bytes | None = None,
                 pad_nonce: bytes | None = None, workspace=None, n=None, stream=None) -> None:
    """hyobfs_gecko_encode_batch: every frame's wire datagram in one device pass.
    Arguments are device tensors (torch) or device pointers; ``workspace`` is accepted
    and ignored (ABI 3: no scratch).  Padding is a keyed keystream
    (include/hyobfs_gecko.h): a fresh OS-random key per call unless pad_key and
    pad_nonce are given (reproducible output for tests)."""
    from .salamander import _ptr, _stream
    if n is None:   # frames: 16-byte hyobfs_gecko_frame records
        n = frames.numel() * frames.element_size() // FRAME_DTYPE.itemsize if hasattr(frames, "numel") else len(frames)
    if pad_key is None or pad_nonce is None:
        pad_key, pad_nonce = random_pad_key()
    if len(pad_key) != 32 or len(pad_nonce) != 12:
        raise ValueError("pad_key must be 32 bytes and pad_nonce 12")
    b = HyobfsGeckoBatch(n=n, msg=_ptr(msg), frames=_ptr(frames), salts=_ptr(salts),
                         pad_key=(ctypes.c_uint8 * 32).from_buffer_copy(pad_key),
                         pad_nonce=(ctypes.c_uint8 * 12).from_buffer_copy(pad_nonce),
                         out=_ptr(out), out_off=_ptr(out_off))
    lib = _glib(getattr(obfuscator, "_lib", None))   # the library the context came from
    check(lib.hyobfs_gecko_encode_batch(obfuscator._h, ctypes.byref(b), _stream(stream, out)), "gecko_encode_batch")


def parse_batch(inp, in_off, in_len, n: int, out, stream=None) -> None:
    """hyobfs_gecko_parse_batch: classify n deobfuscated device datagrams into ``out``
    (PARSED_DTYPE records, 16 bytes each)."""
    from .salamander import _ptr, _stream
    check(_glib().hyobfs_gecko_parse_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), n, _ptr(out),
                                           _stream(stream, out)), "gecko_parse_batch")
