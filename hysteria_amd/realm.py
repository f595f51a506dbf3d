"""Realm hole-punch packets -- ``extras/realm/punch.go`` on MI355X.

=============================================  =============================================
reference (Go)                                 here
=============================================  =============================================
``PunchMetadata{Nonce, Obfs}`` (client.go:52)  ``PunchMetadata(nonce, obfs)`` (hex strings)
``EncodePunchPacket(type, meta)`` (:42-71)     ``encode_punch_packet(type, meta)``
``DecodePunchPacket(packet, meta)`` (:73-100)  ``decode_punch_packet(packet, meta)``
``ErrInvalidPunchPacket`` (:24)                ``InvalidPunchPacketError``
``xorPunchPacket`` mask (:133-141)             ``punch_mask(key, salt)``
``decodePunchPacket`` over all attempts        ``PunchMatcher.match_batch`` (GPU, every
(punch_conn.go:146-165)                        datagram x every attempt in one launch)
=============================================  =============================================

Salt and padding come from ``os.urandom`` (crypto/rand in the reference); the
codec and the SHA-256 mask run in ``libhyobfs.so`` (``include/hyobfs_realm.h``).
"""
from __future__ import annotations

import ctypes
import os
import secrets
from dataclasses import dataclass

import numpy as np

from . import _lib

MAX_PUNCH_PADDING = 1024
PUNCH_SALT_LEN = 8
PUNCH_HEADER_LEN = 25
PUNCH_MIN_WIRE_LEN = PUNCH_SALT_LEN + PUNCH_HEADER_LEN
PUNCH_MAX_WIRE_LEN = PUNCH_MIN_WIRE_LEN + MAX_PUNCH_PADDING
PUNCH_NONCE_SIZE = 16
PUNCH_OBFS_KEY_SIZE = 32
PUNCH_HELLO = 0x01
PUNCH_ACK = 0x02

_REASONS = {-30: "packet too short", -31: "packet too long", -32: "bad magic", -33: "unknown packet type",
            -34: "nonce mismatch"}


class InvalidPunchPacketError(ValueError):
    """ErrInvalidPunchPacket (punch.go:24), with the reason the reference wraps it in."""


class HyobfsPunchAttempt(ctypes.Structure):
    _fields_ = [("nonce", ctypes.c_uint8 * PUNCH_NONCE_SIZE), ("key", ctypes.c_uint8 * PUNCH_OBFS_KEY_SIZE)]


ATTEMPT_DTYPE = np.dtype([("nonce", "u1", (PUNCH_NONCE_SIZE,)), ("key", "u1", (PUNCH_OBFS_KEY_SIZE,))])


def _rlib():
    lib = _lib.load()
    if not getattr(lib, "_realm_declared", False):
        vp, sz, u64, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        ap = ctypes.POINTER(HyobfsPunchAttempt)
        for name, res, args in (
                ("hyobfs_punch_encode", ctypes.c_int64, [ctypes.c_uint8, ap, vp, vp, sz, vp, sz]),
                ("hyobfs_punch_decode", i32, [vp, sz, ap, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(u32)]),
                ("hyobfs_punch_mask", None, [vp, vp, vp]),
                ("hyobfs_punch_match_batch", i32, [vp, vp, vp, u64, vp, u32, vp, vp, vp, vp])):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        lib._realm_declared = True
    return lib


@dataclass(frozen=True)
class PunchMetadata:
    """PunchMetadata (client.go:52-55): hex-encoded 16-byte nonce and 32-byte obfs key."""
    nonce: str
    obfs: str


def new_punch_metadata() -> PunchMetadata:
    """Random metadata as the realm client makes it (client.go:127-139)."""
    return PunchMetadata(secrets.token_hex(PUNCH_NONCE_SIZE), secrets.token_hex(PUNCH_OBFS_KEY_SIZE))


def _decode_hex(name: str, value: str, size: int) -> bytes:
    """decodeHexSize (punch.go:115-124)."""
    if len(value) % 2 or any(c not in "0123456789abcdefABCDEF" for c in value):   # hex.DecodeString
        raise InvalidPunchPacketError(f"invalid punch packet: invalid {name}")
    b = bytes.fromhex(value)
    if len(b) != size:
        raise InvalidPunchPacketError(f"invalid punch packet: invalid {name} length")
    return b


def attempt_of(meta: PunchMetadata) -> HyobfsPunchAttempt:
    """decodePunchMetadata (punch.go:102-113) into the ABI struct."""
    nonce = _decode_hex("nonce", meta.nonce, PUNCH_NONCE_SIZE)
    key = _decode_hex("obfs", meta.obfs, PUNCH_OBFS_KEY_SIZE)
    return HyobfsPunchAttempt((ctypes.c_uint8 * PUNCH_NONCE_SIZE)(*nonce), (ctypes.c_uint8 * PUNCH_OBFS_KEY_SIZE)(*key))


def punch_mask(key: bytes, salt: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    _rlib().hyobfs_punch_mask(bytes(key), bytes(salt), out)
    return out.raw


def random_padding_length() -> int:
    """randomPaddingLength (punch.go:126-131): uniform in [0, 1024]."""
    return secrets.randbelow(MAX_PUNCH_PADDING + 1)


def encode_punch_packet(packet_type: int, meta: PunchMetadata, *, salt: bytes | None = None,
                        padding: bytes | None = None) -> bytes:
    """EncodePunchPacket (punch.go:42-71).  salt/padding default to fresh random bytes."""
    if packet_type not in (PUNCH_HELLO, PUNCH_ACK):
        raise InvalidPunchPacketError("invalid punch packet: unknown packet type")
    a = attempt_of(meta)
    if padding is None:
        padding = os.urandom(random_padding_length())
    if salt is None:
        salt = os.urandom(PUNCH_SALT_LEN)
    out = ctypes.create_string_buffer(PUNCH_MIN_WIRE_LEN + len(padding))
    r = _rlib().hyobfs_punch_encode(packet_type, ctypes.byref(a), bytes(salt), bytes(padding), len(padding), out,
                                    len(out))
    if r < 0:
        if r in _REASONS:
            raise InvalidPunchPacketError(f"invalid punch packet: {_REASONS[r]}")
        _lib.check(int(r), "punch_encode")
    return out.raw[:r]


def decode_punch_packet(packet: bytes, meta: PunchMetadata) -> tuple[int, int]:
    """DecodePunchPacket (punch.go:73-100): (type, padding length).  The length
    checks come before the metadata is parsed, as in the reference."""
    packet = bytes(packet)
    if len(packet) < PUNCH_MIN_WIRE_LEN:
        raise InvalidPunchPacketError("invalid punch packet: packet too short")
    if len(packet) > PUNCH_MAX_WIRE_LEN:
        raise InvalidPunchPacketError("invalid punch packet: packet too long")
    a = attempt_of(meta)
    t, pad = ctypes.c_uint8(), ctypes.c_uint32()
    r = _rlib().hyobfs_punch_decode(packet, len(packet), ctypes.byref(a), ctypes.byref(t), ctypes.byref(pad))
    if r != 0:
        if r in _REASONS:
            raise InvalidPunchPacketError(f"invalid punch packet: {_REASONS[r]}")
        _lib.check(r, "punch_decode")
    return t.value, pad.value


class PunchMatcher:
    """The registered attempts of a punch conn (punch_conn.go:146-165), matched
    against batches of received datagrams on the GPU."""

    def __init__(self, metas):
        self.metas = list(metas)
        arr = np.zeros(len(self.metas), ATTEMPT_DTYPE)
        for j, m in enumerate(self.metas):
            a = attempt_of(m)
            arr[j]["nonce"] = np.frombuffer(bytes(a.nonce), np.uint8)
            arr[j]["key"] = np.frombuffer(bytes(a.key), np.uint8)
        self.attempts = arr

    def match_batch(self, inp, in_off, in_len, n: int, match, ptype=None, padding=None, attempts=None,
                    stream=None) -> None:
        """match[i] = first attempt index datagram i decodes under, or -1 (device tensors).
        ``attempts``: the device copy of ``self.attempts`` (uint8 tensor) -- made by the caller."""
        from .salamander import _ptr, _stream
        _lib.check(_rlib().hyobfs_punch_match_batch(_ptr(inp), _ptr(in_off), _ptr(in_len), n, _ptr(attempts),
                                                    len(self.metas), _ptr(match), _ptr(ptype), _ptr(padding),
                                                    _stream(stream, match)), "punch_match_batch")
