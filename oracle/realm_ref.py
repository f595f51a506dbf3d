"""Python restatement of the realm hole-punch packet codec, used to check the device path.

TEST INFRASTRUCTURE ONLY.  Only tests/ may import this module, and only as the
checker.  The product package ``hysteria_amd`` never imports it.

Restated from the reference (paths relative to apernet/hysteria):

* ``extras/realm/punch.go:13-31``   -- 8-byte salt, 25-byte header, padding 0..1024, magic ``HYRLMv1\\0``
* ``extras/realm/punch.go:42-71``   -- ``EncodePunchPacket``: ``salt || (magic | type | nonce | padding) ^ mask``
* ``extras/realm/punch.go:73-100``  -- ``DecodePunchPacket``: length, magic, type, nonce checks in that order
* ``extras/realm/punch.go:133-141`` -- ``xorPunchPacket``: mask = SHA-256(obfsKey || salt), ``mask[i % 32]``
* ``extras/realm/punch_conn.go:146-165`` -- every registered attempt is tried on every packet

SHA-256 is CPython's ``hashlib.sha256``, independent of the HIP and C code.  The
reference's tests (``punch_test.go``) pin behaviour, not bytes; the tests here
check this restatement against those behaviours and the device against it.
"""
from __future__ import annotations

import hashlib

SALT_LEN = 8
HEADER_LEN = 25
MAX_PADDING = 1024
MIN_WIRE = SALT_LEN + HEADER_LEN
MAX_WIRE = MIN_WIRE + MAX_PADDING
MAGIC = b"HYRLMv1\x00"
HELLO, ACK = 0x01, 0x02
TOO_SHORT, TOO_LONG, BAD_MAGIC, UNKNOWN_TYPE, NONCE_MISMATCH = (
    "too short", "too long", "bad magic", "unknown type", "nonce mismatch")


class PunchError(ValueError):
    def __init__(self, reason: str):
        super().__init__(f"invalid punch packet: {reason}")
        self.reason = reason


def mask(key: bytes, salt: bytes) -> bytes:
    return hashlib.sha256(bytes(key) + bytes(salt)).digest()


def _xor(data: bytes, m: bytes) -> bytes:
    return bytes(b ^ m[i % 32] for i, b in enumerate(data))


def encode(ptype: int, nonce: bytes, key: bytes, salt: bytes, padding: bytes) -> bytes:
    if ptype not in (HELLO, ACK):
        raise PunchError(UNKNOWN_TYPE)
    plain = MAGIC + bytes([ptype]) + bytes(nonce) + bytes(padding)
    return bytes(salt) + _xor(plain, mask(key, salt))


def decode(packet: bytes, nonce: bytes, key: bytes) -> tuple[int, int]:
    """(type, padding length) or PunchError."""
    if len(packet) < MIN_WIRE:
        raise PunchError(TOO_SHORT)
    if len(packet) > MAX_WIRE:
        raise PunchError(TOO_LONG)
    salt = packet[:SALT_LEN]
    plain = _xor(packet[SALT_LEN:], mask(key, salt))
    if plain[:8] != MAGIC:
        raise PunchError(BAD_MAGIC)
    if plain[8] not in (HELLO, ACK):
        raise PunchError(UNKNOWN_TYPE)
    if plain[9:HEADER_LEN] != bytes(nonce):
        raise PunchError(NONCE_MISMATCH)
    return plain[8], len(plain) - HEADER_LEN


def match(packet: bytes, attempts) -> tuple[int, int, int]:
    """(attempt index, type, padding) of the first attempt the packet decodes under, or (-1, 0, 0)."""
    for j, (nonce, key) in enumerate(attempts):
        try:
            t, pad = decode(packet, nonce, key)
        except PunchError:
            continue
        return j, t, pad
    return -1, 0, 0
