"""Python restatement of Hysteria's Gecko framing, used to check the device path.

TEST INFRASTRUCTURE ONLY.  Only tests/ and ``__graft_entry__.smoke()`` may
import this module, and only as the checker.  The product package
``hysteria_amd`` never imports it.

Restated from the reference (paths relative to apernet/hysteria):

* ``extras/obfs/gecko_frame.go:9-21``   -- flag 0x80, 5-byte header, 2..8 chunks, the two errors
* ``extras/obfs/gecko_frame.go:39-61``  -- ``encodeFrame``: ``0x80 | msgID | idx<<4|total | padLen BE16 | pad | payload``
* ``extras/obfs/gecko_frame.go:65-86``  -- ``decodeFrame``, checks in this order: length, flag, chunk count, index, padding
* ``extras/obfs/gecko.go:107-129``      -- ``writeFragmented``: chunkSize = len/chunks, the last chunk takes the rest
* ``extras/obfs/gecko.go:131-138``      -- ``randomPadLen``
* ``extras/obfs/gecko.go:170-193``      -- ``ReadFrom``: ``n <= 0`` skipped, top bit clear passed through

Randomness (crypto/rand in the reference) is an explicit input here: pad bytes
come from the keyed keystream of ``include/hyobfs_gecko.h`` -- ChaCha with 8
rounds (RFC 8439 block layout), block bytes in column order, pad byte *j* of frame
*i* = keystream byte ``out_off[i] + 13 + j`` -- so with an explicit key the device
output is deterministic and comparable byte for byte.  The block function is
pinned to RFC 8439 section 2.3.2 at 20 rounds (``tests/test_gecko.py``).  The reference's own tests
(``gecko_frame_test.go``, ``gecko_test.go``) check round trips, header fields,
error kinds and size bands, not wire bytes; the same properties are what this
restatement is tested against (``tests/test_gecko.py``).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

from . import salamander_ref as sref

FLAG_FRAGMENT = 0x80
HEADER_LEN = 5
MIN_CHUNKS, MAX_CHUNKS = 2, 8
BUFFER_SIZE = 2048

TRUNCATED, INVALID = "truncated", "invalid"
PASS, FRAGMENT, EMPTY = "pass", "fragment", "empty"


class FrameError(ValueError):
    def __init__(self, kind: str):
        super().__init__(f"gecko frame {kind}")
        self.kind = kind


@dataclass(frozen=True)
class Header:
    pad_len: int
    msg_id: int
    chunk_idx: int
    total_chunks: int


def encode_frame(h: Header, payload: bytes, pad: bytes, cap: int | None = None) -> bytes:
    """gecko_frame.go:39-61 with the pad bytes given."""
    if not MIN_CHUNKS <= h.total_chunks <= MAX_CHUNKS or h.chunk_idx >= h.total_chunks:
        raise FrameError(INVALID)
    needed = HEADER_LEN + h.pad_len + len(payload)
    if cap is not None and cap < needed:
        raise FrameError(TRUNCATED)
    assert len(pad) == h.pad_len
    hdr = bytes([FLAG_FRAGMENT, h.msg_id & 0xFF, (h.chunk_idx << 4 | (h.total_chunks & 0x0F)) & 0xFF,
                 h.pad_len >> 8 & 0xFF, h.pad_len & 0xFF])
    return hdr + pad + bytes(payload)


def decode_frame(buf: bytes) -> tuple[Header, bytes]:
    """gecko_frame.go:65-86."""
    if len(buf) < HEADER_LEN:
        raise FrameError(TRUNCATED)
    if not buf[0] & FLAG_FRAGMENT:
        raise FrameError(INVALID)
    h = Header(pad_len=buf[3] << 8 | buf[4], msg_id=buf[1], chunk_idx=buf[2] >> 4, total_chunks=buf[2] & 0x0F)
    if not MIN_CHUNKS <= h.total_chunks <= MAX_CHUNKS or h.chunk_idx >= h.total_chunks:
        raise FrameError(INVALID)
    if HEADER_LEN + h.pad_len > len(buf):
        raise FrameError(TRUNCATED)
    return h, bytes(buf[HEADER_LEN + h.pad_len:])


def pad_len(min_pkt: int, max_pkt: int, chunk_len: int, rnd: int) -> int:
    """randomPadLen (gecko.go:131-138), randIntn(n) = rnd % n for n > 1 (gecko.go:145-153)."""
    base = sref.SM_SALT_LEN + HEADER_LEN + chunk_len
    lo = max(min_pkt, base)
    if lo > max_pkt:
        return 0
    span = max_pkt - lo + 1
    return lo - base + (0 if span <= 1 else rnd % span)


def split_chunks(msg_len: int, chunks: int) -> list[tuple[int, int]]:
    """(start, end) of each chunk (gecko.go:109-118)."""
    size = msg_len // chunks
    return [(i * size, msg_len if i == chunks - 1 else (i + 1) * size) for i in range(chunks)]


CHACHA_C = (0x61707865, 0x3320646E, 0x79622D32, 0x6B206574)
PAD_ROUNDS = 8


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def chacha_block(key: bytes, counter: int, nonce: bytes, rounds: int = PAD_ROUNDS) -> list[int]:
    """RFC 8439 2.3 block function with ``rounds`` rounds: the 16 output words.  A
    block index past 32 bits folds its high word into nonce word 0
    (include/hyobfs_gecko.h), so the keystream never repeats a block."""
    n0, n1, n2 = struct.unpack("<3I", nonce)
    s = list(CHACHA_C) + list(struct.unpack("<8I", key)) + [counter & 0xFFFFFFFF,
                                                            n0 ^ ((counter >> 32) & 0xFFFFFFFF), n1, n2]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[c], 7)
    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(a + b) & 0xFFFFFFFF for a, b in zip(x, s)]


def keystream(key: bytes, nonce: bytes, start: int, n: int) -> bytes:
    """Pad keystream bytes [start, start + n): block b's bytes 16c..16c+15 are its
    words c, c+4, c+8, c+12 (column order, include/hyobfs_gecko.h)."""
    out = bytearray()
    pos = start
    while len(out) < n:
        blk = pos // 64
        w = chacha_block(key, blk, nonce)
        col = b"".join(struct.pack("<4I", w[c], w[c + 4], w[c + 8], w[c + 12]) for c in range(4))
        take = min(64 - pos % 64, n - len(out))
        out += col[pos % 64:pos % 64 + take]
        pos += take
    return bytes(out)


def pad_bytes(key: bytes, nonce: bytes, wire_off: int, n: int) -> bytes:
    """Pad bytes of the frame whose wire datagram starts at out offset wire_off."""
    return keystream(key, nonce, wire_off + 8 + HEADER_LEN, n)


def encode_wire(psk: bytes, msg: bytes, frames, salts, pad_key: bytes, pad_nonce: bytes, out_off) -> list[bytes]:
    """Wire datagrams of a frame batch: Salamander(encodeFrame(...)).

    frames: iterable of (chunk_off, chunk_len, pad_len, msg_id, idx_total);
    out_off[i]: frame i's offset in the output (it selects its pad keystream)."""
    out = []
    for i, (off, clen, plen, mid, it) in enumerate(frames):
        h = Header(pad_len=plen, msg_id=mid, chunk_idx=it >> 4, total_chunks=it & 0x0F)
        plain = encode_frame(h, msg[off:off + clen], pad_bytes(pad_key, pad_nonce, int(out_off[i]), plen))
        out.append(sref.obfuscate(psk, plain, int(salts[i]).to_bytes(8, "little")))
    return out


def parse(datagram: bytes):
    """ReadFrom's classification of one deobfuscated datagram (gecko.go:176-193)."""
    if len(datagram) == 0:
        return EMPTY, None, None
    if not datagram[0] & FLAG_FRAGMENT:
        return PASS, None, bytes(datagram)
    try:
        h, payload = decode_frame(datagram)
    except FrameError as e:
        return e.kind, None, None
    return FRAGMENT, h, payload
