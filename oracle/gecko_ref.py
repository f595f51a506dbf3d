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
come from the SplitMix64 stream of ``include/hyobfs_gecko.h`` (byte ``i*2048+5+j``
of stream ``pad_seed`` for pad byte *j* of frame *i*), so device output is
deterministic and comparable byte for byte.  The reference's own tests
(``gecko_frame_test.go``, ``gecko_test.go``) check round trips, header fields,
error kinds and size bands, not wire bytes; the same properties are what this
restatement is tested against (``tests/test_gecko.py``).
"""
from __future__ import annotations

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


def pad_bytes(pad_seed: int, frame: int, n: int) -> bytes:
    """Pad bytes of frame i: bytes i*2048 + 5 + j (plaintext positions) of the stream."""
    return sref.stream_bytes(pad_seed, frame * BUFFER_SIZE + HEADER_LEN, n)


def encode_wire(psk: bytes, msg: bytes, frames, salts, pad_seed: int) -> list[bytes]:
    """Wire datagrams of a frame batch: Salamander(encodeFrame(...)).

    frames: iterable of (chunk_off, chunk_len, pad_len, msg_id, idx_total)."""
    out = []
    for i, (off, clen, plen, mid, it) in enumerate(frames):
        h = Header(pad_len=plen, msg_id=mid, chunk_idx=it >> 4, total_chunks=it & 0x0F)
        plain = encode_frame(h, msg[off:off + clen], pad_bytes(pad_seed, i, plen))
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
