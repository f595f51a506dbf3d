"""Gecko framing, CPU tier: the C-ABI frame codec (hyobfs_gecko_*_frame, pad_len)
against the reference's own frame tests (extras/obfs/gecko_frame_test.go) and the
oracle restatement (oracle/gecko_ref.py), and the host-side GeckoPacketConn
(hysteria_amd/gecko.py) against the reference's conn tests (gecko_test.go) over
an in-memory lossy packet pipe.  The inner conn here adds/strips an 8-byte
stand-in salt so packet sizes match what a Salamander inner conn puts on the
wire; the real Salamander inner runs in tests/test_gpu_gecko.py."""
import queue
import random
import threading
import time

import numpy as np
import pytest

from hysteria_amd import gecko
from hysteria_amd.gecko import FrameHeader, FrameInvalidError, FrameTruncatedError
from oracle import gecko_ref as gref


# ------------------------------------------------------------ frame codec
def test_encode_decode_frame():
    """TestEncodeDecodeFrame (gecko_frame_test.go:9-42)."""
    payload = bytes([0xA1, 0xB2, 0xC3, 0xD4])
    for total in range(gecko.MIN_FRAGMENT_CHUNKS, gecko.MAX_FRAGMENT_CHUNKS + 1):
        for idx in range(total):
            for pad in (0, 1, 64, 127, 512, 1100):
                h = FrameHeader(pad, 0xA5, idx, total)
                out = gecko.encode_frame(h, payload)
                assert len(out) == gecko.HEADER_LEN + pad + len(payload)
                got, body = gecko.decode_frame(out)
                assert got == h and body == payload
                # the oracle restatement reads the same header and payload
                oh, ob = gref.decode_frame(out)
                assert (oh.pad_len, oh.msg_id, oh.chunk_idx, oh.total_chunks) == (pad, 0xA5, idx, total)
                assert ob == payload
                # and writes the same bytes given the same padding
                assert gref.encode_frame(gref.Header(pad, 0xA5, idx, total), payload,
                                         out[5:5 + pad]) == out


@pytest.mark.parametrize("h", [FrameHeader(0, 0, 0, 0), FrameHeader(0, 0, 0, 1), FrameHeader(0, 0, 0, 9),
                               FrameHeader(0, 0, 4, 4)])
def test_encode_frame_rejects_invalid(h):
    """TestEncodeFrameRejectsInvalid (gecko_frame_test.go:44-66)."""
    with pytest.raises(FrameInvalidError):
        gecko.encode_frame(h, b"\xff", cap=1024)
    with pytest.raises(gref.FrameError) as e:
        gref.encode_frame(gref.Header(h.pad_len, h.msg_id, h.chunk_idx, h.total_chunks), b"\xff", b"")
    assert e.value.kind == gref.INVALID


def test_encode_frame_rejects_short_buffer():
    """TestEncodeFrameRejectsShortBuffer (gecko_frame_test.go:68-75)."""
    with pytest.raises(FrameTruncatedError):
        gecko.encode_frame(FrameHeader(8, 0, 0, 2), b"\x01\x02\x03", cap=5)


@pytest.mark.parametrize("data,kind", [
    (b"", gref.TRUNCATED),
    (bytes([0x80, 0x55, 0x22, 0x00]), gref.TRUNCATED),
    (bytes([0x00, 0x00, 0x22, 0x00, 0x00]), gref.INVALID),
    (bytes([0x80, 0x00, 0x00, 0x00, 0x00]), gref.INVALID),
    (bytes([0x80, 0x00, 0x01, 0x00, 0x00]), gref.INVALID),
    (bytes([0x80, 0x00, 0x09, 0x00, 0x00]), gref.INVALID),
    (bytes([0x80, 0x00, 0x44, 0x00, 0x00]), gref.INVALID),
    (bytes([0x80, 0x00, 0x02, 0x00, 0x12, 0x01, 0x02]), gref.TRUNCATED),
])
def test_decode_frame_rejects_invalid(data, kind):
    """TestDecodeFrameRejectsInvalid (gecko_frame_test.go:77-96)."""
    exc = FrameTruncatedError if kind == gref.TRUNCATED else FrameInvalidError
    with pytest.raises(exc):
        gecko.decode_frame(data)
    with pytest.raises(gref.FrameError) as e:
        gref.decode_frame(data)
    assert e.value.kind == kind


def test_decode_frame_random_bytes_match_oracle():
    rng = np.random.default_rng(7)
    for _ in range(3000):
        n = int(rng.integers(0, 40))
        data = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        if n and rng.random() < 0.7:
            data = bytes([data[0] | 0x80]) + data[1:]
        try:
            oh, ob = gref.decode_frame(data)
            exp = ("ok", (oh.pad_len, oh.msg_id, oh.chunk_idx, oh.total_chunks), ob)
        except gref.FrameError as e:
            exp = (e.kind, None, None)
        try:
            h, b = gecko.decode_frame(data)
            got = ("ok", (h.pad_len, h.msg_id, h.chunk_idx, h.total_chunks), b)
        except FrameTruncatedError:
            got = (gref.TRUNCATED, None, None)
        except FrameInvalidError:
            got = (gref.INVALID, None, None)
        assert got == exp, data.hex()


def test_pad_len_matches_oracle_and_band():
    """randomPadLen (gecko.go:131-138): C ABI vs restatement; datagram in [min, max] when it fits."""
    lib = gecko._glib()
    rng = random.Random(3)
    for _ in range(20000):
        lo = rng.randint(1, 2048)
        hi = rng.randint(lo, 2048)
        chunk = rng.randint(0, 2100)
        rnd = rng.getrandbits(32)
        p = lib.hyobfs_gecko_pad_len(lo, hi, chunk, rnd)
        assert p == gref.pad_len(lo, hi, chunk, rnd)
        size = 8 + 5 + chunk + p
        if 8 + 5 + chunk <= hi:
            assert lo <= size <= hi or (size == 8 + 5 + chunk and size >= lo)
        else:
            assert p == 0


# ------------------------------------------------ in-memory lossy packet pipe
class MemEnd:
    """memEnd (gecko_test.go:18-84): one side of an in-memory packet pipe."""

    def __init__(self, addr):
        self.addr = addr
        self.other = None
        self.inbox = queue.Queue(maxsize=100_000)
        self.write_count = 0
        self.drop_fn = None
        self.closed = threading.Event()
        self._lk = threading.Lock()

    def write_to(self, p, addr):
        with self._lk:
            idx = self.write_count
            self.write_count += 1
        if self.drop_fn is not None and self.drop_fn(idx):
            return len(p)
        self.other.inbox.put((self.addr, bytes(p)))
        return len(p)

    def read_from(self, bufsize=2048):
        while True:
            if self.closed.is_set():
                raise OSError("use of closed network connection")
            try:
                src, data = self.inbox.get(timeout=0.05)
            except queue.Empty:
                continue
            return data[:bufsize], src

    def close(self):
        self.closed.set()

    def local_addr(self):
        return self.addr


def mem_pipe():
    a, b = MemEnd(("127.0.0.1", 1111)), MemEnd(("127.0.0.1", 2222))
    a.other, b.other = b, a
    return a, b


class SaltStandIn:
    """Adds / strips 8 bytes like a Salamander inner conn would (sizes only)."""

    def __init__(self, inner):
        self.inner = inner

    def write_to(self, p, addr):
        self.inner.write_to(b"\0" * 8 + bytes(p), addr)
        return len(p)

    def read_from(self, bufsize=2048):
        while True:
            d, src = self.inner.read_from(bufsize + 8)
            if len(d) > 8:
                return d[8:], src

    def close(self):
        self.inner.close()

    def local_addr(self):
        return self.inner.local_addr()


def wrap(end, lo=gecko.DEFAULT_MIN_PACKET, hi=gecko.DEFAULT_MAX_PACKET):
    return gecko.GeckoPacketConn(SaltStandIn(end), lo, hi)


def quic_long(n, seed=1):
    p = bytearray(random.Random(seed).randbytes(n))
    p[0] = 0xC0
    return bytes(p)


def quic_short(n, seed=2):
    p = bytearray(random.Random(seed).randbytes(n))
    p[0] = 0x40
    return bytes(p)


def read_with_timeout(conn, timeout=5.0):
    box = {}

    def run():
        try:
            box["r"] = conn.read_from(4096)
        except Exception as e:  # noqa: BLE001
            box["e"] = e
    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(timeout)
    if "r" not in box:
        raise AssertionError(f"read_from did not return: {box.get('e')}")
    return box["r"]


def test_round_trip_short_header():
    """TestGeckoRoundTripShortHeader (gecko_test.go:121-152): one wire datagram."""
    a, b = mem_pipe()
    ga, gb = wrap(a), wrap(b)
    p = quic_short(400)
    ga.write_to(p, b.addr)
    assert a.write_count == 1
    got, src = read_with_timeout(gb)
    assert got == p and src == a.addr
    ga.close(), gb.close()


def test_round_trip_long_header():
    """TestGeckoRoundTripLongHeader (gecko_test.go:154-182): 2..8 wire datagrams."""
    a, b = mem_pipe()
    ga, gb = wrap(a), wrap(b)
    p = quic_long(1200)
    ga.write_to(p, b.addr)
    assert gecko.MIN_FRAGMENT_CHUNKS <= a.write_count <= gecko.MAX_FRAGMENT_CHUNKS
    assert read_with_timeout(gb)[0] == p
    ga.close(), gb.close()


@pytest.mark.parametrize("size", [1, 2, 5, 10, 15, 20, 25, 27, 30, 40, 64, 128])
def test_round_trip_small_long_header(size):
    """TestGeckoRoundTripSmallLongHeader (gecko_test.go:184-212)."""
    a, b = mem_pipe()
    ga, gb = wrap(a), wrap(b)
    p = quic_long(size)
    ga.write_to(p, b.addr)
    assert read_with_timeout(gb)[0] == p
    ga.close(), gb.close()


def test_write_fragmented_never_fails():
    """TestGeckoWriteFragmentedNeverPanics (gecko_test.go:214-232)."""
    a, b = mem_pipe()
    g = wrap(a)
    for size in range(1, 65):
        assert g.write_to(quic_long(size), b.addr) == size
    g.close()


def test_reassembles_out_of_order():
    """TestGeckoReassemblesOutOfOrder (gecko_test.go:234-284): frames fed in reverse."""
    a, b = mem_pipe()
    ga = wrap(a)
    p = quic_long(900)
    ga.write_to(p, b.addr)
    pkts = [b.inbox.get_nowait() for _ in range(a.write_count)]
    c, d = mem_pipe()
    gd = wrap(d)
    for pk in reversed(pkts):
        d.inbox.put(pk)
    assert read_with_timeout(gd)[0] == p
    ga.close(), gd.close()


def test_expires_incomplete_fragment():
    """TestGeckoExpiresIncompleteFragment (gecko_test.go:286-348)."""
    a, b = mem_pipe()
    a.drop_fn = lambda i: i == 0
    ga, gb = wrap(a), wrap(b)
    ga.write_to(quic_long(900), b.addr)
    t = threading.Thread(target=lambda: _swallow(gb), daemon=True)
    t.start()
    deadline = time.time() + 2
    while time.time() < deadline:
        with gb.mu:
            if gb.reassembly:
                break
        time.sleep(0.005)
    with gb.mu:
        assert gb.reassembly, "expected at least one reassembly entry"
    gb.gc_expired(time.monotonic() + gecko.REASSEMBLY_TTL + 1)
    with gb.mu:
        assert not gb.reassembly and not gb.per_source
    gb.close()
    t.join(2)


def _swallow(conn):
    try:
        while True:
            conn.read_from(4096)
    except OSError:
        pass


def test_enforces_per_source_cap():
    """TestGeckoEnforcesPerSourceCap (gecko_test.go:350-389)."""
    a, b = mem_pipe()
    a.drop_fn = lambda i: i > 0 and i % 2 == 0
    ga, gb = wrap(a), wrap(b)
    t = threading.Thread(target=lambda: _swallow(gb), daemon=True)
    t.start()
    for _ in range(gecko.MAX_PER_SOURCE + 5):
        ga.write_to(quic_long(1200), b.addr)
    time.sleep(0.3)
    with gb.mu:
        assert gb.per_source.get(str(a.addr), 0) <= gecko.MAX_PER_SOURCE
    gb.close()
    t.join(2)


def test_evicts_oldest_on_global_cap():
    """TestGeckoEvictsOldestOnGlobalCap (gecko_test.go:391-423)."""
    g = gecko.GeckoPacketConn(None)
    now = time.monotonic()
    for i in range(gecko.MAX_REASSEMBLY):
        k = (f"src-{i}", 1)
        g.reassembly[k] = gecko._Entry([None] * 4, 0, 4, now + i * 1e-3)
        g.per_source[k[0]] = g.per_source.get(k[0], 0) + 1
    with g.mu:
        g.evict_oldest_locked()
    assert len(g.reassembly) == gecko.MAX_REASSEMBLY - 1
    assert ("src-0", 1) not in g.reassembly
    assert g.per_source.get("src-0", 0) == 0
    g.close()


def test_bounded_under_garbage_flood():
    """TestGeckoBoundedUnderGarbageFlood (gecko_test.go:425-470), 20k datagrams."""
    a, b = mem_pipe()
    gb = wrap(b)
    rng = random.Random(42)
    for i in range(20_000):
        junk = b"\0" * 8 + rng.randbytes(16 + rng.randrange(200))
        b.inbox.put(((f"10.0.0.{i % 256}", 1024 + i % 4096), junk))
    t = threading.Thread(target=lambda: _swallow(gb), daemon=True)
    t.start()
    deadline = time.time() + 30
    while b.inbox.qsize() and time.time() < deadline:
        time.sleep(0.02)
    with gb.mu:
        assert len(gb.reassembly) <= gecko.MAX_REASSEMBLY
    gb.close()
    t.join(2)


def test_requires_password():
    """TestGeckoRequiresPassword (gecko_test.go:505-509): no device or socket touched."""
    with pytest.raises(gecko.GeckoError):
        gecko.wrap_packet_conn_gecko(None, gecko.GeckoOptions())


@pytest.mark.parametrize("opts", [gecko.GeckoOptions(b"x", 1000, 500), gecko.GeckoOptions(b"x", -1, 0),
                                  gecko.GeckoOptions(b"x", 0, gecko.BUFFER_SIZE + 1)])
def test_rejects_invalid_packet_size(opts):
    """TestGeckoRejectsInvalidPacketSize (gecko_test.go:511-524)."""
    with pytest.raises(gecko.GeckoError):
        gecko.wrap_packet_conn_gecko(None, opts)


def test_padding_within_bounds():
    """TestGeckoPaddingWithinBounds (gecko_test.go:526-565): every fragment's wire size in [400, 900]."""
    a, b = mem_pipe()
    ga = wrap(a, 400, 900)
    for size in (1, 50, 200, 600, 1200):
        ga.write_to(quic_long(size), b.addr)
    n = 0
    while not b.inbox.empty():
        _, d = b.inbox.get_nowait()
        assert 400 <= len(d) <= 900, len(d)
        n += 1
    assert n >= 10
    ga.close()


def test_non_udp_inner_is_unsupported():
    """TestGeckoNonUDPInnerReturnsUnsupported (gecko_test.go:567-586)."""
    a, _ = mem_pipe()
    g = wrap(a)
    for f in (g.fileno, lambda: g.set_read_buffer(1 << 20), lambda: g.set_write_buffer(1 << 20)):
        with pytest.raises(gecko.UnsupportedError):
            f()
    g.close()


# ------------------------------------------------------------ batch planning
def test_plan_fragments_covers_messages_in_band():
    lens = [1, 5, 27, 64, 300, 900, 1200, 1350, 2000]
    fr, off, total = gecko.plan_fragments(lens, 400, 900, first_msg_id=250)
    base = np.concatenate([[0], np.cumsum(lens)])
    i = 0
    for m, L in enumerate(lens):
        total_chunks = int(fr[i]["idx_total"]) & 0x0F
        assert 2 <= total_chunks <= 8
        got = []
        for k in range(total_chunks):
            f = fr[i + k]
            assert int(f["idx_total"]) == (k << 4) | total_chunks
            assert int(f["msg_id"]) == (250 + m) & 0xFF
            got.append((int(f["chunk_off"]) - base[m], int(f["chunk_len"])))
            size = 13 + int(f["chunk_len"]) + int(f["pad_len"])
            assert size <= 900 or int(f["pad_len"]) == 0
            assert size >= 400 or 13 + int(f["chunk_len"]) > 900
        assert got == [(s, e - s) for s, e in gref.split_chunks(L, total_chunks)]
        i += total_chunks
    assert i == len(fr)
    widths = 13 + fr["chunk_len"].astype(np.uint64) + fr["pad_len"]
    assert np.array_equal(off[1:], np.cumsum(widths)[:-1]) and total == int(widths.sum())


def test_pad_keystream_block_pinned_to_rfc8439():
    """The Gecko padding keystream (include/hyobfs_gecko.h) is the RFC 8439 ChaCha
    block with 8 rounds and column-ordered bytes.  At 20 rounds the same block
    function gives RFC 8439 2.3.2's test vector (row order), so only the round
    count and the byte order differ from the published function."""
    import struct
    from oracle import gecko_ref as gref
    key, nonce = bytes(range(32)), bytes.fromhex("000000090000004a00000000")
    w = gref.chacha_block(key, 1, nonce, rounds=20)
    assert struct.pack("<16I", *w).hex() == (
        "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
        "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")
    w8 = gref.chacha_block(key, 1, nonce)
    col = b"".join(struct.pack("<4I", w8[c], w8[c + 4], w8[c + 8], w8[c + 12]) for c in range(4))
    assert gref.keystream(key, nonce, 64, 64) == col
    assert gref.keystream(key, nonce, 70, 20) == col[6:26]
