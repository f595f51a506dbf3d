"""Gecko on the GPU: the one-pass frame encode kernel and the parse kernel
(include/hyobfs_gecko.h) against oracle/gecko_ref.py, reassembly of the parsed
fragments through the host GeckoPacketConn, and the full Gecko-over-Salamander
packet conn on a loopback UDP socket (gecko.go:34-55, gecko_test.go round trips)."""
import random
import socket

import numpy as np
import pytest

from oracle import gecko_ref as gref
from oracle import salamander_ref as sref

pytestmark = pytest.mark.gpu
PSK = b"average_password"
KEY, NONCE = bytes(range(7, 39)), bytes(range(100, 112))   # explicit pad keystream key: reproducible wire


def _dev(a, gpu):
    import torch
    return torch.from_numpy(np.array(a, copy=True).view(np.uint8)).to(gpu)   # writable copy (torch warns on read-only arrays)


def _messages(n, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 1400, n)
    lens[:4] = [1, 5, 27, 2000][:min(4, n)]
    msg = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    return lens, msg


@pytest.mark.parametrize("n_msgs,lo,hi", [(1, 512, 1200), (300, 512, 1200), (500, 400, 900), (64, 2048, 2048),
                                          (3000, 512, 1200)])
def test_encode_batch_vs_oracle(gpu, n_msgs, lo, hi):
    """Device frames byte for byte against oracle/gecko_ref.py (the wave-group kernel),
    sentinel bytes after the wire."""
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    lens, msg = _messages(n_msgs, n_msgs + lo)
    fr, off, total = gecko.plan_fragments(lens, lo, hi, first_msg_id=3)
    nf = len(fr)
    salts = sref.splitmix64_array(5, 0, nf)
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        out = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device=gpu)
        gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), pad_key=KEY, pad_nonce=NONCE,
                           out=out, out_off=_dev(off, gpu), n=nf)
        got = out.cpu().numpy()
    finally:
        o.close()
    exp = gref.encode_wire(PSK, msg.tobytes(), fr.tolist(), salts, KEY, NONCE, off)
    assert got[total:].tobytes() == b"\xa5" * 64
    for i in range(nf):
        assert got[int(off[i]):int(off[i]) + len(exp[i])].tobytes() == exp[i], i
        w = len(exp[i])
        assert w <= hi or int(fr[i]["pad_len"]) == 0
        assert w >= lo or 13 + int(fr[i]["chunk_len"]) > hi


@pytest.mark.parametrize("psk_len", [4, 9, 24, 57, 100, 113, 119, 120, 121, 127, 128, 200, 300])
def test_encode_batch_psk_lengths(gpu, psk_len):
    """The encode kernel hashes keys in registers, instantiated per salt word of the
    device block (salt_pos >> 3): PSK lengths cover every word, the two-block chain
    (salt_pos 121..127) and multi-block prefixes."""
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    psk = bytes((7 * i + psk_len) & 0xff for i in range(psk_len))
    lens, msg = _messages(40, psk_len)
    fr, off, total = gecko.plan_fragments(lens, 512, 1200, first_msg_id=psk_len)
    nf = len(fr)
    salts = sref.splitmix64_array(psk_len, 0, nf)
    o = hysteria_amd.SalamanderObfuscator(psk, 0)
    try:
        out = torch.zeros((total,), dtype=torch.uint8, device=gpu)
        ws = torch.empty(gecko.workspace_size(nf), dtype=torch.uint8, device=gpu)
        gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), pad_key=KEY, pad_nonce=NONCE,
                           out=out, out_off=_dev(off, gpu), workspace=ws, n=nf)
        got = out.cpu().numpy()
    finally:
        o.close()
    exp = gref.encode_wire(psk, msg.tobytes(), fr.tolist(), salts, KEY, NONCE, off)
    for i in range(nf):
        assert got[int(off[i]):int(off[i]) + len(exp[i])].tobytes() == exp[i], i


def test_encode_batch_skips_impossible_frames(gpu):
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    msg = np.arange(64, dtype=np.uint8)
    fr = np.array([(0, 10, 0, 1, 0x02), (0, 10, 0, 1, 0x01), (0, 10, 0, 1, 0x22), (0, 10, 2040, 1, 0x12),
                   (10, 10, 3, 2, 0x12)], dtype=gecko.FRAME_DTYPE)
    off = np.arange(len(fr), dtype=np.uint64) * 2100
    salts = sref.splitmix64_array(9, 0, len(fr))
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        out = torch.full((2100 * len(fr),), 0xA5, dtype=torch.uint8, device=gpu)
        ws = torch.empty(gecko.workspace_size(len(fr)), dtype=torch.uint8, device=gpu)
        gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), pad_key=KEY, pad_nonce=NONCE,
                           out=out, out_off=_dev(off, gpu), workspace=ws)
        got = out.cpu().numpy()
    finally:
        o.close()
    exp = gref.encode_wire(PSK, msg.tobytes(), fr.tolist()[:1], salts[:1], KEY, NONCE, off[:1])[0]
    assert got[:len(exp)].tobytes() == exp
    for i in (1, 2, 3):   # one chunk, index >= total, datagram over 2048 bytes: untouched
        assert (got[2100 * i:2100 * (i + 1)] == 0xA5).all(), i
    plain4 = gref.encode_frame(gref.Header(3, 2, 1, 2), msg[10:20].tobytes(), gref.pad_bytes(KEY, NONCE, 4 * 2100, 3))
    exp4 = sref.obfuscate(PSK, plain4, int(salts[4]).to_bytes(8, "little"))
    assert got[4 * 2100:4 * 2100 + len(exp4)].tobytes() == exp4


def test_parse_batch_and_reassembly(gpu):
    """Wire -> Salamander deobfuscate batch -> Gecko parse kernel -> host reassembly
    (acceptChunk, gecko.go:195-250) in shuffled order: every message comes back."""
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    lens, msg = _messages(200, 11)
    fr, off, total = gecko.plan_fragments(lens, 512, 1200, first_msg_id=0)
    nf = len(fr)
    salts = sref.splitmix64_array(6, 0, nf)
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        wire = torch.empty(total + 16, dtype=torch.uint8, device=gpu)
        ws = torch.empty(gecko.workspace_size(nf), dtype=torch.uint8, device=gpu)
        d_off = _dev(off, gpu)
        gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), pad_key=KEY, pad_nonce=NONCE,
                           out=wire, out_off=d_off, workspace=ws, n=nf)
        wl = (13 + fr["chunk_len"].astype(np.uint32) + fr["pad_len"]).astype(np.uint32)
        # append a short-header datagram, a dropped (8-byte) one and a malformed fragment
        extra = [sref.obfuscate(PSK, b"\x40hello", b"\x01" * 8), b"\x02" * 8,
                 sref.obfuscate(PSK, bytes([0x80, 1, 0x44, 0, 0]), b"\x03" * 8)]
        tail = np.frombuffer(b"".join(extra), np.uint8)
        wire_h = np.concatenate([wire.cpu().numpy()[:total], tail])
        all_off = np.concatenate([off, total + np.cumsum([0] + [len(e) for e in extra[:-1]])]).astype(np.uint64)
        all_len = np.concatenate([wl, [len(e) for e in extra]]).astype(np.uint32)
        n = nf + len(extra)
        d_wire = _dev(wire_h, gpu)
        plain = torch.empty(len(wire_h) + 16, dtype=torch.uint8, device=gpu)
        poff = torch.empty(n, dtype=torch.int64, device=gpu)
        plen = torch.empty(n, dtype=torch.int32, device=gpu)
        ws2 = torch.empty(hysteria_amd.workspace_size(n), dtype=torch.uint8, device=gpu)
        o.deobfuscate_batch(d_wire, n, in_off=_dev(all_off, gpu).view(torch.int64),
                            in_len=_dev(all_len, gpu).view(torch.int32), out=plain, out_cap=len(wire_h),
                            out_off=poff, out_len=plen, workspace=ws2, workspace_bytes=ws2.numel())
        parsed = torch.empty(n * 16, dtype=torch.uint8, device=gpu)
        gecko.parse_batch(plain, poff, plen, n, parsed)
        torch.cuda.synchronize()
        pr = parsed.cpu().numpy().view(gecko.PARSED_DTYPE)
        ph, ho, hl = plain.cpu().numpy(), poff.cpu().numpy().view(np.uint64), plen.cpu().numpy().view(np.uint32)
    finally:
        o.close()
    assert int(pr[nf]["status"]) == gecko.PASS and int(pr[nf]["payload_len"]) == 6
    assert int(pr[nf + 1]["status"]) == gecko.EMPTY          # 8-byte wire: Deobfuscate returns 0
    assert int(pr[nf + 2]["status"]) == gecko.ERR_INVALID
    for i in range(n):   # every datagram's classification matches the oracle's
        d = ph[int(ho[i]):int(ho[i]) + int(hl[i])].tobytes()
        kind = gref.parse(d)[0]
        assert {gref.PASS: 0, gref.FRAGMENT: 1, gref.EMPTY: -22, gref.TRUNCATED: -20,
                gref.INVALID: -21}[kind] == int(pr[i]["status"]), i
    g = gecko.GeckoPacketConn(None)
    order = list(range(nf))
    random.Random(5).shuffle(order)
    done = {}
    for i in order:
        r = pr[i]
        po = int(ho[i]) + int(r["payload_off"])
        payload = ph[po:po + int(r["payload_len"])].tobytes()
        it = int(r["idx_total"])
        h = gecko.FrameHeader(int(r["pad_len"]), int(r["msg_id"]), it >> 4, it & 0x0F)
        # one source per message: shuffled fragments of 200 messages from ONE source
        # would hit the per-source cap of 8 partial messages (gecko.go:209-212)
        out = g.accept_chunk(("127.0.0.1", 1000 + h.msg_id), h, payload)
        if out is not None:
            done[h.msg_id] = out
    g.close()
    base = np.concatenate([[0], np.cumsum(lens)])
    # msg ids wrap at 256: with 200 messages every id is unique
    assert len(done) == len(lens)
    for m in range(len(lens)):
        assert done[m & 0xFF] == msg[base[m]:base[m + 1]].tobytes(), m


def test_gecko_over_salamander_udp_loopback(gpu):
    """WrapPacketConnGecko over a real UDP socket: short and long headers round-trip
    (TestGeckoRoundTripShortHeader / LongHeader / SmallLongHeader)."""
    from hysteria_amd import gecko
    sa = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sb = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sa.bind(("127.0.0.1", 0))
    sb.bind(("127.0.0.1", 0))
    ga = gecko.wrap_packet_conn_gecko(sa, gecko.GeckoOptions(b"test"))
    gb = gecko.wrap_packet_conn_gecko(sb, gecko.GeckoOptions(b"test"))
    try:
        gb.inner.settimeout(5.0)
        for size, first in [(400, 0x40), (1200, 0xC0), (1, 0xC0), (27, 0xC0), (128, 0xC0), (2000, 0xC0)]:
            p = bytearray(random.Random(size).randbytes(size))
            p[0] = first
            assert ga.write_to(bytes(p), sb.getsockname()) == size
            got, src = gb.read_from(4096)
            assert got == bytes(p), size
            assert src[1] == sa.getsockname()[1]
    finally:
        ga.close()
        gb.close()


def test_encode_kernel_frame_grid(gpu):
    """TestEncodeDecodeFrame (gecko_frame_test.go:9-42) through the DEVICE encoder:
    totals 2..8, every chunk index, pad lengths 0/1/64/127/512/1100, payload
    a1 b2 c3 d4, msg id 0xa5.  Every wire datagram deobfuscates (oracle) and
    decodes (decodeFrame restated) to the same header and payload, and equals the
    oracle's wire byte for byte.  No workspace is passed (the shipped kernel needs none)."""
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    payload = bytes([0xA1, 0xB2, 0xC3, 0xD4])
    grid = [(t, i, pad) for t in range(2, 9) for i in range(t) for pad in (0, 1, 64, 127, 512, 1100)]
    fr = np.array([(0, len(payload), pad, 0xA5, (i << 4) | t) for t, i, pad in grid], dtype=gecko.FRAME_DTYPE)
    wl = 8 + 5 + fr["pad_len"].astype(np.uint64) + len(payload)
    off = np.concatenate([[0], np.cumsum(wl)[:-1]]).astype(np.uint64)
    total = int(wl.sum())
    salts = sref.splitmix64_array(21, 0, len(fr))
    msg = np.frombuffer(payload + b"\0" * 12, np.uint8)
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        out = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device=gpu)
        gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), pad_key=KEY, pad_nonce=NONCE,
                           out=out, out_off=_dev(off, gpu), n=len(fr))
        got = out.cpu().numpy()
    finally:
        o.close()
    assert got[total:].tobytes() == b"\xa5" * 64
    exp = gref.encode_wire(PSK, msg.tobytes(), fr.tolist(), salts, KEY, NONCE, off)
    for k, (t, i, pad) in enumerate(grid):
        wire = got[int(off[k]):int(off[k]) + int(wl[k])].tobytes()
        assert wire == exp[k], (t, i, pad)
        plain = sref.deobfuscate(PSK, wire)
        h, body = gref.decode_frame(plain)
        assert (h.pad_len, h.msg_id, h.chunk_idx, h.total_chunks) == (pad, 0xA5, i, t), (t, i, pad)
        assert body == payload


@pytest.mark.parametrize("order", ["ascending", "shuffled"])
def test_encode_dense_small_frames_with_gaps(gpu, order):
    """Frames of 14..72 wire bytes (one 16-byte chunk can hold parts of three frames),
    pad 0..23 and chunk 1..35 bytes taken from anywhere in the message buffer, with
    random gaps of 0..40 bytes between the wire datagrams.  In ascending wire order the
    groups take the aligned sweep (frame-record walk, edge chunks merged across frames,
    padding and message chunks next to gaps); shuffled, the per-frame window path.
    Every frame's wire equals the oracle's; gap bytes keep their sentinel."""
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    rng = np.random.default_rng(11 if order == "ascending" else 12)
    n = 3000
    pad, clen = rng.integers(0, 24, n), rng.integers(1, 36, n)
    coff = rng.integers(0, 4096 - 40, n)
    tot = rng.integers(2, 9, n)
    idx = rng.integers(0, 8, n) % tot
    msg = rng.integers(0, 256, 4096, dtype=np.uint8)
    fr = np.array([(int(coff[i]), int(clen[i]), int(pad[i]), i & 0xFF, (int(idx[i]) << 4) | int(tot[i]))
                   for i in range(n)], dtype=gecko.FRAME_DTYPE)
    wl = (13 + pad + clen).astype(np.uint64)
    gaps = rng.integers(0, 41, n).astype(np.uint64)
    off = np.cumsum(np.concatenate([[gaps[0]], wl[:-1] + gaps[1:]])).astype(np.uint64)
    total = int(off[-1] + wl[-1])
    if order == "shuffled":
        perm = rng.permutation(n)
        fr, off, wl = fr[perm], off[perm], wl[perm]
    salts = sref.splitmix64_array(33, 0, n)
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        out = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device=gpu)
        gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), pad_key=KEY,
                           pad_nonce=NONCE, out=out, out_off=_dev(off, gpu), n=n)
        got = out.cpu().numpy()
    finally:
        o.close()
    exp = gref.encode_wire(PSK, msg.tobytes(), fr.tolist(), salts, KEY, NONCE, off)
    covered = np.zeros(total + 64, bool)
    for k in range(n):
        a, b = int(off[k]), int(off[k] + wl[k])
        assert got[a:b].tobytes() == exp[k], (order, k)
        covered[a:b] = True
    assert (got[~covered] == 0xA5).all()


# TestDecodeFrameRejectsInvalid (gecko_frame_test.go:77-96) through the DEVICE parser.
# The parser classifies as ReadFrom does (gecko.go:176-193): an empty datagram is
# skipped before decodeFrame (EMPTY) and a clear top bit is passed through (PASS);
# every datagram with the top bit set gets decodeFrame's verdict.
DECODE_REJECTS = [
    ("empty", b"", "EMPTY"),
    ("header truncated", bytes([0x80, 0x55, 0x22, 0x00]), "ERR_TRUNCATED"),
    ("not a fragment", bytes([0x00, 0x00, 0x22, 0x00, 0x00]), "PASS"),
    ("totalChunks zero", bytes([0x80, 0x00, 0x00, 0x00, 0x00]), "ERR_INVALID"),
    ("totalChunks one", bytes([0x80, 0x00, 0x01, 0x00, 0x00]), "ERR_INVALID"),
    ("totalChunks nine", bytes([0x80, 0x00, 0x09, 0x00, 0x00]), "ERR_INVALID"),
    ("chunkIdx == totalChunks", bytes([0x80, 0x00, 0x44, 0x00, 0x00]), "ERR_INVALID"),
    ("padLen overrun", bytes([0x80, 0x00, 0x02, 0x00, 0x12, 0x01, 0x02]), "ERR_TRUNCATED"),
]


def test_parse_kernel_decode_frame_rejects(gpu):
    import torch
    from hysteria_amd import gecko
    data = b"".join(d for _, d, _ in DECODE_REJECTS)
    lens = np.array([len(d) for _, d, _ in DECODE_REJECTS], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    n = len(lens)
    parsed = torch.empty(n * 16, dtype=torch.uint8, device=gpu)
    gecko.parse_batch(_dev(np.frombuffer(data + b"\0" * 16, np.uint8), gpu), _dev(offs, gpu).view(torch.int64),
                      _dev(lens, gpu).view(torch.int32), n, parsed)
    torch.cuda.synchronize()
    pr = parsed.cpu().numpy().view(gecko.PARSED_DTYPE)
    oracle_status = {gref.PASS: gecko.PASS, gref.FRAGMENT: gecko.FRAGMENT, gref.EMPTY: gecko.EMPTY,
                     gref.TRUNCATED: gecko.ERR_TRUNCATED, gref.INVALID: gecko.ERR_INVALID}
    for k, (name, d, want) in enumerate(DECODE_REJECTS):
        assert int(pr[k]["status"]) == getattr(gecko, want), name
        assert int(pr[k]["status"]) == oracle_status[gref.parse(d)[0]], name


def test_encode_random_pad_key_padding_is_keystream(gpu):
    """Default encode_batch draws a fresh OS-random pad key per call (the reference
    pads from crypto/rand, gecko_frame.go:55): two calls give different padding and
    the same frames.  Salamander's key repeats every 32 bytes, so the wire exposes
    pad[j] ^ pad[j+32]; for a keystream pad those bytes are uniform (chi-square over
    256 bins), unlike a structured generator's."""
    import torch
    import hysteria_amd
    from hysteria_amd import gecko
    lens, msg = _messages(400, 77)
    fr, off, total = gecko.plan_fragments(lens, 1100, 1200, first_msg_id=1)
    nf = len(fr)
    salts = sref.splitmix64_array(8, 0, nf)
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        outs = []
        for _ in range(2):
            out = torch.zeros((total,), dtype=torch.uint8, device=gpu)
            gecko.encode_batch(o, msg=_dev(msg, gpu), frames=_dev(fr, gpu), salts=_dev(salts, gpu), out=out,
                               out_off=_dev(off, gpu), n=nf)
            outs.append(out.cpu().numpy())
    finally:
        o.close()
    diffs, same_frames = [], 0
    for i in range(nf):
        plen = int(fr[i]["pad_len"])
        w = [x[int(off[i]):int(off[i]) + 13 + plen + int(fr[i]["chunk_len"])].tobytes() for x in outs]
        p = [sref.deobfuscate(PSK, x) for x in w]
        h0, b0 = gref.decode_frame(p[0])
        h1, b1 = gref.decode_frame(p[1])
        assert (h0, b0) == (h1, b1)   # same frames ...
        same_frames += p[0][5:5 + plen] == p[1][5:5 + plen] and plen > 0
        if plen > 32:                 # ... what the wire exposes of the padding
            wire = np.frombuffer(w[0], np.uint8)
            diffs.append(wire[13:13 + plen - 32] ^ wire[13 + 32:13 + plen])
    assert same_frames == 0          # ... different padding
    d = np.concatenate(diffs)
    counts = np.bincount(d, minlength=256)
    exp = d.size / 256
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    assert d.size > 100_000 and chi2 < 400, (d.size, chi2)   # 255 dof: mean 255, sd ~22.6
