"""QUIC Initial unprotection cases shared by the CPU-emulated tier
(tests/emu/run_case.py quic) and the GPU tier (tests/test_gpu_quic.py).

Expected results come from oracle/quic_ref.py, which tests/test_quic.py pins to
the reference's own vectors (packet_protector_test.go:15-77).
"""
import re

import numpy as np

from oracle import quic_ref as ref

# packet_protector_test.go:17-31 (draft-ietf-quic-tls-32 A.3, server Initial)
_h = lambda s: bytes.fromhex(re.sub(r"\s", "", s))  # noqa: E731
AES_PROTECTED = _h("""c7ff0000200008f067a5502a4262b500 4075fb12ff07823a5d24534d906ce4c7
    6782a2167e3479c0f7f6395dc2c91676 302fe6d70bb7cbeb117b4ddb7d173498
    44fd61dae200b8338e1b932976b61d91 e64a02e9e0ee72e3a6f63aba4ceeeec5
    be2f24f2d86027572943533846caa13e 6f163fb257473d0eda5047360fd4a47e
    fd8142fafc0f76""")
AES_PLAIN = _h("""02000000000600405a020000560303ee fce7f7b37ba1d1632e96677825ddf739
    88cfc79825df566dc5430b9a045a1200 130100002e00330024001d00209d3c94
    0d89690b84d08a60993c144eca684d10 81287c834d5311bcf32bb9da1a002b00
    020304""")
AES_CONN_ID = _h("8394c8f03e515708")
# packet_protector_test.go:57-61 (draft-ietf-quic-tls-32 A.5, ChaCha20 short header)
CHACHA_PROTECTED = _h("4cfe4189655e5cd55c41f69080575d7999c25a5bfb")
CHACHA_PLAIN = _h("01")
CHACHA_HDR = _h("4200bff4")
CHACHA_SECRET = _h("9ac312a7f877468ebe69422748ad00a15443f18203a07d6060f688f30f21632b")
CHACHA_PN_MAX = 654360564

STATUS = {
    "EOF": -40, "not a QUIC packet": -41, "unsupported version": -42, "invalid packet": -43,
    "packet is too short": -44, "packet with long header is too small": -45,
    "packet too small for the header protection sample": -45, "negative packet-number offset": -45, "message authentication failed": -46,
    "ciphertext shorter than the tag": -46, "encountered unexpected frame type": -47, "unexpected EOF": -48,
    "crypto frame data too large": -49, "unable to assemble crypto frames": -50,
}


def status_of(exc: Exception) -> int:
    msg = str(exc)
    if msg.startswith("encountered unexpected frame type"):
        msg = "encountered unexpected frame type"
    return STATUS[msg]


def oracle_read(packet: bytes):
    """(status, crypto data) by the oracle's ReadCryptoPayload."""
    try:
        return 0, ref.read_crypto_payload(packet)
    except ref.QuicError as e:
        return status_of(e), b""


def oracle_unprotect(key, packet: bytes, pn_offset: int, pn_max: int):
    """(status, unmasked header, plaintext, pn)."""
    buf = bytearray(packet)
    try:
        hdr, plain, pn = ref.unprotect(key, buf, pn_offset, pn_max)
        return 0, hdr, plain, pn
    except ref.QuicError as e:
        return status_of(e), b"", b"", 0


def _crypto(off, data, n_off=None, n_len=None):
    return b"\x06" + ref.encode_varint(off, n_off) + ref.encode_varint(len(data), n_len) + data


def client_hello_like(rng, n):
    return b"\x01\x00" + n.to_bytes(2, "big") + rng.integers(0, 256, n, dtype=np.uint8).tobytes()


def frame_layouts(rng):
    """(name, frames payload) covering extractCryptoFrames / assembleCryptoFrames."""
    ch = client_hello_like(rng, 300)
    out = [
        ("single", _crypto(0, ch) + b"\x00" * 800),
        ("single_at_offset", _crypto(77, ch[:100]) + b"\x00" * 50),    # one frame: returned as is, offset ignored
        ("padding_first", b"\x00" * 200 + b"\x01" + _crypto(0, ch) + b"\x00" * 500),
        ("split_sorted", _crypto(0, ch[:100]) + _crypto(100, ch[100:]) + b"\x00" * 400),
        ("split_shuffled", _crypto(200, ch[200:]) + b"\x01\x00\x00" + _crypto(0, ch[:120]) + b"\x01" +
         _crypto(120, ch[120:200]) + b"\x00" * 333),
        ("nonminimal_varints", _crypto(0, ch[:50], 8, 4) + b"\x40\x00" + b"\x80\x00\x00\x01" +
         _crypto(50, ch[50:], 2, 2) + b"\x00" * 64),
        ("zero_prefix", _crypto(1000, ch[:40]) + _crypto(1040, ch[40:90])),   # assembled with 1000 zero bytes
        ("zero_len_frames", _crypto(0, b"") + _crypto(0, ch[:10]) + _crypto(10, b"") + _crypto(10, ch[10:30])),
        ("many_frames", b"".join(_crypto(5 * k, ch[5 * k:5 * k + 5]) for k in range(40)) + b"\x00" * 64),
        ("padding_tail_63", _crypto(0, ch[:70]) + b"\x00" * 63),
        ("padding_tail_64", _crypto(0, ch[:70]) + b"\x01" * 64),
        ("padding_tail_65", _crypto(0, ch[:70]) + b"\x00" * 65),
        # errors
        ("gap", _crypto(0, ch[:50]) + _crypto(60, ch[60:100]) + b"\x00" * 100),
        ("overlap", _crypto(0, ch[:50]) + _crypto(40, ch[40:100]) + b"\x00" * 100),
        ("no_crypto", b"\x01" + b"\x00" * 300),
        ("ack_frame", _crypto(0, ch[:50]) + b"\x02\x00\x00\x00\x00" + b"\x00" * 100),
        ("frame_eof_len", _crypto(0, ch[:50]) + b"\x06\x00"),
        ("frame_eof_data", _crypto(0, ch[:50]) + b"\x06\x00\x44\x00" + ch[:20]),
        ("frame_too_large", b"\x06\x00\x80\x04\x00\x01" + b"\x00" * 40),
        ("end_past_max_payload", _crypto(256 * 1024 - 10, ch[:5]) + _crypto(256 * 1024 - 5, ch[5:20])),
        ("offset_past_max_payload", _crypto(256 * 1024 + 1, ch[:3]) + _crypto(256 * 1024 + 4, ch[3:6])),
        ("single_far_offset", _crypto(1 << 40, ch[:33], 8)),   # one frame: no offset check at all
        ("too_many_frames", b"".join(_crypto(k, ch[k:k + 1]) for k in range(300))),
        ("type_varint_eof", _crypto(0, ch[:30]) + b"\x40"),
    ]
    return out


def crypto_packets(seed: int = 1):
    """A list of (name, packet bytes) of client Initials, good and bad."""
    rng = np.random.default_rng(seed)
    pkts = []
    layouts = frame_layouts(rng)
    for k, (name, frames) in enumerate(layouts):
        version = ref.V2 if k % 3 == 2 else ref.V1
        dl = [8, 0, 20, 1, 255, 18][k % 6]
        dcid = rng.integers(0, 256, dl, dtype=np.uint8).tobytes()
        scid = rng.integers(0, 256, k % 9, dtype=np.uint8).tobytes()
        token = rng.integers(0, 256, [0, 0, 33][k % 3], dtype=np.uint8).tobytes()
        pn_len = 1 + k % 4
        pkts.append((name, ref.client_initial(dcid, scid, version, token, 2, pn_len, frames)))
    ch = client_hello_like(rng, 200)
    good = _crypto(0, ch) + b"\x00" * 900
    dcid = bytes(range(8))
    base = ref.client_initial(dcid, b"", ref.V1, b"", 2, 4, good)
    tampered = bytearray(base)
    tampered[-1] ^= 1
    ct_flip = bytearray(base)
    ct_flip[60] ^= 0x80
    pkts += [
        ("v1_plain", base),
        ("coalesced_tail", ref.client_initial(dcid, b"", ref.V1, b"", 2, 4, good, tail=b"\xaa" * 50)),
        ("tag_tampered", bytes(tampered)),
        ("ct_tampered", bytes(ct_flip)),
        ("draft29_version", ref.client_initial(dcid, b"", 0xFF00001D, b"", 2, 4, good)),
        ("version_zero", bytes([0x80]) + b"\0\0\0\0" + b"\x08" + dcid + b"\x00\x00\x05" + b"\0" * 30),
        ("not_quic", bytes([0x80]) + b"\0\0\0\1" + b"\x08" + dcid + b"\x00" * 40),
        ("length_past_end", ref.client_initial(dcid, b"", ref.V1, b"", 2, 4, good, length_override=5000)),
        ("length_zero", base[:base.index(dcid) + 9 + 1] + b"\x40\x00" + base[base.index(dcid) + 12:]),
        ("length_tiny", ref.client_initial(dcid, b"", ref.V1, b"", 2, 1, good, length_override=12)),
        ("truncated_4", base[:4]),
        ("truncated_dcid", base[:9]),
        ("truncated_scid_len", base[:14]),
        ("truncated_token_len", base[:15]),
        ("truncated_length", base[:17]),
        ("empty", b""),
        ("short_header_bit", bytes([base[0] & 0x7F]) + base[1:]),
        ("v2_long_dcid", ref.client_initial(bytes(range(20)) * 2, b"abc", ref.V2, b"tok" * 20, 2, 2, good)),
    ]
    return pkts


def unprotect_cases(seed: int = 2):
    """(name, key, packet, pn_offset, pn_max) for UnProtect with explicit keys,
    both suites, long and short headers, several packet-number windows."""
    rng = np.random.default_rng(seed)
    cases = []
    aes_key = ref.initial_protection_key(ref.initial_secret(AES_CONN_ID, 0xFF000020, True), 0xFF000020)
    cases.append(("ref_aes_server_initial", aes_key, AES_PROTECTED, 18, 1))
    cc_key = ref.ProtectionKey(ref.TLS_CHACHA20_POLY1305_SHA256, CHACHA_SECRET, ref.V1)
    cases.append(("ref_chacha_short_header", cc_key, CHACHA_PROTECTED, 1, CHACHA_PN_MAX))
    for k in range(24):
        suite = ref.TLS_AES_128_GCM_SHA256 if k % 2 == 0 else ref.TLS_CHACHA20_POLY1305_SHA256
        version = [ref.V1, ref.V2, 0xFF00001D][k % 3]
        key = ref.ProtectionKey(suite, rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), version)
        pn_len = 1 + (k // 2) % 4
        long_hdr = k % 4 < 2
        plen = [0, 1, 15, 16, 17, 63, 64, 65, 700, 1150, 2047, 4100][k % 12]
        payload = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        pn_max = int(rng.integers(0, 1 << 40))
        pn = pn_max + 1 + int(rng.integers(-(1 << (8 * pn_len - 2)), 1 << (8 * pn_len - 2)))
        pn = max(pn, 0)
        if long_hdr:
            first = 0xC0 | (pn_len - 1)
            pre = bytes([first]) + struct_be(version) + b"\x04abcd\x00" + b"\x00" + ref.encode_varint(
                pn_len + plen + 16, 2)
        else:
            first = 0x40 | (pn_len - 1)
            pre = bytes([first]) + rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        hdr = pre + (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big")
        if len(hdr) + plen + 16 < len(pre) + 20:   # pad the payload so the sample fits
            payload += bytes(len(pre) + 20 - len(hdr) - plen - 16)
        pkt = ref.protect(key, hdr, len(pre), pn, payload)
        cases.append((f"rand{k}", key, pkt, len(pre), pn_max))
    # errors: too small for the sample, tampered tag, negative offset
    key = cases[2][1]
    pkt = cases[2][2]
    bad = bytearray(pkt)
    bad[-3] ^= 0x10
    cases += [("tag_flip", key, bytes(bad), cases[2][3], cases[2][4]),
              ("too_small", key, pkt[:cases[2][3] + 19], cases[2][3], 0),
              ("neg_offset", key, pkt, -1, 0),
              ("offset_past_end", key, pkt, len(pkt) + 3, 0)]
    return cases


def struct_be(v: int) -> bytes:
    return v.to_bytes(4, "big")


def key_record(key) -> bytes:
    """oracle ProtectionKey -> struct hyobfs_quic_key bytes (80)."""
    k = key.key + bytes(32 - len(key.key))
    hp = key.hp + bytes(32 - len(key.hp))
    return key.suite.to_bytes(4, "little") + key.iv + k + hp


def pack(packets):
    lens = np.array([len(p) for p in packets], np.uint32)
    off = np.zeros(len(packets), np.uint64)
    if len(packets) > 1:
        np.cumsum(lens[:-1], out=off[1:])
    buf = np.frombuffer(b"".join(packets) + bytes(64), np.uint8).copy()
    return buf, off, lens


def check_unprotect(cases, buf, off, res):
    """Compare device results (in-place buffer + RESULT_DTYPE records) with the oracle."""
    for i, (name, key, pkt, pn_offset, pn_max) in enumerate(cases):
        st, hdr, plain, pn = oracle_unprotect(key, pkt, pn_offset, pn_max)
        r = res[i]
        assert int(r["status"]) == st, (name, int(r["status"]), st)
        if st:
            continue
        o = int(off[i])
        got_hdr = buf[o:o + int(r["hdr_len"])].tobytes()
        got = buf[o + int(r["hdr_len"]):o + int(r["hdr_len"]) + int(r["plain_len"])].tobytes()
        assert (got_hdr, got, int(r["pn"])) == (hdr, plain, pn), name


def check_crypto(pkts, out, out_off, caps, res):
    """Device ReadCryptoPayload results vs the oracle.  Two device limits with no
    reference counterpart: more than 256 CRYPTO frames (-52) and assembled data
    larger than the caller's out_cap (-51, out_len = the size needed)."""
    for i, (name, pkt) in enumerate(pkts):
        st, data = oracle_read(pkt)
        r = res[i]
        if st == 0 and name == "too_many_frames":
            st = -52
        if st == 0 and len(data) > int(caps[i]):
            assert int(r["status"]) == -51 and int(r["out_len"]) == len(data), name
            continue
        assert int(r["status"]) == st, (name, int(r["status"]), st)
        if st == 0:
            o = int(out_off[i])
            assert int(r["out_len"]) == len(data), (name, int(r["out_len"]), len(data))
            assert out[o:o + len(data)].tobytes() == data, name
