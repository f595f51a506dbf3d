"""QUIC packet protection oracle -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's QUIC Initial sniff decryption
(apernet/hysteria extras/sniff/internal/quic), used only by tests/ as the
checker of the device kernels (hysteria_amd/csrc/quic.hip).  Never imported by
the product.

Reference lines followed:
  packet_protector.go:21-31   NewProtectionKey / NewInitialProtectionKey
  packet_protector.go:46-79   PacketProtector.UnProtect (header protection, AEAD open)
  packet_protector.go:93-100  ProtectionKey.nonce
  packet_protector.go:102-156 newProtectionKey (AES-128-GCM, ChaCha20-Poly1305 suites)
  packet_protector.go:161-174 decodePacketNumber
  packet_protector.go:177-193 hkdfExpandLabel
  header.go:24-105            ParseInitialHeader / parseLongHeader
  quic.go:3-59                versions, initial salts, HKDF labels
  payload.go:21-60            ReadCryptoPayload
  payload.go:73-112           extractCryptoFrames
  payload.go:116-148          assembleCryptoFrames (sort.Slice there is not stable:
                              frames sharing an offset are kept in packet order here)
The ciphers come from Go's crypto/aes, crypto/cipher (GCM), golang.org/x/crypto
chacha20 / chacha20poly1305 / hkdf (extras/go.mod); they are restated here from
FIPS 197, NIST SP 800-38D, RFC 8439 and RFC 5869 (hashlib/hmac give SHA-256).
Pinned by the reference's own vectors (packet_protector_test.go:15-77) in
tests/test_quic.py, plus FIPS 197 C.1 and RFC 8439 2.5.2 / 2.4.2.
"""
from __future__ import annotations

import hashlib
import hmac
import struct

V1 = 0x1
V2 = 0x6B3343CF
TLS_AES_128_GCM_SHA256 = 0x1301
TLS_CHACHA20_POLY1305_SHA256 = 0x1303

SALT_OLD = bytes([0xaf, 0xbf, 0xec, 0x28, 0x99, 0x93, 0xd2, 0x4c, 0x9e, 0x97, 0x86, 0xf1, 0x9c, 0x61, 0x11, 0xe0,
                  0x43, 0x90, 0xa8, 0x99])
SALT_V1 = bytes([0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17, 0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad,
                 0xcc, 0xbb, 0x7f, 0x0a])
SALT_V2 = bytes([0x0d, 0xed, 0xe3, 0xde, 0xf7, 0x00, 0xa6, 0xdb, 0x81, 0x93, 0x81, 0xbe, 0x6e, 0x26, 0x9d, 0xcb,
                 0xf9, 0xbd, 0x2e, 0xd9])


class QuicError(Exception):
    pass


def get_salt(v: int) -> bytes:   # quic.go:28-36
    return SALT_V1 if v == V1 else SALT_V2 if v == V2 else SALT_OLD


def labels(v: int):               # quic.go:38-59: key, iv, hp
    return ("quicv2 key", "quicv2 iv", "quicv2 hp") if v == V2 else ("quic key", "quic iv", "quic hp")


# ------------------------------------------------------------------ HKDF (RFC 5869)
def hkdf_extract(salt: bytes, ikm: bytes) -> bytes:
    return hmac.new(salt, ikm, hashlib.sha256).digest()


def hkdf_expand(prk: bytes, info: bytes, n: int) -> bytes:
    out, t, i = b"", b"", 1
    while len(out) < n:
        t = hmac.new(prk, t + info + bytes([i]), hashlib.sha256).digest()
        out += t
        i += 1
    return out[:n]


def hkdf_expand_label(secret: bytes, label: str, context: bytes, n: int) -> bytes:   # packet_protector.go:177-193
    full = b"tls13 " + label.encode()
    info = struct.pack(">H", n) + bytes([len(full)]) + full + bytes([len(context)]) + context
    return hkdf_expand(secret, info, n)


def initial_secret(dcid: bytes, v: int, server: bool) -> bytes:   # payload.go:34-35 / packet_protector_test.go:39-40
    s = hkdf_extract(get_salt(v), dcid)
    return hkdf_expand_label(s, "server in" if server else "client in", b"", 32)


# ------------------------------------------------------------------ AES-128 (FIPS 197)
_SBOX = [0] * 256


def _init_sbox():
    p = q = 1
    while True:
        p = p ^ ((p << 1) & 0xFF) ^ (0x1B if p & 0x80 else 0)          # multiply by 3
        q ^= q << 1
        q ^= q << 2
        q ^= q << 4
        q &= 0xFF
        if q & 0x80:
            q ^= 0x09                                                  # divide by 3
        x = q ^ ((q << 1) | (q >> 7)) ^ ((q << 2) | (q >> 6)) ^ ((q << 3) | (q >> 5)) ^ ((q << 4) | (q >> 4))
        _SBOX[p] = (x ^ 0x63) & 0xFF
        if p == 1:
            break
    _SBOX[0] = 0x63


_init_sbox()


def _xtime(a):
    return ((a << 1) ^ 0x1B) & 0xFF if a & 0x80 else a << 1


def aes128_expand(key: bytes) -> list[list[int]]:
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    rcon = 1
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [_SBOX[b] for b in t[1:] + t[:1]]
            t[0] ^= rcon
            rcon = _xtime(rcon)
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return [sum(w[4 * r:4 * r + 4], []) for r in range(11)]


def aes128_encrypt_block(rk, block: bytes) -> bytes:
    s = [b ^ k for b, k in zip(block, rk[0])]
    for r in range(1, 11):
        s = [_SBOX[b] for b in s]
        s = [s[(i + 4 * (i % 4)) % 16] for i in range(16)]          # ShiftRows (column-major state)
        if r != 10:
            t = []
            for c in range(4):
                a = s[4 * c:4 * c + 4]
                x = a[0] ^ a[1] ^ a[2] ^ a[3]
                t += [a[i] ^ x ^ _xtime(a[i] ^ a[(i + 1) % 4]) for i in range(4)]
            s = t
        s = [b ^ k for b, k in zip(s, rk[r])]
    return bytes(s)


# ------------------------------------------------------------------ GCM (NIST SP 800-38D)
def _gf_mult(x: int, y: int) -> int:
    r = 0xE1 << 120
    z, v = 0, y
    for i in range(127, -1, -1):
        if (x >> i) & 1:
            z ^= v
        v = (v >> 1) ^ r if v & 1 else v >> 1
    return z


def _ghash(h: int, aad: bytes, ct: bytes) -> int:
    def blocks(b):
        b = b + b"\0" * (-len(b) % 16)
        return [int.from_bytes(b[i:i + 16], "big") for i in range(0, len(b), 16)]
    y = 0
    for x in blocks(aad) + blocks(ct) + [(len(aad) * 8) << 64 | (len(ct) * 8)]:
        y = _gf_mult(y ^ x, h)
    return y


def aes_gcm_open(key: bytes, nonce: bytes, ct_tag: bytes, aad: bytes) -> bytes:
    if len(ct_tag) < 16:
        raise QuicError("ciphertext shorter than the tag")
    rk = aes128_expand(key)
    ct, tag = ct_tag[:-16], ct_tag[-16:]
    h = int.from_bytes(aes128_encrypt_block(rk, b"\0" * 16), "big")
    j0 = nonce + b"\0\0\0\1"
    s = _ghash(h, aad, ct)
    want = (int.from_bytes(aes128_encrypt_block(rk, j0), "big") ^ s).to_bytes(16, "big")
    if not hmac.compare_digest(want, tag):
        raise QuicError("message authentication failed")
    out = bytearray()
    for i in range(0, len(ct), 16):
        ks = aes128_encrypt_block(rk, nonce + struct.pack(">I", 2 + i // 16))
        out += bytes(a ^ b for a, b in zip(ct[i:i + 16], ks))
    return bytes(out)


# ------------------------------------------------------------------ ChaCha20-Poly1305 (RFC 8439)
def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    c = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    s = c + list(struct.unpack("<8I", key)) + [counter & 0xFFFFFFFF] + list(struct.unpack("<3I", nonce))
    x = list(s)

    def qr(a, b, cc, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 16)
        x[cc] = (x[cc] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[cc], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = _rotl(x[d] ^ x[a], 8)
        x[cc] = (x[cc] + x[d]) & 0xFFFFFFFF; x[b] = _rotl(x[b] ^ x[cc], 7)
    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(a + b) & 0xFFFFFFFF for a, b in zip(x, s)])


def chacha20_xor(key: bytes, counter: int, nonce: bytes, data: bytes) -> bytes:
    out = bytearray()
    for i in range(0, len(data), 64):
        ks = chacha20_block(key, counter + i // 64, nonce)
        out += bytes(a ^ b for a, b in zip(data[i:i + 64], ks))
    return bytes(out)


def poly1305(key: bytes, msg: bytes) -> bytes:
    r = int.from_bytes(key[:16], "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    s = int.from_bytes(key[16:], "little")
    p = (1 << 130) - 5
    acc = 0
    for i in range(0, len(msg), 16):
        n = int.from_bytes(msg[i:i + 16] + b"\1", "little")
        acc = (acc + n) * r % p
    return ((acc + s) & ((1 << 128) - 1)).to_bytes(16, "little")


def chacha20_poly1305_open(key: bytes, nonce: bytes, ct_tag: bytes, aad: bytes) -> bytes:
    if len(ct_tag) < 16:
        raise QuicError("ciphertext shorter than the tag")
    ct, tag = ct_tag[:-16], ct_tag[-16:]
    otk = chacha20_block(key, 0, nonce)[:32]
    mac = (aad + b"\0" * (-len(aad) % 16) + ct + b"\0" * (-len(ct) % 16)
           + struct.pack("<QQ", len(aad), len(ct)))
    if not hmac.compare_digest(poly1305(otk, mac), tag):
        raise QuicError("message authentication failed")
    return chacha20_xor(key, 1, nonce, ct)


# ------------------------------------------------------------------ protection key / UnProtect
class ProtectionKey:
    """newProtectionKey (packet_protector.go:107-160)."""

    def __init__(self, suite: int, secret: bytes, v: int):
        kl, ivl, hpl = labels(v)
        if suite == TLS_AES_128_GCM_SHA256:
            self.key = hkdf_expand_label(secret, kl, b"", 16)
            self.iv = hkdf_expand_label(secret, ivl, b"", 12)
            self.hp = hkdf_expand_label(secret, hpl, b"", 16)
        elif suite == TLS_CHACHA20_POLY1305_SHA256:
            self.key = hkdf_expand_label(secret, kl, b"", 32)
            self.iv = hkdf_expand_label(secret, ivl, b"", 12)
            self.hp = hkdf_expand_label(secret, hpl, b"", 32)
        else:
            raise QuicError("not supported cipher suite")
        self.suite = suite

    def header_mask(self, sample: bytes) -> bytes:
        if self.suite == TLS_AES_128_GCM_SHA256:
            return aes128_encrypt_block(aes128_expand(self.hp), sample)
        return chacha20_xor(self.hp, int.from_bytes(sample[:4], "little"), sample[4:16], b"\0" * 5)

    def nonce(self, pn: int) -> bytes:   # packet_protector.go:96-104
        return bytes(a ^ b for a, b in zip(self.iv, b"\0" * 4 + struct.pack(">Q", pn & 0xFFFFFFFFFFFFFFFF)))

    def open(self, nonce: bytes, ct_tag: bytes, aad: bytes) -> bytes:
        if self.suite == TLS_AES_128_GCM_SHA256:
            return aes_gcm_open(self.key, nonce, ct_tag, aad)
        return chacha20_poly1305_open(self.key, nonce, ct_tag, aad)


def initial_protection_key(secret: bytes, v: int) -> ProtectionKey:   # packet_protector.go:29-31
    return ProtectionKey(TLS_AES_128_GCM_SHA256, secret, v)


def decode_packet_number(largest: int, truncated: int, nbytes: int) -> int:   # packet_protector.go:165-178
    expected = largest + 1
    win = 1 << (nbytes * 8)
    hwin = win // 2
    mask = win - 1
    candidate = (expected & ~mask) | truncated
    if candidate <= expected - hwin and candidate < (1 << 62) - win:
        return candidate + win
    if candidate > expected + hwin and candidate >= win:
        return candidate - win
    return candidate


def unprotect(key: ProtectionKey, packet: bytearray, pn_offset: int, pn_max: int):
    """UnProtect (packet_protector.go:46-84): unmasks the header in place and
    returns (header, plaintext, pn).  Raises QuicError like the reference errors."""
    if pn_offset < 0:
        raise QuicError("negative packet-number offset")   # the reference's slicing panics
    long_hdr = bool(packet[0] & 0x80)
    if long_hdr and len(packet) < pn_offset + 4 + 16:
        raise QuicError("packet with long header is too small")
    sample = bytes(packet[pn_offset + 4:pn_offset + 20])
    if len(sample) < 16:
        # a short-header packet with no room for the sample: the reference's
        # slice expression panics (or reads past the slice into its capacity)
        raise QuicError("packet too small for the header protection sample")
    mask = key.header_mask(sample)
    packet[0] ^= mask[0] & (0x0F if long_hdr else 0x1F)
    pn_len = (packet[0] & 0x3) + 1
    pn = 0
    for i in range(pn_len):
        packet[pn_offset + i] ^= mask[1 + i]
        pn = (pn << 8) | packet[pn_offset + i]
    pn = decode_packet_number(pn_max, pn, pn_len)
    hdr = bytes(packet[:pn_offset + pn_len])
    payload = bytes(packet[pn_offset + pn_len:])
    return hdr, key.open(key.nonce(pn), payload, hdr), pn


# ------------------------------------------------------------------ sealing (test-packet construction)
def aes_gcm_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes) -> bytes:
    rk = aes128_expand(key)
    ct = bytearray()
    for i in range(0, len(pt), 16):
        ks = aes128_encrypt_block(rk, nonce + struct.pack(">I", 2 + i // 16))
        ct += bytes(a ^ b for a, b in zip(pt[i:i + 16], ks))
    h = int.from_bytes(aes128_encrypt_block(rk, b"\0" * 16), "big")
    s = _ghash(h, aad, bytes(ct))
    tag = (int.from_bytes(aes128_encrypt_block(rk, nonce + b"\0\0\0\1"), "big") ^ s).to_bytes(16, "big")
    return bytes(ct) + tag


def chacha20_poly1305_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes) -> bytes:
    ct = chacha20_xor(key, 1, nonce, pt)
    otk = chacha20_block(key, 0, nonce)[:32]
    mac = (aad + b"\0" * (-len(aad) % 16) + ct + b"\0" * (-len(ct) % 16)
           + struct.pack("<QQ", len(aad), len(ct)))
    return ct + poly1305(otk, mac)


def protect(key: ProtectionKey, header: bytes, pn_offset: int, pn: int, payload: bytes) -> bytes:
    """The sender side of UnProtect (RFC 9001 5.3-5.4): header = the plain header
    ending with the truncated packet number (its length in the low 2 bits of
    byte 0); returns the protected packet."""
    pn_len = (header[0] & 3) + 1
    assert len(header) == pn_offset + pn_len
    nonce = key.nonce(pn)
    if key.suite == TLS_AES_128_GCM_SHA256:
        body = aes_gcm_seal(key.key, nonce, payload, header)
    else:
        body = chacha20_poly1305_seal(key.key, nonce, payload, header)
    pkt = bytearray(header + body)
    sample = bytes(pkt[pn_offset + 4:pn_offset + 20])
    mask = key.header_mask(sample)
    pkt[0] ^= mask[0] & (0x0F if pkt[0] & 0x80 else 0x1F)
    for i in range(pn_len):
        pkt[pn_offset + i] ^= mask[1 + i]
    return bytes(pkt)


def encode_varint(v: int, n: int | None = None) -> bytes:
    """quicvarint encoding, minimal unless n (1/2/4/8 bytes) is given."""
    if n is None:
        n = 1 if v < 64 else 2 if v < 1 << 14 else 4 if v < 1 << 30 else 8
    bits = {1: 0, 2: 1, 4: 2, 8: 3}[n]
    b = bytearray(v.to_bytes(n, "big"))
    b[0] |= bits << 6
    return bytes(b)


def client_initial(dcid: bytes, scid: bytes, version: int, token: bytes, pn: int, pn_len: int,
                   frames: bytes, length_override: int | None = None, tail: bytes = b"") -> bytes:
    """A protected client Initial packet (long header, RFC 9000 17.2.2) whose
    payload is `frames`; Length covers the packet number, payload and tag."""
    ptype = 0b01 if version == V2 else 0b00
    first = 0xC0 | ptype << 4 | (pn_len - 1)
    length = pn_len + len(frames) + 16
    hdr = (bytes([first]) + struct.pack(">I", version) + bytes([len(dcid)]) + dcid + bytes([len(scid)]) + scid
           + encode_varint(len(token)) + token + encode_varint(length if length_override is None else length_override,
                                                                 2))
    pn_offset = len(hdr)
    hdr += (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big")
    key = initial_protection_key(initial_secret(dcid, version, server=False), version)
    return protect(key, hdr, pn_offset, pn, frames) + tail


# ------------------------------------------------------------------ header + crypto frames
def read_varint(b: bytes, i: int, err: str = "EOF"):
    if i >= len(b):
        raise QuicError(err)
    n = 1 << (b[i] >> 6)
    if i + n > len(b):
        raise QuicError(err)
    v = b[i] & 0x3F
    for k in range(1, n):
        v = (v << 8) | b[i + k]
    return v, i + n


def parse_initial_header(data: bytes):
    """ParseInitialHeader (header.go:23-94): (fields, pn_offset)."""
    if len(data) < 5:
        raise QuicError("EOF")
    type_byte = data[0]
    version = struct.unpack(">I", data[1:5])[0]
    if version != 0 and type_byte & 0x40 == 0:
        raise QuicError("not a QUIC packet")
    i = 5
    if i >= len(data):
        raise QuicError("EOF")
    dl = data[i]
    i += 1
    dcid = data[i:i + dl]
    if len(dcid) < dl:
        raise QuicError("EOF")
    i += dl
    if i >= len(data):
        raise QuicError("EOF")
    sl = data[i]
    i += 1
    scid = data[i:i + sl]
    if len(scid) < sl:
        raise QuicError("EOF")
    i += sl
    token = b""
    if (type_byte >> 4 & 0b11) == (0b01 if version == V2 else 0b00):
        tl, i = read_varint(data, i)
        if tl > len(data) - i:
            raise QuicError("EOF")
        token = data[i:i + tl]
        i += tl
    length, i = read_varint(data, i)
    return dict(type=type_byte, version=version, dcid=dcid, scid=scid, token=token, length=length), i


def read_crypto_payload(packet: bytes) -> bytes:
    """ReadCryptoPayload (payload.go:21-63) of a client Initial packet."""
    hdr, offset = parse_initial_header(packet)
    if hdr["version"] not in (V1, V2):
        raise QuicError("unsupported version")
    if offset == 0 or hdr["length"] == 0:
        raise QuicError("invalid packet")
    key = initial_protection_key(initial_secret(hdr["dcid"], hdr["version"], server=False), hdr["version"])
    if len(packet) < offset + hdr["length"]:
        raise QuicError("packet is too short")
    buf = bytearray(packet[:offset + hdr["length"]])
    _, plain, _ = unprotect(key, buf, offset, 2)
    frames = extract_crypto_frames(plain)
    data = assemble_crypto_frames(frames)
    if data is None:
        raise QuicError("unable to assemble crypto frames")
    return data


def extract_crypto_frames(p: bytes):   # payload.go:76-116
    frames, i = [], 0
    while i < len(p):
        typ, i = read_varint(p, i, "unexpected EOF")
        if typ in (0x00, 0x01):
            continue
        if typ != 0x06:
            raise QuicError(f"encountered unexpected frame type: {typ}")
        off, i = read_varint(p, i, "unexpected EOF")
        if off > (1 << 63) - 1:
            raise QuicError("invalid crypto frame offset")
        n, i = read_varint(p, i, "unexpected EOF")
        if n > 256 * 1024:
            raise QuicError("crypto frame data too large")
        if n > len(p) - i:
            raise QuicError("unexpected EOF")
        frames.append((off, p[i:i + n]))
        i += n
    return frames


def assemble_crypto_frames(frames):   # payload.go:118-148
    if not frames:
        return None
    if len(frames) == 1:
        return frames[0][1]
    frames = sorted(frames, key=lambda f: f[0])
    for a, b in zip(frames, frames[1:]):
        if b[0] != a[0] + len(a[1]):
            return None
    last = frames[-1]
    if last[0] > 256 * 1024:
        return None
    end = last[0] + len(last[1])
    if end > 256 * 1024:
        return None
    out = bytearray(end)
    for off, d in frames:
        out[off:off + len(d)] = d
    return bytes(out)


# ------------------------------------------------------------------ C restatement (oracle/quic_ref.c)
class CQuicOracle:
    """ctypes view of oracle/libquic_ref.so: ReadCryptoPayload over a batch on
    host threads (the CPU baseline of scripts/bench_quic.py)."""

    def __init__(self, path: str | None = None):
        import ctypes
        import os
        path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libquic_ref.so")
        self.lib = ctypes.CDLL(path)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        self.lib.quic_read_crypto_payload_batch.argtypes = [vp, vp, vp, u64, vp, u32, vp, vp, i32]
        self.lib.quic_read_crypto_payload_batch.restype = i32

    def read_batch(self, buf, off, lens, n: int, cap: int, threads: int = 1):
        """(status int32[n], out_len uint32[n], out uint8[n*cap])."""
        import numpy as np
        out = np.zeros(n * cap, np.uint8)
        st = np.zeros(n, np.int32)
        ol = np.zeros(n, np.uint32)
        self.lib.quic_read_crypto_payload_batch(buf.ctypes.data, off.ctypes.data, lens.ctypes.data, n,
                                                out.ctypes.data, cap, st.ctypes.data, ol.ctypes.data, threads)
        return st, ol, out
