"""QUIC Initial unprotection for the sniffer -- ``extras/sniff/internal/quic`` on MI355X.

==================================================  ==================================================
reference (Go)                                      here
==================================================  ==================================================
``V1`` / ``V2``, salts, labels (quic.go:3-59)       ``V1`` / ``V2`` (the rest lives in the C ABI)
``Header`` / ``ParseInitialHeader`` (header.go)     ``Header`` / ``parse_initial_header(data)``
``hkdfExpandLabel`` (packet_protector.go:177-193)   ``hkdf_expand_label(secret, label, ctx, n)``
Initial secret (payload.go:34-35)                   ``initial_secret(dcid, version, server)``
``NewProtectionKey`` (packet_protector.go:21-23)    ``new_protection_key(suite, secret, version)``
``NewInitialProtectionKey`` (:29-31)                ``new_initial_protection_key(secret, version)``
``(*PacketProtector).UnProtect`` (:46-79)           ``PacketProtector(key).unprotect(packet, off, max)``
                                                    and ``unprotect_batch`` (GPU, many packets)
``ReadCryptoPayload`` (payload.go:21-60)            ``read_crypto_payload(packet)`` and
                                                    ``read_crypto_payload_batch`` (GPU)
==================================================  ==================================================

Key derivation, header parsing and both batch kernels are in ``libhyobfs.so``
(``include/hyobfs_quic.h``); there is no CPU path.  The one-packet helpers
move the packet to ``cuda:<device>`` and run a batch of one.  Errors raise
``QuicError`` carrying the reference's message and the ABI status.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

V1 = 0x1
V2 = 0x6B3343CF
TLS_AES_128_GCM_SHA256 = 0x1301
TLS_CHACHA20_POLY1305_SHA256 = 0x1303
MAX_CRYPTO_PAYLOAD_LEN = 256 * 1024
MAX_FRAMES = 256

ERRORS = {
    -40: "EOF",
    -41: "not a QUIC packet",
    -42: "unsupported version",
    -43: "invalid packet",
    -44: "packet is too short",
    -45: "packet with long header is too small",
    -46: "decryption failed",
    -47: "encountered unexpected frame type",
    -48: "unexpected EOF",
    -49: "crypto frame data too large",
    -50: "unable to assemble crypto frames",
    -51: "output buffer too small",
    -52: "too many crypto frames",
    -53: "not supported cipher suite",
}
ERR_EOF, ERR_NOT_QUIC, ERR_VERSION, ERR_INVALID, ERR_SHORT, ERR_TOO_SMALL, ERR_AUTH = range(-40, -47, -1)
ERR_FRAME_TYPE, ERR_FRAME_EOF, ERR_FRAME_TOO_LARGE, ERR_ASSEMBLE, ERR_OUT_CAP, ERR_FRAMES, ERR_SUITE = \
    range(-47, -54, -1)


class QuicError(ValueError):
    def __init__(self, status: int):
        self.status = status
        super().__init__(f"{ERRORS.get(status, 'error')} ({status})")


class HyobfsQuicKey(ctypes.Structure):
    _fields_ = [("suite", ctypes.c_uint32), ("iv", ctypes.c_uint8 * 12), ("key", ctypes.c_uint8 * 32),
                ("hp", ctypes.c_uint8 * 32)]


class HyobfsQuicHeader(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint8), ("dcid_len", ctypes.c_uint8), ("scid_len", ctypes.c_uint8),
                ("pad_", ctypes.c_uint8), ("version", ctypes.c_uint32), ("dcid_off", ctypes.c_uint32),
                ("scid_off", ctypes.c_uint32), ("token_off", ctypes.c_uint32), ("token_len", ctypes.c_uint32),
                ("length", ctypes.c_uint64), ("offset", ctypes.c_int64)]


# struct hyobfs_quic_key / hyobfs_quic_result as numpy records
KEY_DTYPE = np.dtype([("suite", "<u4"), ("iv", "u1", (12,)), ("key", "u1", (32,)), ("hp", "u1", (32,))])
RESULT_DTYPE = np.dtype([("status", "<i4"), ("hdr_len", "<u4"), ("plain_len", "<u4"), ("out_len", "<u4"),
                         ("pn", "<i8")])
assert KEY_DTYPE.itemsize == ctypes.sizeof(HyobfsQuicKey) == 80 and RESULT_DTYPE.itemsize == 24


def _qlib():
    lib = _lib.load()
    if not getattr(lib, "_quic_declared", False):
        vp, sz, u64, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        for name, res, args in (
                ("hyobfs_quic_parse_initial_header", i32, [vp, sz, ctypes.POINTER(HyobfsQuicHeader)]),
                ("hyobfs_quic_initial_secret", i32, [vp, sz, u32, i32, vp]),
                ("hyobfs_quic_new_protection_key", i32, [ctypes.c_uint16, vp, sz, u32,
                                                         ctypes.POINTER(HyobfsQuicKey)]),
                ("hyobfs_quic_hkdf_expand_label", i32, [vp, sz, ctypes.c_char_p, vp, sz, vp, sz]),
                ("hyobfs_quic_unprotect_batch", i32, [vp, vp, vp, u64, vp, u32, vp, vp, vp, vp]),
                ("hyobfs_quic_workspace_size", u64, [u64]),
                ("hyobfs_quic_read_crypto_payload_batch", i32, [vp, vp, vp, u64, vp, vp, vp, vp, vp, vp])):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        lib._quic_declared = True
    return lib


def _raise(st: int, what: str) -> None:
    if st in ERRORS:
        raise QuicError(st)
    _lib.check(st, what)


@dataclass(frozen=True)
class Header:
    """Header (header.go:13-20)."""
    type: int
    version: int
    src_connection_id: bytes
    dest_connection_id: bytes
    length: int
    token: bytes


def parse_initial_header(data: bytes) -> tuple[Header, int]:
    """ParseInitialHeader (header.go:24-32): (header, bytes read so far)."""
    data = bytes(data)
    h = HyobfsQuicHeader()
    st = _qlib().hyobfs_quic_parse_initial_header(data, len(data), ctypes.byref(h))
    if st:
        _raise(st, "parse_initial_header")
    cut = lambda o, n: data[o:o + n]  # noqa: E731
    return Header(h.type, h.version, cut(h.scid_off, h.scid_len), cut(h.dcid_off, h.dcid_len), h.length,
                  cut(h.token_off, h.token_len)), h.offset


def hkdf_expand_label(secret: bytes, label: str, context: bytes, length: int) -> bytes:
    """hkdfExpandLabel (packet_protector.go:177-193), SHA-256."""
    out = ctypes.create_string_buffer(max(length, 1))
    ctx = bytes(context)
    _raise(_qlib().hyobfs_quic_hkdf_expand_label(bytes(secret), len(secret), label.encode(), ctx, len(ctx), out,
                                                 length), "hkdf_expand_label")
    return out.raw[:length]


def initial_secret(dcid: bytes, version: int, server: bool = False) -> bytes:
    """HKDF-Extract(getSalt(v), dcid) -> "client in" / "server in" (payload.go:34-35)."""
    out = ctypes.create_string_buffer(32)
    dcid = bytes(dcid)
    _raise(_qlib().hyobfs_quic_initial_secret(dcid, len(dcid), version, int(server), out), "initial_secret")
    return out.raw


class ProtectionKey:
    """ProtectionKey (packet_protector.go:82-86): the derived key material."""

    def __init__(self, k: HyobfsQuicKey):
        self.raw = k

    @property
    def suite(self) -> int:
        return self.raw.suite

    @property
    def key(self) -> bytes:
        return bytes(self.raw.key)[:16 if self.suite == TLS_AES_128_GCM_SHA256 else 32]

    @property
    def iv(self) -> bytes:
        return bytes(self.raw.iv)

    @property
    def hp(self) -> bytes:
        return bytes(self.raw.hp)[:16 if self.suite == TLS_AES_128_GCM_SHA256 else 32]

    def record(self) -> np.ndarray:
        """The key as one KEY_DTYPE record (for a device key array)."""
        return np.frombuffer(bytes(self.raw), KEY_DTYPE).copy()


def new_protection_key(suite: int, secret: bytes, version: int) -> ProtectionKey:
    """NewProtectionKey (packet_protector.go:21-23, 102-156)."""
    k = HyobfsQuicKey()
    secret = bytes(secret)
    _raise(_qlib().hyobfs_quic_new_protection_key(suite, secret, len(secret), version, ctypes.byref(k)),
           "new_protection_key")
    return ProtectionKey(k)


def new_initial_protection_key(secret: bytes, version: int) -> ProtectionKey:
    """NewInitialProtectionKey (packet_protector.go:29-31): AES-128-GCM."""
    return new_protection_key(TLS_AES_128_GCM_SHA256, secret, version)


# ------------------------------------------------------------------ device batches
def workspace_size(n: int) -> int:
    return int(_qlib().hyobfs_quic_workspace_size(n))


def unprotect_batch(packets, off, lens, n: int, keys, pn_offset, res, *, key_stride: int = 1, pn_max=None,
                    stream=None) -> None:
    """hyobfs_quic_unprotect_batch: UnProtect n device packets in place; ``res``
    gets RESULT_DTYPE records.  Arguments are device tensors or pointers."""
    from .salamander import _ptr, _stream
    st = _qlib().hyobfs_quic_unprotect_batch(_ptr(packets), _ptr(off), _ptr(lens), n, _ptr(keys), key_stride,
                                             _ptr(pn_offset), _ptr(pn_max), _ptr(res), _stream(stream, res))
    _lib.check(st, "quic_unprotect_batch")


def read_crypto_payload_batch(packets, off, lens, n: int, out, out_off, out_cap, res, workspace,
                              stream=None) -> None:
    """hyobfs_quic_read_crypto_payload_batch: ReadCryptoPayload of n device
    packets (unprotected in place), CRYPTO data to out[out_off[i], +out_cap[i])."""
    from .salamander import _ptr, _stream
    st = _qlib().hyobfs_quic_read_crypto_payload_batch(_ptr(packets), _ptr(off), _ptr(lens), n, _ptr(out),
                                                       _ptr(out_off), _ptr(out_cap), _ptr(res), _ptr(workspace),
                                                       _stream(stream, res))
    _lib.check(st, "quic_read_crypto_payload_batch")


def _pack(packets):
    lens = np.array([len(p) for p in packets], np.uint32)
    off = np.zeros(len(packets), np.uint64)
    if len(packets) > 1:
        np.cumsum(lens[:-1], out=off[1:])
    buf = np.frombuffer(b"".join(bytes(p) for p in packets) + bytes(16), np.uint8).copy()
    return buf, off, lens


def _to(dev, a):
    import torch
    return torch.from_numpy(np.array(a, copy=True)).to(dev)   # writable copy (torch warns on read-only arrays)


def _records(t, dtype):
    return np.frombuffer(t.cpu().numpy().tobytes(), dtype)


class PacketProtector:
    """PacketProtector (packet_protector.go:38-43) on one GPU."""

    def __init__(self, key: ProtectionKey, device: int = 0):
        self.key = key
        self.device = device

    def unprotect_many(self, packets, pn_offsets, pn_max: int | list = 0):
        """UnProtect each packet: a list of (header bytes, plaintext) or QuicError."""
        import torch
        dev = torch.device("cuda", self.device)
        n = len(packets)
        buf, off, lens = _pack(packets)
        pmax = np.broadcast_to(np.asarray(pn_max, np.int64), (n,))
        d_buf = _to(dev, buf)
        d_res = torch.zeros(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        unprotect_batch(d_buf, _to(dev, off), _to(dev, lens), n, _to(dev, self.key.record().view(np.uint8)),
                        _to(dev, np.asarray(pn_offsets, np.int64)), d_res, key_stride=0, pn_max=_to(dev, pmax))
        res = _records(d_res, RESULT_DTYPE)
        host = d_buf.cpu().numpy()
        outs = []
        for i in range(n):
            if res[i]["status"]:
                outs.append(QuicError(int(res[i]["status"])))
                continue
            o, h = int(off[i]), int(res[i]["hdr_len"])
            outs.append((host[o:o + h].tobytes(), host[o + h:o + h + int(res[i]["plain_len"])].tobytes()))
        return outs

    def unprotect(self, packet: bytes, pn_offset: int, pn_max: int) -> bytes:
        """UnProtect (packet_protector.go:46-79): the decrypted payload."""
        r = self.unprotect_many([packet], [pn_offset], pn_max)[0]
        if isinstance(r, QuicError):
            raise r
        return r[1]


def read_crypto_payloads(packets, device: int = 0, out_cap: int = 4096):
    """ReadCryptoPayload over a list of packets on cuda:<device>: each entry is
    the assembled CRYPTO data or a QuicError."""
    import torch
    dev = torch.device("cuda", device)
    n = len(packets)
    buf, off, lens = _pack(packets)
    caps = np.full(n, out_cap, np.uint32)
    ooff = np.arange(n, dtype=np.uint64) * np.uint64(out_cap)
    d_out = torch.zeros(max(n * out_cap, 1), dtype=torch.uint8, device=dev)
    d_res = torch.zeros(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    ws = torch.empty(max(workspace_size(n), 1), dtype=torch.uint8, device=dev)
    read_crypto_payload_batch(_to(dev, buf), _to(dev, off), _to(dev, lens), n, d_out, _to(dev, ooff),
                              _to(dev, caps), d_res, ws)
    res = _records(d_res, RESULT_DTYPE)
    host = d_out.cpu().numpy()
    return [QuicError(int(r["status"])) if r["status"] else host[i * out_cap:i * out_cap + int(r["out_len"])].tobytes()
            for i, r in enumerate(res)]


def read_crypto_payload(packet: bytes, device: int = 0) -> bytes:
    """ReadCryptoPayload (payload.go:21-60)."""
    # assembled data is at most 256 KiB (several frames) or the packet length (one frame)
    r = read_crypto_payloads([packet], device, max(MAX_CRYPTO_PAYLOAD_LEN, len(packet)))[0]
    if isinstance(r, QuicError):
        raise r
    return r
