"""QUIC Initial unprotection (extras/sniff/internal/quic): CPU tier.

1. The oracle (oracle/quic_ref.py) against the reference's own vectors
   (packet_protector_test.go:15-77) and published cipher vectors.
2. The host half of the C ABI (include/hyobfs_quic.h: header parse, HKDF,
   key derivation) against the oracle -- these entry points touch no GPU.
The device kernels run in tests/test_emulated_kernels.py (CPU emulation) and
tests/test_gpu_quic.py (MI355X).
"""
import numpy as np
import pytest

import quic_cases as qc
from hysteria_amd import quic
from oracle import quic_ref as ref


# ------------------------------------------------------------------ oracle pinning
def test_oracle_reference_vector_aes_server_initial():
    """TestInitialPacketProtector_UnProtect (packet_protector_test.go:15-53)."""
    hdr, offset = ref.parse_initial_header(qc.AES_PROTECTED)
    assert offset == 18 and hdr["version"] == 0xFF000020
    secret = ref.initial_secret(qc.AES_CONN_ID, hdr["version"], server=True)
    key = ref.initial_protection_key(secret, hdr["version"])
    _, plain, pn = ref.unprotect(key, bytearray(qc.AES_PROTECTED), offset, 1)
    assert plain == qc.AES_PLAIN and pn == 1


def test_oracle_reference_vector_chacha_short_header():
    """TestPacketProtectorShortHeader_UnProtect (packet_protector_test.go:55-77)."""
    key = ref.ProtectionKey(ref.TLS_CHACHA20_POLY1305_SHA256, qc.CHACHA_SECRET, ref.V1)
    pn_len = (qc.CHACHA_HDR[0] & 3) + 1
    offset = len(qc.CHACHA_HDR) - pn_len
    _, plain, pn = ref.unprotect(key, bytearray(qc.CHACHA_PROTECTED), offset, qc.CHACHA_PN_MAX)
    assert plain == qc.CHACHA_PLAIN and pn == 654360564   # RFC 9001 A.5


def test_oracle_published_cipher_vectors():
    # FIPS 197 C.1
    rk = ref.aes128_expand(bytes(range(16)))
    assert ref.aes128_encrypt_block(rk, bytes.fromhex("00112233445566778899aabbccddeeff")).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"
    # GCM spec test cases 1 and 2 (McGrew & Viega)
    assert ref.aes_gcm_open(bytes(16), bytes(12), bytes.fromhex("58e2fccefa7e3061367f1d57a4e7455a"), b"") == b""
    assert ref.aes_gcm_open(bytes(16), bytes(12), bytes.fromhex(
        "0388dace60b6a392f328c2b971b2fe78ab6e47d42cec13bdf53a67b21257bddf"), b"") == bytes(16)
    # RFC 8439 2.3.2 and 2.5.2
    assert ref.chacha20_block(bytes(range(32)), 1, bytes.fromhex("000000090000004a00000000"))[:16].hex() == \
        "10f1e7e4d13b5915500fdd1fa32071c4"
    assert ref.poly1305(bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b"),
                        b"Cryptographic Forum Research Group").hex() == "a8061dc1305136c6c22b8baf0c0127a9"
    # RFC 9001 A.1 client Initial keys
    s = ref.initial_secret(qc.AES_CONN_ID, ref.V1, server=False)
    assert s.hex() == "c00cf151ca5be075ed0ebfb5c80323c42d6b7db67881289af4008f1f6c357aea"
    k = ref.initial_protection_key(s, ref.V1)
    assert (k.key.hex(), k.iv.hex(), k.hp.hex()) == (
        "1f369613dd76d5467730efcbe3b1a22d", "fa044b2f42a3fd3b46fb255c", "9f50449e04a0e810283a1e9933adedd2")


def test_oracle_protect_roundtrip_and_tamper():
    for suite in (ref.TLS_AES_128_GCM_SHA256, ref.TLS_CHACHA20_POLY1305_SHA256):
        key = ref.ProtectionKey(suite, bytes(range(32)), ref.V2)
        hdr = bytes([0xC1]) + bytes(range(20)) + b"\x12\x34"
        pkt = ref.protect(key, hdr, 21, 0x1234, b"hello quic" * 7)
        h, plain, pn = ref.unprotect(key, bytearray(pkt), 21, 0x1200)
        assert (h, plain, pn) == (hdr, b"hello quic" * 7, 0x1234)
        bad = bytearray(pkt)
        bad[30] ^= 4
        with pytest.raises(ref.QuicError):
            ref.unprotect(key, bad, 21, 0x1200)


def test_oracle_decode_packet_number():
    """decodePacketNumber (packet_protector.go:161-174), RFC 9000 A.3's example."""
    assert ref.decode_packet_number(0xA82F30EA, 0x9B32, 2) == 0xA82F9B32
    assert ref.decode_packet_number(-1, 0, 1) == 0


def test_crypto_cases_cover_every_status():
    seen = {qc.oracle_read(p)[0] for _, p in qc.crypto_packets(1)}
    assert {0, -40, -41, -42, -43, -44, -45, -46, -47, -48, -49, -50} <= seen


# ------------------------------------------------------------------ host C ABI vs oracle
def test_abi_initial_secret_and_keys():
    rng = np.random.default_rng(3)
    for version in (ref.V1, ref.V2, 0xFF000020, 0):
        for dl in (0, 1, 8, 20, 55, 56, 64, 119, 255):
            dcid = rng.integers(0, 256, dl, dtype=np.uint8).tobytes()
            for server in (False, True):
                s = quic.initial_secret(dcid, version, server)
                assert s == ref.initial_secret(dcid, version, server)
            for suite in (quic.TLS_AES_128_GCM_SHA256, quic.TLS_CHACHA20_POLY1305_SHA256):
                k = quic.new_protection_key(suite, s, version)
                o = ref.ProtectionKey(suite, s, version)
                assert (k.key, k.iv, k.hp) == (o.key, o.iv, o.hp)
    with pytest.raises(quic.QuicError) as e:
        quic.new_protection_key(0x1302, bytes(32), ref.V1)   # TLS_AES_256_GCM_SHA384
    assert e.value.status == quic.ERR_SUITE


def test_abi_hkdf_expand_label():
    rng = np.random.default_rng(4)
    for n in (1, 12, 16, 32, 33, 64, 100, 255):
        secret = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        ctx = rng.integers(0, 256, n % 40, dtype=np.uint8).tobytes()
        assert quic.hkdf_expand_label(secret, "quic ku", ctx, n) == ref.hkdf_expand_label(secret, "quic ku", ctx, n)


def test_abi_parse_initial_header():
    for name, pkt in qc.crypto_packets(1):
        try:
            want, woff = ref.parse_initial_header(pkt)
            wst = 0
        except ref.QuicError as e:
            wst = qc.status_of(e)
        if wst:
            with pytest.raises(quic.QuicError) as e:
                quic.parse_initial_header(pkt)
            assert e.value.status == wst, name
            continue
        h, off = quic.parse_initial_header(pkt)
        assert off == woff, name
        assert (h.type, h.version, h.dest_connection_id, h.src_connection_id, h.token, h.length) == (
            want["type"], want["version"], want["dcid"], want["scid"], want["token"], want["length"]), name
    h, off = quic.parse_initial_header(qc.AES_PROTECTED)
    assert off == 18 and h.version == 0xFF000020 and h.dest_connection_id == b"" and h.length == 117


def test_abi_result_and_key_layouts():
    assert quic.KEY_DTYPE.itemsize == 80 and quic.RESULT_DTYPE.itemsize == 24
    assert quic.workspace_size(10) == 960
    key = ref.ProtectionKey(ref.TLS_AES_128_GCM_SHA256, bytes(range(32)), ref.V1)
    rec = np.frombuffer(qc.key_record(key), quic.KEY_DTYPE)[0]
    assert int(rec["suite"]) == 0x1301 and bytes(rec["iv"]) == key.iv and bytes(rec["key"][:16]) == key.key


def test_c_oracle_matches_python_oracle():
    """oracle/quic_ref.c (the CPU baseline) against oracle/quic_ref.py on every
    ReadCryptoPayload case, on 3 host threads."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    co = ref.CQuicOracle()
    pkts = qc.crypto_packets(1) + qc.crypto_packets(6)
    buf, off, lens = qc.pack([p for _, p in pkts])
    st, ol, out = co.read_batch(buf, off, lens, len(pkts), 4096, threads=3)
    for i, (name, p) in enumerate(pkts):
        s, d = qc.oracle_read(p)
        assert int(st[i]) == s, name
        if s == 0:
            assert out[i * 4096:i * 4096 + int(ol[i])].tobytes() == d, name
