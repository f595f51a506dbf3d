"""CPU tests: the oracle pinned against known answers and golden fixtures.

Mirrors the reference's own test (extras/obfs/salamander_test.go:32-45:
1000 x 1200-byte payloads, PSK "average_password", round-trip identity) and
adds the known-answer checks the reference lacks.
"""
import hashlib
import os
import random

import numpy as np
import pytest

from oracle import salamander_ref as ref


def test_blake2b_kat_rfc7693(coracle, golden):
    kat = golden[0]["hash_kat"]
    assert coracle.blake2b(b"abc", 64).hex() == kat["rfc7693_appendix_a_blake2b512_abc"]
    assert coracle.blake2b(b"abc", 32).hex() == kat["blake2b256_abc"]
    assert coracle.blake2b(b"", 32).hex() == kat["blake2b256_empty"]


def test_blake2b_c_matches_hashlib_all_lengths(coracle):
    rng = random.Random(5)
    for n in list(range(0, 300)) + [383, 384, 385, 1000]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        for outlen in (32, 64):
            assert coracle.blake2b(data, outlen) == hashlib.blake2b(data, digest_size=outlen).digest(), n


def test_survey_spot_values(golden):
    s = golden[0]["survey_spot"]
    psk, salt = bytes.fromhex(s["psk"]), bytes.fromhex(s["salt"])
    assert ref.key(psk, salt).hex() == s["key"]
    assert ref.obfuscate(psk, bytes.fromhex(s["payload"]), salt).hex() == s["wire"]
    assert ref.key(bytes.fromhex(s["two_block_psk"]), salt).hex() == s["two_block_key"]


@pytest.mark.parametrize("impl", ["python", "c"])
def test_golden_vectors(impl, coracle, golden):
    for v in golden[0]["vectors"]:
        psk, salt = bytes.fromhex(v["psk"]), bytes.fromhex(v["salt"])
        payload = ref.stream_bytes(v["payload_seed"], v["payload_start"], v["payload_len"])
        if "payload" in v:
            assert payload.hex() == v["payload"]
        if impl == "python":
            k = ref.key(psk, salt)
            wire = ref.obfuscate(psk, payload, salt)
            back = ref.deobfuscate(psk, wire)
        else:
            k = coracle.key(psk, salt)
            wire = coracle.obfuscate(psk, payload, salt, len(payload) + 8)
            back = coracle.deobfuscate(psk, wire, len(payload))
        assert k.hex() == v["key"]
        assert len(wire) == v["wire_len"] == len(payload) + 8
        assert hashlib.sha256(wire).hexdigest() == v["wire_sha256"]
        if "wire" in v:
            assert wire.hex() == v["wire"]
        if v["payload_len"] > 0:
            assert back == payload
        else:
            assert back == b""   # an 8-byte salt-only datagram is rejected (salamander.go:75-76)


def test_reference_roundtrip_1000x1200(coracle):
    """TestSalamanderObfuscator (salamander_test.go:32-45), with seeded salts."""
    psk = b"average_password"
    rng = np.random.default_rng(1)
    for i in range(1000):
        payload = rng.integers(0, 256, 1200, dtype=np.uint8).tobytes()
        salt = ref.splitmix64_at(2, i).to_bytes(8, "little")
        wire = coracle.obfuscate(psk, payload, salt, 2048)
        assert len(wire) == len(payload) + ref.SM_SALT_LEN
        back = coracle.deobfuscate(psk, wire, 2048)
        assert back == payload
        if i % 100 == 0:
            assert wire == ref.obfuscate(psk, payload, salt)


def test_edge_rules(coracle):
    psk = b"average_password"
    salt = b"\x01" * 8
    # Obfuscate: len(out) < len(in)+8 -> 0 (salamander.go:60-62)
    assert coracle.obfuscate(psk, b"x" * 10, salt, 17) == b""
    assert len(coracle.obfuscate(psk, b"x" * 10, salt, 18)) == 18
    # empty payload -> salt-only datagram
    assert coracle.obfuscate(psk, b"", salt, 8) == salt
    # Deobfuscate: len(in) <= 8 -> 0 (salamander.go:75-76); out too small -> 0 (:76-77)
    for n in (0, 1, 7, 8):
        assert coracle.deobfuscate(psk, b"\x00" * n, 2048) == b""
    assert coracle.deobfuscate(psk, b"\x00" * 20, 11) == b""
    assert len(coracle.deobfuscate(psk, b"\x00" * 20, 12)) == 12
    with pytest.raises(ref.PSKTooShortError):
        ref.check_psk(b"abc")
    ref.check_psk(b"abcd")


def test_splitmix_python_matches_c(coracle):
    assert ref.stream_bytes(1, 13, 1000) == coracle.fill_stream(1, 13, 1000).tobytes()
    assert list(ref.splitmix64_array(2, 5, 100)) == list(coracle.salts(2, 5, 100))
    assert np.array_equal(ref.bimodal_lengths(3, 0, 1000), coracle.bimodal_lengths(3, 0, 1000))
    frac64 = float((ref.bimodal_lengths(3, 0, 100_000) == 64).mean())
    assert abs(frac64 - 0.4) < 0.01


def _python_batch(obf, psk, lens, inp, in_off, salts, out_cap, out_stride, pkt_cap):
    """Per-packet reference loop (python restatement) defining the batch rules."""
    out = bytearray(out_cap)
    offs, olens, cursor = [], [], 0
    for i, L in enumerate(lens):
        L, o = int(L), int(in_off[i])
        src = bytes(inp[o: o + L])
        W = L + 8 if obf else L - 8
        cap = pkt_cap if pkt_cap else 1 << 62
        if out_stride:
            cap = min(cap, out_stride)
        valid = W > 0 and W <= cap
        if not valid:
            W = 0
        off = i * out_stride if out_stride else cursor
        if not out_stride:
            cursor += W
        if valid and off + W > out_cap:
            valid, W = False, 0
        offs.append(off)
        olens.append(W)
        if valid:
            if obf:
                res = ref.obfuscate(psk, src, int(salts[i]).to_bytes(8, "little"))
            else:
                res = ref.deobfuscate(psk, src)
            assert len(res) == W
            out[off: off + W] = res
    return bytes(out), offs, olens


@pytest.mark.parametrize("obf", [True, False])
@pytest.mark.parametrize("layout", ["packed", "slotted", "capped"])
def test_batch_rules_c_vs_python(coracle, obf, layout):
    rng = np.random.default_rng(11)
    n = 300
    lens = rng.integers(0, 2100, n).astype(np.uint32)
    lens[:12] = [0, 1, 7, 8, 9, 15, 16, 17, 2040, 2041, 2048, 2049]
    gaps = rng.integers(0, 5, n)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum((lens + gaps)[:-1], dtype=np.uint64)
    inp = rng.integers(0, 256, int(in_off[-1] + lens[-1] + 16), dtype=np.uint8)
    salts = ref.splitmix64_array(2, 0, n)
    psk = b"average_password"
    out_stride, pkt_cap = 0, 0
    out_cap = int(lens.sum()) + 8 * n
    if layout == "slotted":
        out_stride, out_cap = 2048, 2048 * n
    elif layout == "capped":
        pkt_cap, out_cap = 2048, out_cap // 2
    exp, eoff, elen = _python_batch(obf, psk, lens, inp, in_off, salts, out_cap, out_stride, pkt_cap)
    got, goff, glen, tot = coracle.batch(obf, psk, n, inp, in_off=in_off, in_len=lens,
                                         salts=salts if obf else None, out_cap=out_cap,
                                         out_stride=out_stride, pkt_cap=pkt_cap)
    assert list(goff) == eoff
    assert list(glen) == elen
    assert tot == sum(elen)
    assert got.tobytes() == exp


def test_config1_digest_independent_of_c(golden):
    """10k x 1200 (BASELINE configs[0]) digest, recomputed by the hashlib restatement."""
    d = golden[1]["config1_cpu_10k_x_1200"]
    n, L = d["n"], d["len"]
    psk = b"average_password"
    stream = ref.stream_bytes(1, 0, n * L)
    salts = ref.splitmix64_array(2, 0, n)
    h = hashlib.sha256()
    for i in range(n):
        h.update(ref.obfuscate(psk, stream[i * L:(i + 1) * L], int(salts[i]).to_bytes(8, "little")))
    assert h.hexdigest() == d["obf_sha256"]


def test_small_batch_digests_c(coracle, golden):
    d = golden[1]["small_64k_x_1200"]
    n, L = d["n"], d["len"]
    inp = coracle.fill_stream(1, 0, n * L)
    wire, _, _, _ = coracle.batch(True, b"average_password", n, inp, in_stride=L, len_uniform=L,
                                  salts=coracle.salts(2, 0, n), out_cap=n * (L + 8))
    assert hashlib.sha256(wire.tobytes()).hexdigest() == d["obf_sha256"]
