"""Realm punch packets, CPU tier: the C-ABI codec (hyobfs_punch_*) against the
reference's own tests (extras/realm/punch_test.go) and the hashlib restatement
(oracle/realm_ref.py)."""
import random

import pytest

from hysteria_amd import realm
from hysteria_amd.realm import InvalidPunchPacketError, PunchMetadata
from oracle import realm_ref as rref

META = PunchMetadata("00112233445566778899aabbccddeeff",
                     "00112233445566778899aabbccddeeff00112233445566778899aabbccddeeff")
NONCE, KEY = bytes.fromhex(META.nonce), bytes.fromhex(META.obfs)


@pytest.mark.parametrize("ptype", [realm.PUNCH_HELLO, realm.PUNCH_ACK])
def test_encode_decode(ptype):
    """TestPunchPacketEncodeDecode (punch_test.go:12-29)."""
    p = realm.encode_punch_packet(ptype, META)
    assert realm.PUNCH_MIN_WIRE_LEN <= len(p) <= realm.PUNCH_MAX_WIRE_LEN
    assert b"HYRLMv1\x00" not in p
    assert realm.decode_punch_packet(p, META) == (ptype, len(p) - realm.PUNCH_MIN_WIRE_LEN)
    assert rref.decode(p, NONCE, KEY) == (ptype, len(p) - rref.MIN_WIRE)


def test_wire_bytes_match_restatement():
    rng = random.Random(1)
    for _ in range(300):
        salt, pad = rng.randbytes(8), rng.randbytes(rng.randrange(0, 1025))
        nonce, key = rng.randbytes(16), rng.randbytes(32)
        meta = PunchMetadata(nonce.hex(), key.hex())
        t = rng.choice([1, 2])
        assert realm.encode_punch_packet(t, meta, salt=salt, padding=pad) == rref.encode(t, nonce, key, salt, pad)
        assert realm.punch_mask(key, salt) == rref.mask(key, salt)


def test_mask_known_answer():
    """SHA-256 pinned: FIPS 180-4 / hashlib on the 40-byte key || salt block."""
    import hashlib
    key, salt = bytes(range(32)), b"12345678"
    assert realm.punch_mask(key, salt) == hashlib.sha256(key + salt).digest()


def test_rejects_wrong_metadata():
    """TestPunchPacketRejectsWrongMetadata (punch_test.go:31-49)."""
    p = realm.encode_punch_packet(realm.PUNCH_HELLO, META)
    for m in (PunchMetadata("f" * 32, META.obfs), PunchMetadata(META.nonce, "f" * 64)):
        with pytest.raises(InvalidPunchPacketError):
            realm.decode_punch_packet(p, m)


def test_salt_varies_wire_bytes():
    """TestPunchPacketSaltVariesWireBytes (punch_test.go:51-59)."""
    a = realm.encode_punch_packet(realm.PUNCH_HELLO, META)
    b = realm.encode_punch_packet(realm.PUNCH_HELLO, META)
    assert a[:8] != b[:8] and a != b


def test_rejects_corrupted_packet():
    """TestPunchPacketRejectsCorruptedPacket (punch_test.go:61-70): a flipped salt byte."""
    p = bytearray(realm.encode_punch_packet(realm.PUNCH_ACK, META))
    p[0] ^= 0xFF
    with pytest.raises(InvalidPunchPacketError):
        realm.decode_punch_packet(bytes(p), META)


def test_rejects_bad_lengths():
    """TestPunchPacketRejectsBadLengths (punch_test.go:72-82)."""
    for n in (realm.PUNCH_MIN_WIRE_LEN - 1, realm.PUNCH_MAX_WIRE_LEN + 1):
        with pytest.raises(InvalidPunchPacketError):
            realm.decode_punch_packet(bytes(n), META)


def test_rejects_unknown_type():
    """TestPunchPacketRejectsUnknownType (punch_test.go:84-102): valid magic and nonce, type 0xff."""
    salt = b"12345678"
    plain = b"HYRLMv1\x00" + b"\xff" + NONCE
    m = rref.mask(KEY, salt)
    p = salt + bytes(b ^ m[i % 32] for i, b in enumerate(plain))
    with pytest.raises(InvalidPunchPacketError, match="unknown packet type"):
        realm.decode_punch_packet(p, META)
    with pytest.raises(rref.PunchError):
        rref.decode(p, NONCE, KEY)


def test_rejects_bad_metadata():
    """TestPunchPacketRejectsBadMetadata (punch_test.go:104-118)."""
    for m in (PunchMetadata("not-hex", META.obfs), PunchMetadata(META.nonce, "not-hex"),
              PunchMetadata(META.nonce[:-2], META.obfs), PunchMetadata(META.nonce + "0", META.obfs)):
        with pytest.raises(InvalidPunchPacketError):
            realm.encode_punch_packet(realm.PUNCH_HELLO, m)


def test_padding_varies():
    """TestPunchPacketPaddingVaries (punch_test.go:120-133)."""
    seen = set()
    for _ in range(64):
        t, pad = realm.decode_punch_packet(realm.encode_punch_packet(realm.PUNCH_HELLO, META), META)
        assert 0 <= pad <= realm.MAX_PUNCH_PADDING
        seen.add(pad)
    assert len(seen) > 1


def test_decode_reasons_match_restatement():
    """Random corruptions: the C decoder and the restatement agree on accept/reject and reason."""
    rng = random.Random(9)
    reasons = {rref.TOO_SHORT: "too short", rref.TOO_LONG: "too long", rref.BAD_MAGIC: "bad magic",
               rref.UNKNOWN_TYPE: "unknown packet type", rref.NONCE_MISMATCH: "nonce mismatch"}
    for _ in range(2000):
        p = bytearray(rref.encode(rng.choice([1, 2]), NONCE, KEY, rng.randbytes(8), rng.randbytes(rng.randrange(40))))
        k = rng.randrange(5)
        if k == 1:
            p[8 + rng.randrange(8)] ^= 1 << rng.randrange(8)       # magic
        elif k == 2:
            p[16] ^= rng.choice([1, 2, 3, 0x80])                    # type
        elif k == 3:
            p[17 + rng.randrange(16)] ^= 1                          # nonce
        elif k == 4:
            p = p[:rng.randrange(rref.MIN_WIRE)]                   # length
        try:
            exp = rref.decode(bytes(p), NONCE, KEY)
        except rref.PunchError as e:
            with pytest.raises(InvalidPunchPacketError, match=reasons[e.reason]):
                realm.decode_punch_packet(bytes(p), META)
            continue
        assert realm.decode_punch_packet(bytes(p), META) == exp


def test_new_metadata_shape():
    """client_test.go:173-176: hex strings of 2 x 16 and 2 x 32 characters."""
    m = realm.new_punch_metadata()
    assert len(m.nonce) == 32 and len(m.obfs) == 64
    int(m.nonce, 16), int(m.obfs, 16)
    assert realm.decode_punch_packet(realm.encode_punch_packet(1, m), m)[0] == 1
