"""QUIC Initial unprotection kernels on the GPU (hysteria_amd/csrc/quic.hip)
against the oracle (oracle/quic_ref.py, pinned in tests/test_quic.py to
packet_protector_test.go:15-77)."""
import numpy as np
import pytest

import quic_cases as qc
from oracle import quic_ref as ref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _t(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _res(t):
    from hysteria_amd import quic
    return np.frombuffer(t.cpu().numpy().tobytes(), quic.RESULT_DTYPE)


def test_reference_vectors_on_device(dev):
    """TestInitialPacketProtector_UnProtect / TestPacketProtectorShortHeader_UnProtect
    (packet_protector_test.go:15-77) through PacketProtector on cuda:0, keys
    derived by the C ABI."""
    from hysteria_amd import quic
    hdr, offset = quic.parse_initial_header(qc.AES_PROTECTED)
    secret = quic.initial_secret(qc.AES_CONN_ID, hdr.version, server=True)
    pp = quic.PacketProtector(quic.new_initial_protection_key(secret, hdr.version))
    assert pp.unprotect(qc.AES_PROTECTED, offset, 1) == qc.AES_PLAIN
    k = quic.new_protection_key(quic.TLS_CHACHA20_POLY1305_SHA256, qc.CHACHA_SECRET, quic.V1)
    pn_len = (qc.CHACHA_HDR[0] & 3) + 1
    assert quic.PacketProtector(k).unprotect(qc.CHACHA_PROTECTED, len(qc.CHACHA_HDR) - pn_len,
                                             qc.CHACHA_PN_MAX) == qc.CHACHA_PLAIN
    with pytest.raises(quic.QuicError) as e:
        pp.unprotect(qc.AES_PROTECTED[:-1] + b"\x00", offset, 1)
    assert e.value.status == quic.ERR_AUTH


def test_unprotect_batch_vs_oracle(dev):
    from hysteria_amd import quic
    cases = qc.unprotect_cases(2) + qc.unprotect_cases(5)[2:]
    buf, off, lens = qc.pack([c[2] for c in cases])
    keys = np.frombuffer(b"".join(qc.key_record(c[1]) for c in cases), np.uint8).copy()
    d_buf = _t(dev, buf)
    d_res = torch.zeros(len(cases) * 24, dtype=torch.uint8, device=dev)
    quic.unprotect_batch(d_buf, _t(dev, off), _t(dev, lens), len(cases), _t(dev, keys),
                         _t(dev, np.array([c[3] for c in cases], np.int64)), d_res,
                         pn_max=_t(dev, np.array([c[4] for c in cases], np.int64)))
    qc.check_unprotect(cases, d_buf.cpu().numpy(), off, _res(d_res))


def test_read_crypto_payload_batch_vs_oracle(dev):
    """ReadCryptoPayload (payload.go:21-60) over every frame layout and error path."""
    from hysteria_amd import quic
    pkts = qc.crypto_packets(1) + qc.crypto_packets(9)
    buf, off, lens = qc.pack([x[1] for x in pkts])
    caps = np.full(len(pkts), 2048, np.uint32)
    caps[[i for i, x in enumerate(pkts) if x[0] == "zero_prefix"][:1]] = 1089   # one byte short: -51
    out_off = np.concatenate([[0], np.cumsum(caps[:-1], dtype=np.uint64)]).astype(np.uint64)
    d_out = torch.zeros(int(caps.sum()) + 64, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(len(pkts) * 24, dtype=torch.uint8, device=dev)
    ws = torch.empty(quic.workspace_size(len(pkts)), dtype=torch.uint8, device=dev)
    quic.read_crypto_payload_batch(_t(dev, buf), _t(dev, off), _t(dev, lens), len(pkts), d_out, _t(dev, out_off),
                                   _t(dev, caps), d_res, ws)
    out = d_out.cpu().numpy()
    qc.check_crypto(pkts, out, out_off, caps, _res(d_res))
    assert not out[int(caps.sum()):].any()


def test_read_crypto_payload_helpers(dev):
    from hysteria_amd import quic
    pkts = qc.crypto_packets(3)
    got = quic.read_crypto_payloads([p for _, p in pkts])
    for (name, p), g in zip(pkts, got):
        st, data = qc.oracle_read(p)
        if name == "too_many_frames":
            st = -52
        if st:
            assert isinstance(g, quic.QuicError) and g.status == st, name
        else:
            assert g == data, name
    assert quic.read_crypto_payload(pkts[0][1]) == qc.oracle_read(pkts[0][1])[1]


def test_read_crypto_payload_large_batch(dev):
    """100k packets from 64 oracle-made templates (1200-byte client Initials,
    V1 and V2, varied DCIDs, frame layouts, some tampered): every packet's result
    equals its template's, and the header is unmasked in place."""
    from hysteria_amd import quic
    rng = np.random.default_rng(11)
    temps = []
    for k in range(64):
        ch = qc.client_hello_like(rng, int(rng.integers(200, 600)))
        cut = int(rng.integers(1, len(ch)))
        frames = qc._crypto(cut, ch[cut:]) + b"\x00" * int(rng.integers(0, 40)) + qc._crypto(0, ch[:cut])
        dcid = rng.integers(0, 256, int(rng.integers(0, 21)), dtype=np.uint8).tobytes()
        version = ref.V2 if k % 2 else ref.V1
        pad = 1200 - (len(frames) + 16 + 7 + len(dcid) + 1 + 1 + 2 + 4)
        pkt = bytearray(ref.client_initial(dcid, b"", version, b"", 2, 4, frames + b"\x00" * max(pad, 0)))
        if k % 16 == 15:
            pkt[-5] ^= 0x20
        temps.append(bytes(pkt))
    expect = [qc.oracle_read(p) for p in temps]
    assert sum(st == 0 for st, _ in expect) == 60
    n = 100_000
    pick = rng.integers(0, 64, n)
    lens = np.array([len(temps[i]) for i in pick], np.uint32)
    off = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    tbuf = [np.frombuffer(t, np.uint8) for t in temps]
    buf = np.concatenate([tbuf[i] for i in pick] + [np.zeros(64, np.uint8)])
    cap = 1024
    out_off = np.arange(n, dtype=np.uint64) * np.uint64(cap)
    d_buf = _t(dev, buf)
    d_out = torch.zeros(n * cap, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(n * 24, dtype=torch.uint8, device=dev)
    ws = torch.empty(quic.workspace_size(n), dtype=torch.uint8, device=dev)
    quic.read_crypto_payload_batch(d_buf, _t(dev, off), _t(dev, lens), n, d_out, _t(dev, out_off),
                                   _t(dev, np.full(n, cap, np.uint32)), d_res, ws)
    res = _res(d_res)
    out = d_out.cpu().numpy().reshape(n, cap)
    hb = d_buf.cpu().numpy()
    st = res["status"]
    want_st = np.array([expect[i][0] for i in pick])
    assert np.array_equal(st, want_st)
    for t in range(64):
        rows = np.nonzero(pick == t)[0]
        if expect[t][0] == 0:
            d = np.frombuffer(expect[t][1], np.uint8)
            assert (res["out_len"][rows] == len(d)).all()
            assert (out[rows, :len(d)] == d).all(), t
        # header unmasked in place: the oracle's unprotected header
        hdr, hoff = ref.parse_initial_header(temps[t])
        key = ref.initial_protection_key(ref.initial_secret(hdr["dcid"], hdr["version"], False), hdr["version"])
        b = bytearray(temps[t][:hoff + hdr["length"]])
        try:
            h, _, _ = ref.unprotect(key, b, hoff, 2)
        except ref.QuicError:
            h = bytes(b[:hoff + 4])
        o = off[rows].astype(np.int64)
        for j in (0, len(h) - 1):
            assert (hb[o + j] == h[j]).all(), (t, j)
