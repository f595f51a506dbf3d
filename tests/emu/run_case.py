"""Run batches through the CPU-emulated kernels (tests/emu/libhyobfs_emu.so)
and compare with the C oracle.  Invoked by tests/test_emulated_kernels.py in a
subprocess with the ASan runtime preloaded."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

os.environ.setdefault("HYOBFS_LIB", os.path.join(ROOT, "tests", "emu", "libhyobfs_emu.so"))
from hysteria_amd import _lib  # noqa: E402
from hysteria_amd.salamander import SalamanderObfuscator  # noqa: E402
from oracle import salamander_ref as ref  # noqa: E402


def run(obf, psk, lens, in_off, inp, salts, out_cap, out_stride=0, pkt_cap=0, in_stride=0, len_uniform=0,
        contiguous=False, expect_kernel=None, expect_ws=None):
    n = len(lens) if lens is not None else len(salts)
    co = ref.COracle()
    exp, eoff, elen, etot = co.batch(obf, psk, n, inp, in_off=in_off, in_stride=in_stride, in_len=lens,
                                     len_uniform=len_uniform, salts=salts if obf else None, out_cap=out_cap,
                                     out_stride=out_stride, pkt_cap=pkt_cap)
    out = np.full(out_cap + 64, 0xA5, np.uint8)
    out_off = np.zeros(max(n, 1), np.uint64)
    out_len = np.zeros(max(n, 1), np.uint32)
    total = np.zeros(1, np.uint64)
    o = SalamanderObfuscator(psk, 0)
    p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    kw = dict(in_off=None if contiguous else p(in_off), in_stride=in_stride, in_len=p(lens), len_uniform=len_uniform,
              out=p(out), out_cap=out_cap, out_stride=out_stride, pkt_cap=pkt_cap, out_off=p(out_off),
              out_len=p(out_len), out_total=p(total), stream=0)
    if expect_kernel:
        got_k = o.batch_kernel(obf, inp=p(inp), n=n, **{k: v for k, v in kw.items() if k != "stream"},
                               **({"salts": p(salts)} if obf else {}))
        want_k = os.environ.get("HYOBFS_KERNEL") == "wave" and "wave" or expect_kernel
        assert got_k == want_k, ("kernel", got_k, want_k)
    if expect_ws is not None:   # hyobfs_batch_workspace_bytes, then a caller workspace of exactly that size
        need = SalamanderObfuscator.workspace_bytes(inp=p(inp), n=n, **{k: v for k, v in kw.items() if k != "stream"})
        assert need == expect_ws, ("workspace_bytes", need, expect_ws)
        ws = np.zeros(need, np.uint8)   # ASan: a scratch overrun is a heap-buffer-overflow
        kw.update(workspace=p(ws), workspace_bytes=need)
    if obf:
        o.obfuscate_batch(p(inp), n, salts=p(salts), **kw)
    else:
        o.deobfuscate_batch(p(inp), n, **kw)
    o.close()
    assert np.array_equal(out_off[:n], eoff), "out_off"
    assert np.array_equal(out_len[:n], elen), "out_len"
    assert int(total[0]) == etot, ("total", int(total[0]), etot)
    written = np.zeros(out_cap + 64, bool)
    for off, w in zip(eoff, elen):
        written[int(off):int(off) + int(w)] = True
    bad = np.nonzero(written[:out_cap] & (out[:out_cap] != exp))[0]
    assert bad.size == 0, ("mismatch", bad[:10], bad.size)
    assert (out[~written] == 0xA5).all(), "wrote outside regions"


def case_ragged(seed, n, maxlen, obf, layout, psk=b"average_password"):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, n).astype(np.uint32)
    gaps = rng.integers(0, 4, n)
    in_off = np.zeros(n, np.uint64)
    in_off[0] = 5
    in_off[1:] = 5 + np.cumsum((lens + gaps)[:-1], dtype=np.uint64)
    inp = rng.integers(0, 256, int(in_off[-1] + lens[-1] + 32), dtype=np.uint8)
    salts = ref.splitmix64_array(2, 0, n)
    cap = int(lens.sum()) + 8 * n + 16
    stride = 0
    if layout == "slotted":
        stride = maxlen + 8
        cap = stride * n
    run(obf, psk, lens, in_off, inp, salts, cap, out_stride=stride)


def case_packed_cap(seed, n, maxlen, obf, cap_pct, psk_len):
    """Packed output with out_cap cut to cap_pct % of the full size (the regions past
    it, and every later one, dropped), in_off with gaps, a PSK of psk_len bytes; for
    deobfuscate the input is real wire bytes."""
    rng = np.random.default_rng(seed)
    psk = bytes((5 * i + 3) & 0xFF for i in range(psk_len))
    lens = rng.integers(0, maxlen, n).astype(np.uint32)
    gaps = rng.integers(0, 5, n)
    in_off = np.zeros(n, np.uint64)
    in_off[0] = 3
    in_off[1:] = 3 + np.cumsum((lens + gaps)[:-1], dtype=np.uint64)
    inp = rng.integers(0, 256, int(in_off[-1] + lens[-1] + 32), dtype=np.uint8)
    salts = ref.splitmix64_array(2, 0, n)
    if not obf:
        co = ref.COracle()
        cap = int(lens.sum()) + 8 * n
        wire, woff, wlen, _ = co.batch(True, psk, n, inp, in_off=in_off, in_len=lens, salts=salts, out_cap=cap)
        inp, in_off, lens = wire, woff, wlen
    full = int(lens.sum()) + (8 * n if obf else 0)
    run(obf, psk, lens, in_off, inp, salts, max(16, full * cap_pct // 100))


def case_contig(seed, n, dist, obf, cap_pct, psk_len, pkt_cap=0, misalign=0, out_stride=0):
    """Contiguous input (in_off NULL, in_stride 0: datagram i right after datagram
    i-1) into packed output (out_stride 0: the wave kernel scans the lengths itself,
    with HYOBFS_PACKED_RUN_LOG2 < 6 a prepass writes the input offsets; with
    HYOBFS_KERNEL=flat and 16-byte aligned input the flat kernel)
    or into slots of out_stride bytes (the prepass's offsets, then the wave kernel).  dist 0: the
    bimodal 64/1350 mix; 1: 0..2100 B; 2: 0..40 B (several datagrams per chunk);
    3: 1000..5000 B; 4: bimodal with zero-length ones.  out_cap cut to cap_pct % of
    the full size, pkt_cap drops, deobfuscate of real wire (8-byte wire datagrams
    dropped), misalign = input not 16-byte aligned.  The call gets a caller workspace
    of exactly hyobfs_batch_workspace_bytes, whose value is checked."""
    rng = np.random.default_rng(seed)
    psk = bytes((11 * i + 5) & 0xFF for i in range(psk_len))
    if dist == 0:
        lens = ref.bimodal_lengths(3, seed, n)
    elif dist == 1:
        lens = rng.integers(0, 2100, n).astype(np.uint32)
    elif dist == 2:
        lens = rng.integers(0, 41, n).astype(np.uint32)
    elif dist == 3:
        lens = rng.integers(1000, 5000, n).astype(np.uint32)
    else:
        lens = ref.bimodal_lengths(3, seed, n)
        lens[rng.random(n) < 0.05] = 0
    lens = np.ascontiguousarray(lens, np.uint32)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum())
    buf = np.zeros(total + 64 + 16, np.uint8)
    base = (-buf.ctypes.data) % 16 + misalign
    inp = buf[base:base + total + 32]
    inp[:total] = rng.integers(0, 256, total, dtype=np.uint8)
    salts = ref.splitmix64_array(2, seed, n)
    if not obf:
        co = ref.COracle()
        cap = total + 8 * n
        wire, woff, wlen, _ = co.batch(True, psk, n, inp, in_off=in_off, in_len=lens, salts=salts, out_cap=cap)
        wl = int(wlen.sum())
        wbuf = np.zeros(wl + 64 + 16, np.uint8)
        wb = (-wbuf.ctypes.data) % 16 + misalign
        winp = wbuf[wb:wb + wl + 32]
        winp[:wl] = wire[:wl]
        # the wire is contiguous: datagrams back to back, as their out_off say
        assert np.array_equal(woff[1:], np.cumsum(wlen[:-1], dtype=np.uint64))
        inp, in_off, lens, total = winp, woff, np.ascontiguousarray(wlen, np.uint32), wl
    full = n * out_stride if out_stride else total + (8 * n if obf else 0)
    cap = max(16, full * cap_pct // 100)
    tsums = ((n + 255) // 256 + 1) * 8
    # packed output from 16-byte aligned input: the flat kernel when asked for (HYOBFS_KERNEL=flat)
    flat = not out_stride and not misalign and os.environ.get("HYOBFS_KERNEL") == "flat"
    prepass = out_stride or os.environ.get("HYOBFS_PACKED_RUN_LOG2", "6") != "6"
    # hyobfs_batch_workspace_bytes: the largest need over the kernel choices
    ws = 2 * tsums + (8 * n if prepass else 0)   # the wave kernel's
    if not out_stride and not misalign:           # the flat kernel's tile descriptors (16 KiB tiles)
        desc = 16 + 24 * ((cap + 16383) // 16384 + 1)   # + the hashers' key records, 64 B per datagram
        ws = max(ws, 2 * tsums + ((desc + 255) // 256) * 256 + 256 + 64 * n)
    run(obf, psk, lens, in_off, inp, salts, cap, pkt_cap=pkt_cap, contiguous=True,
        out_stride=out_stride, expect_kernel="flat" if flat else "wave", expect_ws=ws)


def case_bimodal(n, obf):
    lens = ref.bimodal_lengths(3, 0, n)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    inp = np.frombuffer(ref.stream_bytes(1, 0, int(lens.sum()) + 16), np.uint8).copy()
    salts = ref.splitmix64_array(2, 0, n)
    if not obf:   # feed real wire bytes
        co = ref.COracle()
        cap = int(lens.sum()) + 8 * n
        wire, woff, wlen, _ = co.batch(True, b"average_password", n, inp, in_off=in_off, in_len=lens, salts=salts,
                                       out_cap=cap)
        run(False, b"average_password", wlen, woff, wire, None, int(lens.sum()) + 16)
    else:
        run(True, b"average_password", lens, in_off, inp, salts, int(lens.sum()) + 8 * n)


def case_uniform(n, L, obf):
    inp = np.frombuffer(ref.stream_bytes(1, 0, n * (L + 8) + 16), np.uint8).copy()
    salts = ref.splitmix64_array(2, 0, n)
    if obf:
        run(True, b"average_password", None, None, inp, salts, n * (L + 8), out_stride=L + 8, in_stride=L,
            len_uniform=L)
    else:
        run(False, b"average_password", None, None, inp, salts, n * L, out_stride=L, in_stride=L + 8,
            len_uniform=L + 8)


def case_slotted(n, L, obf, slot_pad, in_pad, psk_len, exact=0):
    """Uniform lengths into slots of W + slot_pad bytes (gap bytes must stay
    untouched), inputs at a stride of L + in_pad, a PSK of psk_len bytes.  exact=1:
    the input buffer ends right after the last datagram's L bytes ((n-1) stride + L,
    the API's promise; ASan reports any read past it, e.g. the tile kernel's prefetch
    of a short datagram in a long slot)."""
    psk = bytes((7 * i + 1) & 0xFF for i in range(psk_len))
    W = L + 8 if obf else L - 8
    stride, istride = W + slot_pad, L + in_pad
    if exact:
        size = (n - 1) * istride + L
        raw = np.empty(size + 15, np.uint8)
        off = (-raw.ctypes.data) % 16   # 16-byte aligned start (the tile kernel's condition)
        inp = raw[off:off + size]
        inp[:] = np.frombuffer(ref.stream_bytes(1, 0, size), np.uint8)
    else:
        inp = np.frombuffer(ref.stream_bytes(1, 0, n * istride + 16), np.uint8).copy()
    salts = ref.splitmix64_array(2, 0, n)
    run(obf, psk, None, None, inp, salts, n * stride, out_stride=stride, in_stride=istride, len_uniform=L)


def case_slotted_far(n, L, stride_mb, obf):
    """Slotted output whose slots sit beyond 2^31: the output buffer is an untouched
    anonymous mapping, so only the written slots cost memory."""
    import mmap
    stride = stride_mb << 20
    cap = n * stride
    mm = mmap.mmap(-1, cap + 4096)
    out = np.frombuffer(mm, np.uint8)
    rng = np.random.default_rng(n)
    inp = rng.integers(0, 256, n * L + 64, dtype=np.uint8)
    salts = ref.splitmix64_array(2, 0, n)
    o = SalamanderObfuscator(b"average_password", 0)
    if obf:
        o.obfuscate_batch(inp.ctypes.data, n, in_stride=L, len_uniform=L, salts=salts.ctypes.data,
                          out=out.ctypes.data, out_cap=cap, out_stride=stride, stream=0)
    else:
        o.deobfuscate_batch(inp.ctypes.data, n, in_stride=L, len_uniform=L, out=out.ctypes.data, out_cap=cap,
                            out_stride=stride, stream=0)
    o.close()
    for i in range(n):
        src = inp[i * L:(i + 1) * L].tobytes()
        exp = ref.obfuscate(b"average_password", src, int(salts[i]).to_bytes(8, "little")) if obf \
            else ref.deobfuscate(b"average_password", src)
        got = out[i * stride:i * stride + len(exp)].tobytes()
        assert got == exp, i
        assert not out[i * stride + len(exp):i * stride + len(exp) + 16].any()
    del out
    mm.close()


def case_host(n, L, chunk, obf, mapped=0):
    """Host-resident slotted batch through the three-slot pipeline (chunked); mapped=1:
    every array from hyobfs_host_alloc, so the batch runs zero-copy on the mapped
    memory (one batch call) and bytes outside the datagrams' regions stay untouched."""
    import ctypes
    from hysteria_amd import _lib
    rng = np.random.default_rng(n + L)
    stride_in = L + 24
    lens = rng.integers(0, L + 1, n).astype(np.uint32)
    lens[:4] = [0, 8, 9, L]
    inp = rng.integers(0, 256, n * stride_in, dtype=np.uint8)
    salts = ref.splitmix64_array(2, 0, n)
    out_stride = L + 8 if obf else L
    out = np.full(n * out_stride, 0xA5, np.uint8)
    out_len = np.zeros(n, np.uint32)
    held = []
    if mapped:
        lib = _lib.load()

        def host(a):   # a copy of array a in mapped pinned memory (hyobfs_host_alloc)
            ptr = lib.hyobfs_host_alloc(a.nbytes)
            assert ptr
            held.append(ptr)
            m = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (a.nbytes,)).view(a.dtype)
            m[:] = a
            return m
        inp, lens, salts, out, out_len = host(inp), host(lens), host(salts), host(out), host(out_len)
    o = SalamanderObfuscator(b"average_password", 0)
    if obf:
        o.obfuscate_host(inp, n, in_stride=stride_in, in_len=lens, salts=salts, out=out, out_stride=out_stride,
                         out_len=out_len, chunk=chunk)
    else:
        o.deobfuscate_host(inp, n, in_stride=stride_in, in_len=lens, out=out, out_stride=out_stride,
                           out_len=out_len, chunk=chunk)
    o.close()
    for i in range(n):
        src = inp[i * stride_in:i * stride_in + int(lens[i])].tobytes()
        if obf:
            exp = ref.obfuscate(b"average_password", src, int(salts[i]).to_bytes(8, "little"), out_stride)
        else:
            exp = ref.deobfuscate(b"average_password", src, out_stride)
        assert int(out_len[i]) == len(exp), (i, int(out_len[i]), len(exp))
        assert out[i * out_stride:i * out_stride + len(exp)].tobytes() == exp, i
    if mapped:
        untouched = np.ones(n * out_stride, bool)
        for i in range(n):
            untouched[i * out_stride:i * out_stride + int(out_len[i])] = False
        assert (out[untouched] == 0xA5).all()
        del inp, lens, salts, out, out_len
        for ptr in held:
            lib.hyobfs_host_free(ptr)


def case_gecko(n_msgs, seed, layout=0):
    """Gecko frames: one device encode pass vs oracle/gecko_ref, then deobfuscate + parse.
    layout 0: packed wire order (the aligned sweep); 1: ascending with gaps between
    frames (aligned sweep, gap bytes untouched); 2: frames placed in shuffled order
    (the per-frame path); 3: tiny frames packed back to back (0..40 pad bytes,
    1..20 message bytes: several frames per 16-byte chunk)."""
    from hysteria_amd import gecko
    from oracle import gecko_ref as gref
    psk = b"average_password"
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 1400, n_msgs)
    lens[:3] = [1, 5, 2000][:min(3, n_msgs)]
    msg = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    fr, off, total = gecko.plan_fragments(lens, 400, 900, first_msg_id=seed)
    nf = len(fr)
    if layout == 3:
        nf = n_msgs
        cl = rng.integers(1, 21, nf)
        pl = rng.choice([0, 1, 2, 3, 17, 40], nf)
        tot = rng.integers(2, 9, nf)
        fr = np.array([(int(rng.integers(0, len(msg) - 24)), int(cl[i]), int(pl[i]), i & 0xff,
                        int(rng.integers(0, tot[i])) << 4 | int(tot[i])) for i in range(nf)], dtype=gecko.FRAME_DTYPE)
        w = (13 + cl + pl).astype(np.uint64)
        off = np.concatenate([[5], 5 + np.cumsum(w)[:-1]]).astype(np.uint64)
        total = int(5 + w.sum())
    elif layout:
        widths = np.diff(np.append(off, total)).astype(np.uint64)
        order = rng.permutation(nf) if layout == 2 else np.arange(nf)
        gaps = rng.integers(0, 41, nf).astype(np.uint64) if layout == 1 else np.zeros(nf, np.uint64)
        pos = np.zeros(nf, np.uint64)
        cur = np.uint64(3)
        for i in order:
            pos[i] = cur
            cur += widths[i] + gaps[i]
        off, total = pos, int(cur)
    salts = ref.splitmix64_array(5, 0, nf)
    out = np.full(total + 64, 0xA5, np.uint8)
    o = SalamanderObfuscator(psk, 0)
    p = lambda a: a.ctypes.data  # noqa: E731
    key, nonce = bytes(range(3, 35)), bytes(range(40, 52))
    gecko.encode_batch(o, msg=p(msg), frames=p(fr), salts=p(salts), pad_key=key, pad_nonce=nonce, out=p(out),
                       out_off=p(off), n=nf, stream=0)
    exp = gref.encode_wire(psk, msg.tobytes(), fr.tolist(), salts, key, nonce, off)
    assert out[total:].tobytes() == b"\xa5" * 64
    written = np.zeros(total + 64, bool)
    for i in range(nf):
        assert out[int(off[i]):int(off[i]) + len(exp[i])].tobytes() == exp[i], i
        written[int(off[i]):int(off[i]) + len(exp[i])] = True
    assert (out[~written] == 0xA5).all(), "wrote outside the frames"
    # back: Salamander deobfuscate batch, then the Gecko parse kernel
    wl = np.array([len(e) for e in exp], np.uint32)
    plain = np.zeros(total, np.uint8)
    poff = np.zeros(nf, np.uint64)
    plen = np.zeros(nf, np.uint32)
    o.deobfuscate_batch(p(out), nf, in_off=p(off), in_len=p(wl), out=p(plain), out_cap=total, out_off=p(poff),
                        out_len=p(plen), stream=0)
    parsed = np.zeros(nf + 1, gecko.PARSED_DTYPE)
    garbage = np.frombuffer(bytes([0x80, 1, 0x44, 0, 0]), np.uint8).copy()
    gecko.parse_batch(p(plain), p(poff), p(plen), nf, p(parsed), stream=0)
    o.close()
    for i in range(nf):
        d = plain[int(poff[i]):int(poff[i]) + int(plen[i])].tobytes()
        kind, h, payload = gref.parse(d)
        assert kind == gref.FRAGMENT and int(parsed[i]["status"]) == gecko.FRAGMENT, i
        assert int(parsed[i]["msg_id"]) == h.msg_id and int(parsed[i]["pad_len"]) == h.pad_len
        assert int(parsed[i]["idx_total"]) == (h.chunk_idx << 4 | h.total_chunks)
        po, pl = int(parsed[i]["payload_off"]), int(parsed[i]["payload_len"])
        assert d[po:po + pl] == payload
    gecko.parse_batch(p(garbage), p(np.zeros(1, np.uint64)), p(np.array([5], np.uint32)), 1, p(parsed), stream=0)
    assert int(parsed[0]["status"]) == gecko.ERR_INVALID


def case_punch(n, m, seed):
    from hysteria_amd import realm
    from oracle import realm_ref as rref
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from punch_cases import punch_batch
    pk, atts, metas = punch_batch(n, m, seed)
    buf = np.frombuffer(b"".join(pk) + bytes(16), np.uint8).copy()
    off = np.concatenate([[0], np.cumsum([len(x) for x in pk])[:-1]]).astype(np.uint64)
    ln = np.array([len(x) for x in pk], np.uint32)
    match = np.full(n, -7, np.int32)
    ty = np.zeros(n, np.uint8)
    pad = np.zeros(n, np.uint32)
    mt = realm.PunchMatcher(metas)
    p = lambda a: a.ctypes.data  # noqa: E731
    mt.match_batch(p(buf), p(off), p(ln), n, p(match), p(ty), p(pad), attempts=p(mt.attempts), stream=0)
    hits = 0
    for i, x in enumerate(pk):
        j, t, pd = rref.match(x, atts)
        assert (int(match[i]), int(ty[i]) if j >= 0 else 0, int(pad[i])) == (j, t, pd), (i, int(match[i]), j)
        hits += j >= 0
    assert 0 < hits < n


def case_quic(seed):
    """QUIC Initial unprotection: explicit-key UnProtect batch (both suites,
    the reference's two vectors) and the ReadCryptoPayload batch vs the oracle."""
    from hysteria_amd import quic
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import quic_cases as qc
    p = lambda a: a.ctypes.data  # noqa: E731
    cases = qc.unprotect_cases(seed)
    buf, off, lens = qc.pack([c[2] for c in cases])
    keys = np.frombuffer(b"".join(qc.key_record(c[1]) for c in cases), np.uint8).copy()
    pn_off = np.array([c[3] for c in cases], np.int64)
    pn_max = np.array([c[4] for c in cases], np.int64)
    res = np.zeros(len(cases), quic.RESULT_DTYPE)
    quic.unprotect_batch(p(buf), p(off), p(lens), len(cases), p(keys), p(pn_off), p(res), pn_max=p(pn_max), stream=0)
    qc.check_unprotect(cases, buf, off, res)
    pkts = qc.crypto_packets(seed)
    buf, off, lens = qc.pack([x[1] for x in pkts])
    caps = np.full(len(pkts), 2048, np.uint32)
    caps[[i for i, x in enumerate(pkts) if x[0] == "zero_prefix"]] = 1000   # -51 path
    out_off = np.concatenate([[0], np.cumsum(caps[:-1], dtype=np.uint64)]).astype(np.uint64)
    out = np.zeros(int(caps.sum()) + 64, np.uint8)
    res = np.zeros(len(pkts), quic.RESULT_DTYPE)
    ws = np.zeros(quic.workspace_size(len(pkts)), np.uint8)
    quic.read_crypto_payload_batch(p(buf), p(off), p(lens), len(pkts), p(out), p(out_off), p(caps), p(res), p(ws),
                                   stream=0)
    qc.check_crypto(pkts, out, out_off, caps, res)
    assert not out[int(caps.sum()):].any()


if __name__ == "__main__":
    lib = _lib.load()
    which = sys.argv[1]
    args = [int(a) for a in sys.argv[2:]]
    if which == "bimodal":
        case_bimodal(args[0], bool(args[1]))
    elif which == "contig":
        case_contig(*args)
    elif which == "pcap":
        case_packed_cap(*args[:3], bool(args[3]), args[4], args[5])
    elif which == "slotted":
        case_slotted(args[0], args[1], bool(args[2]), args[3], args[4], args[5], args[6] if len(args) > 6 else 0)
    elif which == "uniform":
        case_uniform(args[0], args[1], bool(args[2]))
    elif which == "host":
        case_host(args[0], args[1], args[2], bool(args[3]), args[4] if len(args) > 4 else 0)
    elif which == "conn":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_conn_scenarios
        run_conn_scenarios(batch=args[0], n_batch=args[1])
    elif which == "coalesce":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_coalesce_scenarios
        run_coalesce_scenarios(writers=args[0], per_writer=args[1], readers=args[2], max_batch=args[3],
                               idle_timeout=30.0)   # emulated batches run slowly under a loaded CPU tier
    elif which == "lifecycle":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_lifecycle_scenarios
        run_lifecycle_scenarios(n=args[0], max_batch=args[1])
    elif which == "rxfail":   # run with HYEMU_FAIL_EVENTS_FROM=5 (tests/emu/hip_emu.h)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_rx_gpu_failure_scenario
        run_rx_gpu_failure_scenario()
    elif which == "txfail":   # run with HYEMU_FAIL_EVENTS_FROM=1 (tests/emu/hip_emu.h)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_tx_gpu_failure_scenario
        run_tx_gpu_failure_scenario()
    elif which == "closerace":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_close_race_scenarios
        run_close_race_scenarios(threads=args[0], per_writer=args[1])
    elif which == "deadline":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conn_cases import run_deadline_scenarios
        run_deadline_scenarios()
    elif which == "far":
        case_slotted_far(args[0], args[1], args[2], bool(args[3]))
    elif which == "ragged":
        case_ragged(args[0], args[1], args[2], bool(args[3]), ["packed", "slotted"][args[4]])
    elif which == "punch":
        case_punch(args[0], args[1], args[2])
    elif which == "quic":
        case_quic(args[0])
    elif which == "gecko":
        case_gecko(*args)
    print("ok", which, args)

