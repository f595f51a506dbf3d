"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle.

Bit-exact everywhere (byte work).  Small and medium cases compare every byte
with the C restatement and the golden fixtures; the BASELINE.json full sizes
compare SHA-256 digests committed in tests/golden/batch_digests.json plus a
device round trip (obfuscate -> deobfuscate == input).
"""
import hashlib

import numpy as np
import pytest

from oracle import salamander_ref as ref

pytestmark = pytest.mark.gpu

PSK = b"average_password"


@pytest.fixture(scope="module", params=["auto", "wave", "tile"])
def obfs(gpu, request):
    """One context per batch kernel choice: auto (the shipped per-layout choice:
    the tile kernel where it applies, salamander_tile.h, else the wave kernel),
    the wave-group kernel forced on every layout (salamander_wave.h), and tile
    (= auto, kept as the explicit name)."""
    import hysteria_amd
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    o.set_kernel(request.param)
    yield o
    o.close()


def _dev(a, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _u64(a, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(gpu)


def _u32(a, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(gpu)


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


# ------------------------------------------------------------------ per packet
def test_golden_vectors_per_packet(golden, gpu):
    import hysteria_amd
    ctxs = {}
    try:
        for v in golden[0]["vectors"]:
            psk = bytes.fromhex(v["psk"])
            if psk not in ctxs:
                ctxs[psk] = hysteria_amd.SalamanderObfuscator(psk, 0)
            o = ctxs[psk]
            salt = bytes.fromhex(v["salt"])
            payload = ref.stream_bytes(v["payload_seed"], v["payload_start"], v["payload_len"])
            assert o.key(salt).hex() == v["key"]
            out = bytearray(hysteria_amd.UDP_BUFFER_SIZE + 64)
            n = o.obfuscate(payload, out, salt=salt)
            assert n == len(payload) + 8
            wire = bytes(out[:n])
            assert hashlib.sha256(wire).hexdigest() == v["wire_sha256"]
            if "wire" in v:
                assert wire.hex() == v["wire"]
            back = bytearray(len(wire))
            m = o.deobfuscate(wire, back)
            if payload:
                assert m == len(payload) and bytes(back[:m]) == payload
            else:
                assert m == 0
    finally:
        for o in ctxs.values():
            o.close()


def test_edge_rules_per_packet(obfs):
    salt = b"\x01" * 8
    assert obfs.obfuscate(b"x" * 10, bytearray(17), salt=salt) == 0   # salamander.go:60-62
    out = bytearray(18)
    assert obfs.obfuscate(b"x" * 10, out, salt=salt) == 18
    assert bytes(out) == ref.obfuscate(PSK, b"x" * 10, salt)
    out = bytearray(8)
    assert obfs.obfuscate(b"", out, salt=salt) == 8 and bytes(out) == salt
    for n in (0, 1, 7, 8):                                           # :75-76
        assert obfs.deobfuscate(b"\x00" * n, bytearray(2048)) == 0
    assert obfs.deobfuscate(b"\x00" * 20, bytearray(11)) == 0         # :76-77
    assert obfs.deobfuscate(b"\x00" * 20, bytearray(12)) == 12


def test_set_kernel_accepts_the_header_values_only(gpu):
    """hyobfs_salamander_set_kernel: HYOBFS_KERNEL_AUTO..FLAT accepted, anything else
    HYOBFS_ERR_INVALID (include/hyobfs.h, ABI 4)."""
    import hysteria_amd
    from hysteria_amd import _lib
    with hysteria_amd.SalamanderObfuscator(PSK, 0) as o:
        lib = _lib.load()
        for k in range(4):
            assert lib.hyobfs_salamander_set_kernel(o._h, k) == 0
        for k in (-1, 4, 5, 99):
            assert lib.hyobfs_salamander_set_kernel(o._h, k) == _lib.HYOBFS_ERR_INVALID


def test_reference_roundtrip_1000x1200_auto_salts(obfs):
    """TestSalamanderObfuscator (salamander_test.go:32-45) on the GPU path."""
    rng = np.random.default_rng(3)
    o_out, d_out = bytearray(2048), bytearray(2048)
    obfs.seed(12345)
    for _ in range(1000):
        payload = rng.integers(0, 256, 1200, dtype=np.uint8).tobytes()
        n = obfs.obfuscate(payload, o_out)
        assert n == len(payload) + 8
        m = obfs.deobfuscate(bytes(o_out[:n]), d_out)
        assert m == len(payload) and bytes(d_out[:m]) == payload
        assert bytes(o_out[:n]) == ref.obfuscate(PSK, payload, bytes(o_out[:8]))


@pytest.mark.parametrize("psk_len", [4, 5, 16, 119, 120, 121, 124, 127, 128, 129, 200, 248, 249, 256, 300])
def test_keys_batch_vs_hashlib(gpu, psk_len):
    import hysteria_amd
    import torch
    psk = ref.stream_bytes(9, 0, psk_len)
    n = 20000
    salts = ref.splitmix64_array(17, 0, n)
    with hysteria_amd.SalamanderObfuscator(psk, 0) as o:
        keys = torch.empty(32 * n, dtype=torch.uint8, device=gpu)
        o.keys_batch(_u64(salts, gpu), keys, n)
        got = _host(keys).reshape(n, 32)
    for i in range(0, n, 7):
        assert got[i].tobytes() == ref.key(psk, int(salts[i]).to_bytes(8, "little")), i


# ------------------------------------------------------------------ batches
def _uniform_inputs(gpu, n, L, seed_payload=1, seed_salt=2):
    import torch
    import hysteria_amd
    inp = torch.empty(max(n * L, 16), dtype=torch.uint8, device=gpu)
    hysteria_amd.synth_stream(inp, n * L, seed_payload, 0)
    salts = torch.empty(n, dtype=torch.int64, device=gpu)
    hysteria_amd.synth_u64(salts, n, seed_salt, 0)
    return inp, salts


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 1000, 65536])
def test_uniform_1200_vs_oracle(obfs, gpu, coracle, n):
    import torch
    L = 1200
    inp, salts = _uniform_inputs(gpu, n, L)
    out = torch.empty(n * (L + 8), dtype=torch.uint8, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    total = torch.zeros(1, dtype=torch.int64, device=gpu)
    obfs.obfuscate_batch(inp, n, in_stride=L, len_uniform=L, salts=salts, out=out, out_stride=L + 8,
                         out_len=out_len, out_total=total)
    h_in = _host(inp)[: n * L]
    assert np.array_equal(h_in, coracle.fill_stream(1, 0, n * L))
    exp, _, _, _ = coracle.batch(True, PSK, n, h_in, in_stride=L, len_uniform=L,
                                 salts=coracle.salts(2, 0, n), out_cap=n * (L + 8))
    got = _host(out)
    assert np.array_equal(got, exp)
    assert (_host(out_len) == L + 8).all()
    assert int(_host(total)[0]) == n * (L + 8)
    # deobfuscate back, packed output
    back = torch.empty(n * L, dtype=torch.uint8, device=gpu)
    obfs.deobfuscate_batch(out, n, in_stride=L + 8, len_uniform=L + 8, out=back)
    assert np.array_equal(_host(back), h_in)


def test_uniform_digest_64k_golden(obfs, gpu, golden):
    import torch
    d = golden[1]["small_64k_x_1200"]
    n, L = d["n"], d["len"]
    inp, salts = _uniform_inputs(gpu, n, L)
    out = torch.empty(n * (L + 8), dtype=torch.uint8, device=gpu)
    obfs.obfuscate_batch(inp, n, in_stride=L, len_uniform=L, salts=salts, out=out)   # packed layout
    assert hashlib.sha256(_host(out).tobytes()).hexdigest() == d["obf_sha256"]


def test_config2_1M_x_1200_digest_and_roundtrip(obfs, gpu, golden):
    """BASELINE configs[1] at full size: digest + device round trip."""
    import torch
    d = golden[1]["config2_1M_x_1200"]
    n, L = d["n"], d["len"]
    inp, salts = _uniform_inputs(gpu, n, L)
    out = torch.empty(n * (L + 8), dtype=torch.uint8, device=gpu)
    obfs.obfuscate_batch(inp, n, in_stride=L, len_uniform=L, salts=salts, out=out, out_stride=L + 8)
    assert hashlib.sha256(_host(out).tobytes()).hexdigest() == d["obf_sha256"]
    back = torch.empty(n * L, dtype=torch.uint8, device=gpu)
    obfs.deobfuscate_batch(out, n, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)
    torch.cuda.synchronize()
    assert torch.equal(back, inp[: n * L])


def test_config4_shard7_8M_x_1200_digest_and_roundtrip(gpu, golden):
    """BASELINE configs[3] (64M x 1200 B over 8 GPUs): the shard rank 7 owns,
    datagrams [7*8M, 8*8M) of the global synthetic batch, generated at that offset
    and obfuscated through the product as one 8M batch; digest committed by
    gen_golden.py from the C oracle; device round trip."""
    import torch
    import hysteria_amd
    d = golden[1]["config4_shard7_8M_x_1200"]
    first, n, L = d["first"], d["n"], d["len"]
    inp = torch.empty(n * L, dtype=torch.uint8, device=gpu)
    hysteria_amd.synth_stream(inp, n * L, 1, first * L)
    salts = torch.empty(n, dtype=torch.int64, device=gpu)
    hysteria_amd.synth_u64(salts, n, 2, first)
    out = torch.empty(n * (L + 8), dtype=torch.uint8, device=gpu)
    with hysteria_amd.SalamanderObfuscator(PSK, 0) as o:
        o.obfuscate_batch(inp, n, in_stride=L, len_uniform=L, salts=salts, out=out, out_stride=L + 8)
        torch.cuda.synchronize()
        h = hashlib.sha256()
        step = 1 << 28
        for s in range(0, out.numel(), step):
            h.update(out[s:s + step].cpu().numpy().tobytes())
        assert h.hexdigest() == d["obf_sha256"]
        back = torch.empty(n * L, dtype=torch.uint8, device=gpu)
        o.deobfuscate_batch(out, n, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)
        torch.cuda.synchronize()
        assert torch.equal(back, inp)


@pytest.mark.parametrize("kernel", ["auto", "wave"])
def test_concurrent_batches_one_context(gpu, coracle, kernel):
    """hyobfs.h promises a context may be used from several threads: two host
    threads, each on its own stream, submit 50 batches through ONE context --
    packed ragged batches of changing sizes with no caller workspace (the
    context's pooled scratch, allocated and freed on each stream while the other
    thread's kernels run) alternating with uniform slotted 1200-byte batches
    (the tile kernel under AUTO).  Every output against the oracle."""
    import threading
    import torch
    import hysteria_amd
    nmax = 20_000
    lens, in_off, inp, salts, total_in = _bimodal(gpu, nmax)
    h_lens, h_off, h_inp = _host(lens).view(np.uint32), _host(in_off).view(np.uint64), _host(inp)
    h_salts = coracle.salts(2, 0, nmax)
    sizes = {0: [500, 3000, 20_000, 1000, 12_000], 1: [17_000, 700, 9000, 20_000, 2500]}
    want = {}
    for n in set(sizes[0] + sizes[1]):
        cap = int(h_lens[:n].astype(np.uint64).sum()) + 8 * n
        exp, _, _, _ = coracle.batch(True, PSK, n, h_inp, in_off=h_off[:n], in_len=h_lens[:n], salts=h_salts[:n],
                                     out_cap=cap)
        want[n] = exp
    L, nu = 1200, 4000   # the uniform slotted batch: the first nu * L bytes of the same input
    want_u, _, _, _ = coracle.batch(True, PSK, nu, h_inp, in_stride=L, len_uniform=L, salts=h_salts[:nu],
                                    out_cap=nu * (L + 8), out_stride=L + 8)
    results = {0: [], 1: []}
    errors = []
    with hysteria_amd.SalamanderObfuscator(PSK, 0) as o:
        o.set_kernel(kernel)

        def worker(t):
            try:
                s = torch.cuda.Stream(device=gpu)
                with torch.cuda.stream(s):
                    for i in range(50):
                        if i % 2:
                            out = torch.empty(nu * (L + 8), dtype=torch.uint8, device=gpu)
                            o.obfuscate_batch(inp, nu, in_stride=L, len_uniform=L, salts=salts, out=out,
                                              out_stride=L + 8, stream=s)
                            results[t].append((-1, out))
                            continue
                        n = sizes[t][(i // 2) % 5]
                        cap = want[n].size
                        out = torch.empty(cap, dtype=torch.uint8, device=gpu)
                        o.obfuscate_batch(inp, n, in_off=in_off, in_len=lens, salts=salts, out=out, out_cap=cap,
                                          stream=s)
                        results[t].append((n, out))
                s.synchronize()
            except Exception as e:   # reported from the main thread
                errors.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in (0, 1)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize()
    assert not errors, errors
    for t in (0, 1):
        assert len(results[t]) == 50
        for i, (n, out) in enumerate(results[t]):
            assert np.array_equal(_host(out), want_u if n < 0 else want[n]), (t, i, n)


def test_pooled_scratch_bounded_over_many_streams(gpu):
    """The context's packed-batch scratch (no caller workspace) comes from a pool,
    allocated and freed in stream order: cycling 100 short-lived streams through
    one context must not grow device memory (round 2 kept one buffer per stream
    until the context died)."""
    import torch
    import hysteria_amd
    n = 200_000
    lens, in_off, inp, salts, total_in = _bimodal(gpu, n)
    cap = total_in + 8 * n
    out = torch.empty(cap, dtype=torch.uint8, device=gpu)
    with hysteria_amd.SalamanderObfuscator(PSK, 0) as o:
        def one(s):
            o.obfuscate_batch(inp, n, in_off=in_off, in_len=lens, salts=salts, out=out, out_cap=cap, stream=s)
            s.synchronize()
        for _ in range(3):   # warm the pool
            one(torch.cuda.Stream(device=gpu))
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(gpu)[0]
        for _ in range(100):
            one(torch.cuda.Stream(device=gpu))
        torch.cuda.synchronize()
        free1 = torch.cuda.mem_get_info(gpu)[0]
        # one batch's scratch is 8 B per 256 datagrams; 100 kept buffers would be
        # 100 x that plus allocation granularity: allow 64 MiB of noise
        assert free0 - free1 < (64 << 20), (free0, free1)
        ref_out = out.clone()
        one(torch.cuda.Stream(device=gpu))
        assert torch.equal(out, ref_out)


def _bimodal(gpu, n):
    import torch
    import hysteria_amd
    lens = torch.empty(n, dtype=torch.int32, device=gpu)
    hysteria_amd.synth_bimodal_lengths(lens, n, 3, 0)
    in_off = torch.zeros(n, dtype=torch.int64, device=gpu)
    in_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
    total_in = int(lens.to(torch.int64).sum())
    inp = torch.empty(total_in + 16, dtype=torch.uint8, device=gpu)
    hysteria_amd.synth_stream(inp, total_in, 1, 0)
    salts = torch.empty(n, dtype=torch.int64, device=gpu)
    hysteria_amd.synth_u64(salts, n, 2, 0)
    return lens, in_off, inp, salts, total_in


def test_bimodal_64k_vs_oracle_and_digest(obfs, gpu, coracle, golden):
    import torch
    d = golden[1]["bimodal_64k"]
    n = d["n"]
    lens, in_off, inp, salts, total_in = _bimodal(gpu, n)
    assert total_in == d["in_bytes"]
    cap = total_in + 8 * n
    out = torch.empty(cap, dtype=torch.uint8, device=gpu)
    out_off = torch.empty(n, dtype=torch.int64, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    obfs.obfuscate_batch(inp, n, in_off=in_off, in_len=lens, salts=salts, out=out, out_cap=cap,
                         out_off=out_off, out_len=out_len)
    got = _host(out)
    assert hashlib.sha256(got.tobytes()).hexdigest() == d["obf_sha256"]
    h_lens = _host(lens).view(np.uint32)
    exp, eoff, elen, _ = coracle.batch(True, PSK, n, _host(inp), in_off=_host(in_off).view(np.uint64),
                                       in_len=h_lens, salts=coracle.salts(2, 0, n), out_cap=cap)
    assert np.array_equal(got, exp)
    assert np.array_equal(_host(out_off).view(np.uint64), eoff)
    assert np.array_equal(_host(out_len).view(np.uint32), elen)
    # deobfuscate the packed wire back
    back = torch.empty(total_in + 16, dtype=torch.uint8, device=gpu)
    wlen = out_len
    obfs.deobfuscate_batch(out, n, in_off=out_off, in_len=wlen, out=back, out_cap=total_in)
    assert np.array_equal(_host(back)[:total_in], _host(inp)[:total_in])


def test_config3_bimodal_4M_digest(obfs, gpu, golden):
    import torch
    d = golden[1]["config3_bimodal_4M"]
    n = d["n"]
    lens, in_off, inp, salts, total_in = _bimodal(gpu, n)
    assert total_in == d["in_bytes"]
    cap = total_in + 8 * n
    out = torch.empty(cap, dtype=torch.uint8, device=gpu)
    obfs.obfuscate_batch(inp, n, in_off=in_off, in_len=lens, salts=salts, out=out, out_cap=cap)
    h = hashlib.sha256()
    torch.cuda.synchronize()
    step = 1 << 28
    for s in range(0, cap, step):
        h.update(out[s:s + step].cpu().numpy().tobytes())
    assert h.hexdigest() == d["obf_sha256"]


# ------------------------------------------- contiguous input: the flat kernel, the wave kernel's length scan
@pytest.fixture(params=["auto", "wave", "flat"])
def contig_obfs(gpu, request):
    """auto and wave: the wave kernel scanning the input lengths with the widths
    (packed) or the prepass's input offsets (slotted); flat: the flat kernel into
    packed output from 16-byte aligned input (salamander_flat.h), else the wave kernel."""
    import hysteria_amd
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    o.set_kernel(request.param)
    yield o
    o.close()


def _contig_kernel(o, packed=True, aligned=True):
    """The kernel a contiguous-input batch runs under the context's choice."""
    return "flat" if packed and aligned and o.kernel == "flat" else "wave"


def test_contiguous_bimodal_64k_vs_oracle_and_digest(contig_obfs, gpu, coracle, golden):
    """Contiguous packed input (in_off NULL, in_stride 0: datagram i right after
    datagram i-1, include/hyobfs.h) into packed output, under each kernel choice.
    The wire equals the explicit-offset batch's (the committed digest and the C
    oracle byte for byte); the wire, itself contiguous, deobfuscates back."""
    import torch
    obfs = contig_obfs
    d = golden[1]["bimodal_64k"]
    n = d["n"]
    lens, in_off, inp, salts, total_in = _bimodal(gpu, n)
    cap = total_in + 8 * n
    out = torch.full((cap + 64,), 0xA5, dtype=torch.uint8, device=gpu)
    out_off = torch.empty(n, dtype=torch.int64, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    total = torch.zeros(1, dtype=torch.int64, device=gpu)
    kw = dict(in_len=lens, out=out, out_cap=cap, out_off=out_off, out_len=out_len, out_total=total)
    assert obfs.batch_kernel(True, inp=inp, n=n, salts=salts, **kw) == _contig_kernel(obfs)
    obfs.obfuscate_batch(inp, n, salts=salts, **kw)
    got = _host(out)
    assert hashlib.sha256(got[:cap].tobytes()).hexdigest() == d["obf_sha256"]
    assert (got[cap:] == 0xA5).all()
    h_lens = _host(lens).view(np.uint32)
    exp, eoff, elen, etot = coracle.batch(True, PSK, n, _host(inp), in_off=_host(in_off).view(np.uint64),
                                          in_len=h_lens, salts=coracle.salts(2, 0, n), out_cap=cap)
    assert np.array_equal(got[:cap], exp)
    assert np.array_equal(_host(out_off).view(np.uint64), eoff)
    assert np.array_equal(_host(out_len).view(np.uint32), elen)
    assert int(_host(total)[0]) == etot
    back = torch.full((total_in + 64,), 0x5A, dtype=torch.uint8, device=gpu)
    kw = dict(in_len=out_len, out=back, out_cap=total_in, out_total=total)
    assert obfs.batch_kernel(False, inp=out, n=n, **kw) == _contig_kernel(obfs)
    obfs.deobfuscate_batch(out, n, **kw)
    hb = _host(back)
    assert np.array_equal(hb[:total_in], _host(inp)[:total_in])
    assert (hb[total_in:] == 0x5A).all() and int(_host(total)[0]) == total_in


def test_contiguous_config3_4M_digest_and_roundtrip(contig_obfs, gpu, golden):
    """BASELINE configs[2] at full size through the contiguous layout (what bench.py runs):
    the committed 4M digest, and the device round trip."""
    import torch
    obfs = contig_obfs
    d = golden[1]["config3_bimodal_4M"]
    n = d["n"]
    lens, in_off, inp, salts, total_in = _bimodal(gpu, n)
    del in_off
    cap = total_in + 8 * n
    out = torch.empty(cap, dtype=torch.uint8, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    obfs.obfuscate_batch(inp, n, in_len=lens, salts=salts, out=out, out_cap=cap, out_len=out_len)
    h = hashlib.sha256()
    torch.cuda.synchronize()
    step = 1 << 28
    for s in range(0, cap, step):
        h.update(out[s:s + step].cpu().numpy().tobytes())
    assert h.hexdigest() == d["obf_sha256"]
    back = torch.empty(total_in + 16, dtype=torch.uint8, device=gpu)
    obfs.deobfuscate_batch(out, n, in_len=out_len, out=back, out_cap=total_in)
    torch.cuda.synchronize()
    assert torch.equal(back[:total_in], inp[:total_in])


# seed, n, length distribution, obfuscate, out_cap %, PSK length, pkt_cap, input misalignment,
# out_stride (0: packed output)
# (dist 0 bimodal, 1: 0..2100 B, 2: 0..40 B (several per chunk), 3: 1..5 KB, 4: bimodal + zeros)
CONTIG_GPU = [(1, 20000, 0, 1, 100, 16, 0, 0, 0), (2, 20000, 0, 0, 100, 16, 0, 0, 0),
              (3, 8000, 1, 1, 100, 33, 0, 0, 0), (4, 8000, 1, 0, 100, 121, 0, 0, 0),
              (5, 20000, 2, 1, 100, 16, 0, 0, 0), (6, 20000, 2, 0, 100, 4, 0, 0, 0),
              (7, 2000, 3, 1, 100, 127, 0, 0, 0), (8, 2000, 3, 0, 100, 16, 0, 0, 0),
              (9, 20000, 4, 1, 100, 16, 0, 0, 0), (10, 20000, 4, 0, 100, 16, 0, 0, 0),
              (11, 8000, 1, 1, 60, 16, 0, 0, 0), (12, 8000, 1, 0, 70, 16, 0, 0, 0),
              (13, 8000, 1, 1, 100, 16, 1000, 0, 0), (14, 8000, 1, 0, 100, 16, 900, 0, 0),
              (15, 20000, 0, 1, 100, 16, 0, 1, 0), (16, 20000, 0, 0, 100, 16, 0, 3, 0),
              # slotted output: the prepass writes the input offsets into the workspace
              (21, 20000, 0, 1, 100, 16, 0, 0, 1358), (22, 20000, 0, 0, 100, 16, 0, 0, 1350),
              (23, 8000, 1, 1, 100, 16, 0, 0, 1200), (24, 8000, 1, 0, 100, 33, 0, 0, 1200),
              (25, 8000, 1, 1, 60, 16, 0, 0, 2112), (26, 8000, 1, 0, 70, 127, 0, 0, 2104),
              (27, 8000, 1, 1, 100, 16, 900, 0, 1208), (28, 8000, 1, 0, 100, 16, 700, 1, 2104),
              (29, 20000, 2, 1, 100, 121, 0, 0, 48), (30, 20000, 4, 0, 100, 16, 0, 0, 1350)]


@pytest.mark.parametrize("case", CONTIG_GPU)
def test_contiguous_input_grid_vs_oracle(contig_obfs, gpu, coracle, case):
    """The contiguous layout's edge cases under each kernel choice, byte for byte against
    the C oracle, sentinel bytes past the output: several datagrams per 16-byte chunk,
    zero-length datagrams, out_cap cuts (the tail), pkt_cap drops (holes in the input),
    real wire with 8-byte datagrams, PSKs across salt words and two blocks, misaligned
    input; packed output and slotted output (out_stride > 0: the prepass's input
    offsets).  The call gets a caller workspace of exactly hyobfs_batch_workspace_bytes
    (checked against the documented sizing) with sentinel bytes behind it."""
    import torch
    seed, n, dist, obf, cap_pct, psk_len, pkt_cap, mis, stride = case
    rng = np.random.default_rng(seed)
    psk = bytes((11 * i + 5) & 0xFF for i in range(psk_len))
    lens = {0: lambda: ref.bimodal_lengths(3, seed, n), 1: lambda: rng.integers(0, 2100, n),
            2: lambda: rng.integers(0, 41, n), 3: lambda: rng.integers(1000, 5000, n),
            4: lambda: np.where(rng.random(n) < 0.05, 0, ref.bimodal_lengths(3, seed, n))}[dist]()
    lens = np.ascontiguousarray(lens, np.uint32)
    in_off = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    inp = rng.integers(0, 256, total + 32, dtype=np.uint8)
    salts = ref.splitmix64_array(2, seed, n)
    if not obf:
        wire, woff, wlen, _ = coracle.batch(True, psk, n, inp, in_off=in_off, in_len=lens, salts=salts,
                                            out_cap=total + 8 * n)
        inp, in_off, lens, total = np.concatenate([wire, np.zeros(32, np.uint8)]), woff, wlen.copy(), int(wlen.sum())
    full = n * stride if stride else total + (8 * n if obf else 0)
    cap = max(16, full * cap_pct // 100)
    exp, eoff, elen, etot = coracle.batch(bool(obf), psk, n, inp, in_off=in_off, in_len=lens,
                                          salts=salts if obf else None, out_cap=cap, pkt_cap=pkt_cap,
                                          out_stride=stride)
    d_in = torch.zeros(len(inp) + 16, dtype=torch.uint8, device=gpu)
    d_in[mis:mis + len(inp)] = torch.from_numpy(inp).to(gpu)
    src = d_in[mis:]
    out = torch.full((cap + 64,), 0xA5, dtype=torch.uint8, device=gpu)
    out_off = torch.zeros(n, dtype=torch.int64, device=gpu)
    out_len = torch.zeros(n, dtype=torch.int32, device=gpu)
    tot = torch.zeros(1, dtype=torch.int64, device=gpu)
    kw = dict(in_len=_u32(lens, gpu), out=out, out_cap=cap, pkt_cap=pkt_cap, out_off=out_off, out_len=out_len,
              out_total=tot, out_stride=stride)
    if obf:
        kw["salts"] = _u64(salts, gpu)
    import hysteria_amd
    tsums = ((n + 255) // 256 + 1) * 8
    need = hysteria_amd.SalamanderObfuscator.workspace_bytes(inp=src, n=n, **kw)
    want = 2 * tsums + (8 * n if stride else 0)
    if not stride and not mis:   # the flat kernel's tile descriptors (16 KiB tiles)
        desc = 16 + 24 * ((cap + 16383) // 16384 + 1)   # + the hashers' key records, 64 B per datagram
        want = max(want, 2 * tsums + ((desc + 255) // 256) * 256 + 256 + 64 * n)
    assert need == want
    ws = torch.full((need + 64,), 0x3C, dtype=torch.uint8, device=gpu)
    with hysteria_amd.SalamanderObfuscator(psk, 0) as o:   # the case's PSK (the fixture's is average_password)
        o.set_kernel(contig_obfs.kernel)
        assert o.batch_kernel(bool(obf), inp=src, n=n, **kw) == _contig_kernel(o, not stride, not mis)
        (o.obfuscate_batch if obf else o.deobfuscate_batch)(inp=src, n=n, workspace=ws, workspace_bytes=need, **kw)
        got = _host(out)
    assert (_host(ws)[need:] == 0x3C).all(), "wrote past the workspace"
    assert np.array_equal(_host(out_off).view(np.uint64), eoff)
    assert np.array_equal(_host(out_len).view(np.uint32), elen)
    assert int(_host(tot)[0]) == etot
    written = np.zeros(cap + 64, bool)
    for o, w in zip(eoff, elen):
        written[int(o):int(o) + int(w)] = True
    assert np.array_equal(got[written], exp[written[:cap]])
    assert (got[~written] == 0xA5).all()


def _ragged_case(seed, n, maxlen, gap_max, base_misalign):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, n).astype(np.uint32)
    edge = [0, 1, 7, 8, 9, 15, 16, 17, 31, 32, 33, 2040, 2041, 2048, 2049]
    lens[: len(edge)] = edge[:n]
    gaps = rng.integers(0, gap_max + 1, n)
    in_off = np.zeros(n, np.uint64)
    in_off[0] = base_misalign
    in_off[1:] = base_misalign + np.cumsum((lens + gaps)[:-1], dtype=np.uint64)
    inp = rng.integers(0, 256, int(in_off[-1] + lens[-1] + 64), dtype=np.uint8)
    return lens, in_off, inp


@pytest.mark.parametrize("obf", [True, False])
@pytest.mark.parametrize("layout", ["packed", "slotted", "capped", "tiny"])
def test_ragged_layouts_vs_oracle(obfs, gpu, coracle, obf, layout):
    import torch
    n = 3000 if layout != "tiny" else 1500
    maxlen = 2100 if layout != "tiny" else 40
    lens, in_off, inp = _ragged_case(21 + (layout == "tiny"), n, maxlen, 5, 3)
    salts = ref.splitmix64_array(2, 0, n)
    out_stride, pkt_cap = 0, 0
    out_cap = int(lens.sum()) + 8 * n + 16
    if layout == "slotted":
        out_stride, out_cap = 2048, 2048 * n
    elif layout == "capped":
        pkt_cap, out_cap = 2048, out_cap // 2
    exp, eoff, elen, etot = coracle.batch(obf, PSK, n, inp, in_off=in_off, in_len=lens,
                                          salts=salts if obf else None, out_cap=out_cap,
                                          out_stride=out_stride, pkt_cap=pkt_cap)
    sentinel = 0xA5
    out = torch.full((out_cap + 32,), sentinel, dtype=torch.uint8, device=gpu)
    out_off = torch.empty(n, dtype=torch.int64, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    total = torch.zeros(1, dtype=torch.int64, device=gpu)
    kw = dict(in_off=_u64(in_off, gpu), in_len=_u32(lens, gpu), out=out, out_cap=out_cap,
              out_stride=out_stride, pkt_cap=pkt_cap, out_off=out_off, out_len=out_len, out_total=total)
    if obf:
        obfs.obfuscate_batch(_dev(inp, gpu), n, salts=_u64(salts, gpu), **kw)
    else:
        obfs.deobfuscate_batch(_dev(inp, gpu), n, **kw)
    got = _host(out)
    assert np.array_equal(_host(out_off).view(np.uint64), eoff)
    assert np.array_equal(_host(out_len).view(np.uint32), elen)
    assert int(_host(total)[0]) == etot
    # written regions equal the oracle; everything else keeps the sentinel
    written = np.zeros(out_cap + 32, bool)
    for o, w in zip(eoff, elen):
        written[int(o): int(o) + int(w)] = True
    assert np.array_equal(got[:out_cap][written[:out_cap]], exp[written[:out_cap]])
    assert (got[~written] == sentinel).all()


# ------------------------------------------------------- the tile kernel's grid
from tile_cases import TILE_CASES, expects_tile, slotted_params  # noqa: E402


@pytest.mark.parametrize("kernel", ["auto", "wave"])
@pytest.mark.parametrize("which,args", TILE_CASES)
def test_tile_layout_grid(gpu, coracle, which, args, kernel):
    """The tile kernel's layout grid on the GPU (tests/tile_cases.py, the same cases the
    CPU tier emulates): gapped and 0-mod-16 slots, 4096-byte input strides (64 KiB of
    staged LDS), the 8-byte input tail, multi-pass compose (9000-byte slots), every salt
    word 0..15 including the two-block PSKs, and layouts that fall back to the wave
    kernel.  Byte for byte against the C oracle, sentinel bytes in every gap, the kernel
    AUTO chose checked (hyobfs_salamander_batch_kernel); "wave" runs the same case on
    the wave kernel."""
    import torch
    import hysteria_amd
    n, L, obf, slot_pad, in_pad, psk = slotted_params(which, args)
    W = L + 8 if obf else L - 8
    S, istride = W + slot_pad, L + in_pad
    inp = np.frombuffer(ref.stream_bytes(1, 0, n * istride + 16), np.uint8).copy()
    salts = ref.splitmix64_array(2, 0, n)
    cap = n * S
    exp, eoff, elen, etot = coracle.batch(obf, psk, n, inp, in_stride=istride, len_uniform=L,
                                          salts=salts if obf else None, out_cap=cap, out_stride=S)
    sentinel = 0xA5
    out = torch.full((cap + 64,), sentinel, dtype=torch.uint8, device=gpu)
    out_off = torch.zeros(n, dtype=torch.int64, device=gpu)
    out_len = torch.zeros(n, dtype=torch.int32, device=gpu)
    total = torch.zeros(1, dtype=torch.int64, device=gpu)
    with hysteria_amd.SalamanderObfuscator(psk, 0) as o:
        o.set_kernel(kernel)
        d_in = _dev(inp, gpu)
        kw = dict(inp=d_in, n=n, in_stride=istride, len_uniform=L, out=out, out_cap=cap, out_stride=S,
                  out_off=out_off, out_len=out_len, out_total=total)
        if obf:
            kw["salts"] = _u64(salts, gpu)
        want = "tile" if kernel == "auto" and expects_tile(n, L, obf, slot_pad, in_pad) else "wave"
        assert o.batch_kernel(obf, **kw) == want, (which, args)
        (o.obfuscate_batch if obf else o.deobfuscate_batch)(**kw)
        got = _host(out)
    assert np.array_equal(_host(out_off).view(np.uint64), eoff)
    assert np.array_equal(_host(out_len).view(np.uint32), elen)
    assert int(_host(total)[0]) == etot
    written = np.zeros(cap + 64, bool)
    for off, w in zip(eoff, elen):
        written[int(off):int(off) + int(w)] = True
    assert np.array_equal(got[written], exp[:cap][written[:cap]])
    assert (got[~written] == sentinel).all(), "bytes outside the regions were written"


def test_empty_batch(obfs, gpu):
    import torch
    out = torch.zeros(16, dtype=torch.uint8, device=gpu)
    total = torch.full((1,), 7, dtype=torch.int64, device=gpu)
    salts = torch.zeros(1, dtype=torch.int64, device=gpu)
    obfs.obfuscate_batch(out, 0, salts=salts, out=out, out_total=total)
    assert int(_host(total)[0]) == 0


def test_misaligned_out_rejected(obfs, gpu):
    import torch
    from hysteria_amd._lib import HyobfsError
    buf = torch.zeros(4096, dtype=torch.uint8, device=gpu)
    salts = torch.zeros(1, dtype=torch.int64, device=gpu)
    with pytest.raises(HyobfsError):
        obfs.obfuscate_batch(buf, 1, len_uniform=10, salts=salts, out=buf.data_ptr() + 1, out_cap=100)


# PSK lengths that put salt[0] in every message word 0..15 (aligned and not),
# the two-block tail (121..127 mod 128) and multi-block PSKs
PSK_SWEEP = [4, 5, 8, 13, 16, 23, 24, 31, 36, 40, 47, 52, 56, 63, 64, 71, 72, 79, 80, 88, 95,
             96, 100, 104, 111, 112, 119, 120, 121, 124, 127, 128, 129, 200, 248, 249, 255, 256, 300]


@pytest.mark.parametrize("psk_len", PSK_SWEEP)
@pytest.mark.parametrize("obf", [True, False])
def test_every_salt_word_instantiation(gpu, coracle, psk_len, obf):
    import torch
    import hysteria_amd
    psk = ref.stream_bytes(11, 0, psk_len)
    n = 700
    lens, in_off, inp = _ragged_case(100 + psk_len, n, 1500, 3, 1)
    salts = ref.splitmix64_array(5, 0, n)
    out_cap = int(lens.sum()) + 8 * n + 16
    exp, eoff, elen, _ = coracle.batch(obf, psk, n, inp, in_off=in_off, in_len=lens,
                                       salts=salts if obf else None, out_cap=out_cap)
    out = torch.zeros(out_cap, dtype=torch.uint8, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    with hysteria_amd.SalamanderObfuscator(psk, 0) as o:
        kw = dict(in_off=_u64(in_off, gpu), in_len=_u32(lens, gpu), out=out, out_cap=out_cap, out_len=out_len)
        if obf:
            o.obfuscate_batch(_dev(inp, gpu), n, salts=_u64(salts, gpu), **kw)
        else:
            o.deobfuscate_batch(_dev(inp, gpu), n, **kw)
        got = _host(out)
    assert np.array_equal(_host(out_len).view(np.uint32), elen)
    assert np.array_equal(got, exp)


def test_packed_output_offsets_beyond_4GiB(obfs, gpu):
    """Packed output of 4.6 GB: offsets past 2^31 and 2^32 (64-bit offset arithmetic).
    Inputs alias one 1 MiB region (in_off is free-form), so only the output is large."""
    import torch
    n, L = 3_400_000, 1350
    region = 1 << 20
    src = torch.empty(region, dtype=torch.uint8, device=gpu)
    import hysteria_amd
    hysteria_amd.synth_stream(src, region, 1, 0)
    idx = torch.arange(n, dtype=torch.int64, device=gpu)
    in_off = (idx * 977) % (region - L)
    lens = torch.full((n,), L, dtype=torch.int32, device=gpu)
    salts = torch.empty(n, dtype=torch.int64, device=gpu)
    hysteria_amd.synth_u64(salts, n, 2, 0)
    cap = n * (L + 8)
    assert cap > (1 << 32)
    out = torch.empty(cap, dtype=torch.uint8, device=gpu)
    out_off = torch.empty(n, dtype=torch.int64, device=gpu)
    out_len = torch.empty(n, dtype=torch.int32, device=gpu)
    obfs.obfuscate_batch(src, n, in_off=in_off, in_len=lens, salts=salts, out=out, out_cap=cap,
                         out_off=out_off, out_len=out_len)
    torch.cuda.synchronize()
    assert torch.equal(out_off, idx * (L + 8))
    assert bool((out_len == L + 8).all())
    h_src = src.cpu().numpy().tobytes()
    h_salts = salts.cpu().numpy().view(np.uint64)
    picks = set(range(0, n, 9973)) | {n - 1}
    for edge in ((1 << 31), (1 << 32)):
        p = edge // (L + 8)
        picks |= {p - 1, p, p + 1}
    for p in sorted(picks):
        o = int(p) * (L + 8)
        got = out[o:o + L + 8].cpu().numpy().tobytes()
        io = (int(p) * 977) % (region - L)
        exp = ref.obfuscate(PSK, h_src[io:io + L], int(h_salts[p]).to_bytes(8, "little"))
        assert got == exp, p


def test_packed_offsets_past_one_scan_pass(obfs, gpu):
    """More than 16384 tiles (4M datagrams): the tile-sum scan takes two passes and
    carries between them.  Packed output of 4.5M 16-byte datagrams with in_len given
    (a ragged-batch launch): every offset and a sample of wire datagrams."""
    import torch
    import hysteria_amd
    n, L = 4_500_000, 16
    inp = torch.empty(n * L, dtype=torch.uint8, device=gpu)
    hysteria_amd.synth_stream(inp, n * L, 1, 0)
    lens = torch.full((n,), L, dtype=torch.int32, device=gpu)
    in_off = torch.arange(n, dtype=torch.int64, device=gpu) * L
    salts = torch.empty(n, dtype=torch.int64, device=gpu)
    hysteria_amd.synth_u64(salts, n, 2, 0)
    out = torch.empty(n * (L + 8), dtype=torch.uint8, device=gpu)
    out_off = torch.empty(n, dtype=torch.int64, device=gpu)
    obfs.obfuscate_batch(inp, n, in_off=in_off, in_len=lens, salts=salts, out=out, out_off=out_off)
    torch.cuda.synchronize()
    assert torch.equal(out_off, torch.arange(n, dtype=torch.int64, device=gpu) * (L + 8))
    h_in = inp.cpu().numpy()
    h_salts = salts.cpu().numpy().view(np.uint64)
    for p in list(range(0, n, 99_991)) + [4_194_303, 4_194_304, n - 1]:
        got = out[p * (L + 8):(p + 1) * (L + 8)].cpu().numpy().tobytes()
        assert got == ref.obfuscate(PSK, h_in[p * L:(p + 1) * L].tobytes(), int(h_salts[p]).to_bytes(8, "little")), p


class _Mapped:
    """numpy views of mapped pinned host buffers (hyobfs_host_alloc), freed on close."""

    def __init__(self):
        from hysteria_amd import _lib
        self.lib, self.ptrs = _lib.load(), []

    def array(self, n, dtype):
        import ctypes
        nb = n * np.dtype(dtype).itemsize
        p = self.lib.hyobfs_host_alloc(nb)
        assert p, "hyobfs_host_alloc"
        self.ptrs.append(p)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), (nb,)).view(dtype)

    def close(self):
        for p in self.ptrs:
            self.lib.hyobfs_host_free(p)


@pytest.mark.parametrize("obf", [True, False])
@pytest.mark.parametrize("mem", ["pinned", "pageable", "mapped"])
def test_host_batch_pipeline_vs_oracle(obfs, gpu, obf, mem):
    """Host-resident slotted batch (recvmmsg/sendmmsg ring shape): pageable and torch-pinned
    buffers (with pageable lengths / salts / out_len) through the H2D / kernel / D2H
    pipeline, chunked so several chunks cycle the 3 slots; every array in mapped pinned
    memory (hyobfs_host_alloc) through the zero-copy path: one batch call in place."""
    import torch
    n, L = 5000, 1350
    rng = np.random.default_rng(7 + obf)
    stride_in = 2048
    lens = rng.integers(0, L + 1, n).astype(np.uint32)
    lens[:4] = [0, 8, 9, L]
    inp = rng.integers(0, 256, n * stride_in, dtype=np.uint8)
    salts = ref.splitmix64_array(2, 0, n)
    out_stride = 2048
    out_len = np.zeros(n, np.uint32)
    h_lens, h_salts = lens.copy(), salts.copy()   # the host copies the check reads
    mapped = _Mapped()
    try:
        if mem == "pinned":
            in_buf = torch.from_numpy(inp).pin_memory()
            out_buf = torch.full((n * out_stride,), 0xA5, dtype=torch.uint8).pin_memory()
        elif mem == "mapped":
            in_buf, out_buf = mapped.array(n * stride_in, np.uint8), mapped.array(n * out_stride, np.uint8)
            in_buf[:] = inp
            out_buf[:] = 0xA5
            lens, salts, out_len = mapped.array(n, np.uint32), mapped.array(n, np.uint64), mapped.array(n, np.uint32)
            lens[:], salts[:], out_len[:] = h_lens, h_salts, 0
        else:
            in_buf, out_buf = inp, np.full(n * out_stride, 0xA5, np.uint8)
        kw = dict(in_stride=stride_in, in_len=lens, out=out_buf, out_stride=out_stride, out_len=out_len, chunk=777)
        if obf:
            obfs.obfuscate_host(in_buf, n, salts=salts, **kw)
        else:
            obfs.deobfuscate_host(in_buf, n, **kw)
        got = np.array(out_buf.numpy() if mem == "pinned" else out_buf)
        olen = np.array(out_len)
    finally:
        mapped.close()
    for i in range(n):
        src = inp[i * stride_in:i * stride_in + int(h_lens[i])].tobytes()
        exp = ref.obfuscate(PSK, src, int(h_salts[i]).to_bytes(8, "little"), out_stride) if obf \
            else ref.deobfuscate(PSK, src, out_stride)
        assert int(olen[i]) == len(exp), i
        assert got[i * out_stride:i * out_stride + len(exp)].tobytes() == exp, i
    if mem != "mapped":
        return   # the staged pipeline copies whole output slots back (include/hyobfs.h)
    untouched = np.ones(n * out_stride, bool)   # zero-copy writes only the regions
    for i in range(n):
        untouched[i * out_stride:i * out_stride + int(olen[i])] = False
    assert (got[untouched] == 0xA5).all()


@pytest.mark.gpu
def test_packet_conn_loopback(gpu):
    """obfsPacketConn (conn.go:73-99) over loopback UDP: ReadFrom/WriteTo quirks,
    batched recvmmsg/sendmmsg paths, wire bytes against the oracle."""
    from conn_cases import run_conn_scenarios
    run_conn_scenarios(device=0, batch=1024, n_batch=400)


@pytest.mark.gpu
def test_packet_conn_lifecycle(gpu):
    """close() without flush sends what write_to accepted; close() wakes blocked
    readers with EBADF; a failed queued send is reported by the next write_to."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from conn_cases import run_lifecycle_scenarios
    run_lifecycle_scenarios(device=0)


def test_packet_conn_deadlines(gpu):
    """Set{Read,Write}Deadline (conn.go:109-119) in plain and coalescing mode."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from conn_cases import run_deadline_scenarios
    run_deadline_scenarios(device=0)


def test_packet_conn_close_race(gpu):
    """Close racing 8 threads in read_from / write_to, plain and coalescing mode: every
    thread leaves with EBADF, every later call fails with EBADF, every accepted
    datagram reaches the wire (include/hyobfs_conn.h, hyobfs_conn_close)."""
    from conn_cases import run_close_race_scenarios
    run_close_race_scenarios(device=0, threads=8, per_writer=1500)


def test_packet_conn_coalescing_loopback(gpu):
    """Coalescing mode: 8 writer and 4 reader threads on the per-datagram calls of one
    connection each side, GPU batches behind them; wire bytes against the oracle."""
    from conn_cases import run_coalesce_scenarios
    run_coalesce_scenarios(device=0, writers=8, per_writer=1000, readers=4, max_batch=256, max_wait_us=100)


# ------------------------------------------------------------- sharded batches
@pytest.mark.parametrize("nshards", [1, 2, 3])
def test_sharded_batch_matches_single_batch(gpu, coracle, nshards):
    """hyobfs_salamander_*_batch_sharded: shards planned by hyobfs_shard_bounds (equal
    traffic), one context each (all on device 0 here), packed outputs per shard.  The
    shards' outputs back to back are the single batch's packed output."""
    import torch
    import hysteria_amd
    from hysteria_amd.shard import shard_bounds
    n = 20_000
    lens, in_off, inp, salts, total_in = _bimodal(gpu, n)
    h_lens = _host(lens).view(np.uint32)
    bounds = shard_bounds(h_lens, n, nshards)
    exp, eoff, elen, _ = coracle.batch(True, PSK, n, _host(inp), in_off=_host(in_off).view(np.uint64),
                                       in_len=h_lens, salts=coracle.salts(2, 0, n), out_cap=total_in + 8 * n)
    ctxs = [hysteria_amd.SalamanderObfuscator(PSK, 0) for _ in range(nshards)]
    try:
        shards, outs, back_shards, backs = [], [], [], []
        for i in range(nshards):
            a, b = bounds[i], bounds[i + 1]
            cap = int(h_lens[a:b].astype(np.uint64).sum()) + 8 * (b - a)
            out = torch.empty(max(cap, 16), dtype=torch.uint8, device=gpu)
            olen = torch.empty(max(b - a, 1), dtype=torch.int32, device=gpu)
            ooff = torch.empty(max(b - a, 1), dtype=torch.int64, device=gpu)
            ws = torch.empty(hysteria_amd.workspace_size(b - a), dtype=torch.uint8, device=gpu)
            outs.append((out, ooff, olen, cap, a, b))
            shards.append(dict(inp=inp, n=b - a, in_off=in_off[a:], in_len=lens[a:], salts=salts[a:], out=out,
                               out_cap=cap, out_off=ooff, out_len=olen, workspace=ws, workspace_bytes=ws.numel()))
        hysteria_amd.obfuscate_batch_sharded(ctxs, shards)
        got = np.concatenate([_host(o)[:cap] for o, _, _, cap, _, _ in outs])
        assert np.array_equal(got, exp[:total_in + 8 * n])
        base = 0
        for o, ooff, olen, cap, a, b in outs:
            if b > a:
                assert np.array_equal(_host(ooff)[:b - a].view(np.uint64) + np.uint64(base), eoff[a:b])
                assert np.array_equal(_host(olen)[:b - a].view(np.uint32), elen[a:b])
            base += cap
        # and back, sharded the same way
        for o, ooff, olen, cap, a, b in outs:
            plen = cap - 8 * (b - a)
            back = torch.empty(max(plen, 16), dtype=torch.uint8, device=gpu)
            backs.append((back, plen))
            back_shards.append(dict(inp=o, n=b - a, in_off=ooff, in_len=olen, out=back, out_cap=plen))
        hysteria_amd.deobfuscate_batch_sharded(ctxs, back_shards)
        plain = np.concatenate([_host(bk)[:plen] for bk, plen in backs])
        assert np.array_equal(plain, _host(inp)[:total_in])
    finally:
        for c in ctxs:
            c.close()


def test_sharded_batch_argument_errors(gpu):
    import ctypes
    import hysteria_amd
    from hysteria_amd import _lib
    lib = _lib.load()
    o = hysteria_amd.SalamanderObfuscator(PSK, 0)
    try:
        arr = (_lib.HyobfsBatch * 2)()
        dup = (ctypes.c_void_p * 2)(o._h, o._h)
        assert lib.hyobfs_salamander_obfuscate_batch_sharded(dup, arr, 2) == _lib.HYOBFS_ERR_INVALID
        assert lib.hyobfs_salamander_obfuscate_batch_sharded(None, None, 0) == _lib.HYOBFS_OK
        assert lib.hyobfs_salamander_deobfuscate_batch_sharded(None, arr, 1) == _lib.HYOBFS_ERR_INVALID
    finally:
        o.close()
