#!/usr/bin/env python3
"""Generate tests/golden/*.json -- known-answer fixtures for Salamander.

The reference publishes no Salamander known-answer vector
(extras/obfs/salamander_test.go:32-45 checks round-trip identity only) and its
toolchain (Go + golang.org/x/crypto@v0.54.0) is absent, so the fixtures are
produced by the Python restatement (oracle/salamander_ref.py: hashlib BLAKE2b)
and every derived key is cross-checked against coreutils `b2sum -l 256`, an
independent BLAKE2b.  RFC 7693 Appendix A's BLAKE2b-512("abc") pins the hash.

Usage:  python tests/golden/gen_golden.py          (rewrites the fixtures)
Large-batch digests need the C oracle:  make -C oracle  first.
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import salamander_ref as ref  # noqa: E402

PSK_LENS = [4, 16, 119, 120, 121, 128, 200, 256]
PAYLOAD_LENS = [0, 1, 7, 8, 15, 16, 31, 32, 33, 63, 64, 65, 1199, 1200, 1201, 1350, 2040]
FULL_HEX_MAX = 72   # wire bytes stored verbatim up to this length, SHA-256 beyond


def psk_for(n):
    if n == 16:
        return b"average_password"   # salamander_test.go:11
    return ref.stream_bytes(7, 0, n)


def b2sum256(data: bytes) -> str:
    r = subprocess.run(["b2sum", "-l", "256"], input=data, capture_output=True, check=True)
    return r.stdout.split()[0].decode()


def main():
    # --- hash KATs
    kat = {
        "rfc7693_appendix_a_blake2b512_abc":
            "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
            "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923",
        "blake2b256_abc": hashlib.blake2b(b"abc", digest_size=32).hexdigest(),
        "blake2b256_empty": hashlib.blake2b(b"", digest_size=32).hexdigest(),
    }
    assert hashlib.blake2b(b"abc").hexdigest() == kat["rfc7693_appendix_a_blake2b512_abc"]
    assert b2sum256(b"abc") == kat["blake2b256_abc"]
    assert b2sum256(b"") == kat["blake2b256_empty"]

    # --- Salamander vectors
    vecs = []
    k = 0
    for pl in PSK_LENS:
        psk = psk_for(pl)
        for L in PAYLOAD_LENS:
            salt = ref.splitmix64_at(2, k).to_bytes(8, "little")
            payload = ref.stream_bytes(1, 4096 * k, L)
            key = ref.key(psk, salt)
            assert b2sum256(psk + salt) == key.hex(), (pl, L)
            wire = ref.obfuscate(psk, payload, salt)
            assert ref.deobfuscate(psk, wire) == payload
            v = {"psk_len": pl, "psk": psk.hex(), "salt": salt.hex(), "payload_len": L,
                 "payload_seed": 1, "payload_start": 4096 * k, "key": key.hex(),
                 "wire_len": len(wire), "wire_sha256": hashlib.sha256(wire).hexdigest()}
            if len(wire) <= FULL_HEX_MAX:
                v["payload"] = payload.hex()
                v["wire"] = wire.hex()
            vecs.append(v)
            k += 1

    # SURVEY §8c spot values (hashlib and b2sum agreed on them in the survey)
    spot_psk = b"average_password"
    spot_salt = bytes(range(8))
    spot = {
        "psk": spot_psk.hex(), "salt": spot_salt.hex(),
        "key": ref.key(spot_psk, spot_salt).hex(),
        "payload": bytes(range(40)).hex(),
        "wire": ref.obfuscate(spot_psk, bytes(range(40)), spot_salt).hex(),
        "two_block_psk": (b"a" * 121).hex(),
        "two_block_key": ref.key(b"a" * 121, spot_salt).hex(),
    }
    assert spot["key"] == "7145ab9cb8618c6057681425a251337ddff92fdc6320f58920527b95fff4df33"
    assert spot["two_block_key"] == "a1dceffd71c342b0e7f50a17b225dfb92a5b6921cba9ca550bed1f052e6893f7"

    with open(os.path.join(HERE, "salamander_vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_golden.py", "hash_kat": kat,
                   "survey_spot": spot, "vectors": vecs}, f, indent=1)
        f.write("\n")

    # --- batch digests (configs of BASELINE.json); need the C oracle
    import numpy as np
    co = ref.COracle()
    psk = b"average_password"
    out = {}

    def uniform_digest(n, L):
        inp = co.fill_stream(1, 0, n * L)
        salts = co.salts(2, 0, n)
        wire, _, wl, tot = co.batch(True, psk, n, inp, in_stride=L, len_uniform=L, salts=salts,
                                    out_cap=n * (L + 8))
        assert tot == n * (L + 8)
        d = {"n": n, "len": L, "obf_sha256": hashlib.sha256(wire.tobytes()).hexdigest()}
        # deobfuscate the wire back (identity)
        back, _, _, tot2 = co.batch(False, psk, n, wire, in_stride=L + 8, len_uniform=L + 8, out_cap=n * L)
        assert tot2 == n * L and np.array_equal(back, inp)
        return d

    def bimodal_digest(n):
        lens = co.bimodal_lengths(3, 0, n)
        in_off = np.zeros(n, np.uint64)
        in_off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        total_in = int(lens.sum(dtype=np.uint64))
        inp = co.fill_stream(1, 0, total_in)
        salts = co.salts(2, 0, n)
        cap = total_in + 8 * n
        wire, woff, wl, tot = co.batch(True, psk, n, inp, in_off=in_off, in_len=lens, salts=salts, out_cap=cap)
        assert tot == cap
        return {"n": n, "lens": "bimodal(seed=3)", "in_bytes": total_in,
                "obf_sha256": hashlib.sha256(wire.tobytes()).hexdigest()}

    def shard_digest(first, n, L, chunk=1 << 18):
        """One rank's shard of the configs[3] batch (64M x 1200 B over 8 GPUs): datagrams
        [first, first + n) of the global synthetic batch, obfuscated into dense slots,
        digested chunk by chunk (the whole shard is ~10 GB)."""
        h = hashlib.sha256()
        threads = os.cpu_count() or 1
        for q in range(first, first + n, chunk):
            m = min(chunk, first + n - q)
            inp = co.fill_stream(1, q * L, m * L)
            salts = co.salts(2, q, m)
            wire = np.empty(m * (L + 8), np.uint8)
            co.run_uniform(True, psk, m, inp, L, L, salts, wire, L + 8, threads)
            h.update(wire.tobytes())
        return {"first": first, "n": n, "len": L, "obf_sha256": h.hexdigest()}

    out["config1_cpu_10k_x_1200"] = uniform_digest(10_000, 1200)
    out["small_64k_x_1200"] = uniform_digest(65_536, 1200)
    out["bimodal_64k"] = bimodal_digest(65_536)
    large = ("config2_1M_x_1200", "config3_bimodal_4M", "config4_shard7_8M_x_1200")
    if "--large" in sys.argv:
        out["config2_1M_x_1200"] = uniform_digest(1 << 20, 1200)
        out["config3_bimodal_4M"] = bimodal_digest(1 << 22)
        out["config4_shard7_8M_x_1200"] = shard_digest(7 << 23, 1 << 23, 1200)
    else:
        old = os.path.join(HERE, "batch_digests.json")
        if os.path.exists(old):
            prev = json.load(open(old))
            for k in large:
                if k in prev:
                    out[k] = prev[k]
        if "--shard" in sys.argv:
            out["config4_shard7_8M_x_1200"] = shard_digest(7 << 23, 1 << 23, 1200)
    out["definition"] = ("payload = SplitMix64(seed=1) LE byte stream packed; salts = SplitMix64(seed=2) "
                         "outputs LE; bimodal len_i = 64 if SplitMix64(seed=3)_i % 5 < 2 else 1350; "
                         "PSK = average_password; digest = SHA-256 of the packed wire (obfuscate)")
    with open(os.path.join(HERE, "batch_digests.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print("ok", len(vecs), "vectors")


if __name__ == "__main__":
    main()
