"""Python restatement of Hysteria's Salamander obfuscation + loader for the C oracle.

TEST INFRASTRUCTURE ONLY.  Only tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / CPU baseline.  The product package ``hysteria_amd`` never imports it.

Restated from the reference (paths relative to apernet/hysteria):

* ``extras/obfs/salamander.go:13-17``  -- PSK >= 4 bytes, 8-byte salt, 32-byte key
* ``extras/obfs/salamander.go:34-37``  -- ``ErrPSKTooShort``
* ``extras/obfs/salamander.go:59-72``  -- ``Obfuscate``: ``out = salt || in ^ key[i % 32]``
* ``extras/obfs/salamander.go:74-86``  -- ``Deobfuscate``: ``len(in) <= 8`` -> 0
* ``extras/obfs/salamander.go:88-91``  -- ``keyLocked``: ``blake2b.Sum256(PSK || salt)``
* ``PROTOCOL.md:129-153``              -- normative packet format

The hash is CPython's ``hashlib.blake2b(digest_size=32)`` -- an implementation
independent of the C oracle (``salamander_ref.c``) and of the HIP kernels, and
cross-checked against coreutils ``b2sum -l 256`` by ``tests/golden/gen_golden.py``.
"""
from __future__ import annotations

import ctypes
import hashlib
import os

import numpy as np

SM_PSK_MIN_LEN = 4
SM_SALT_LEN = 8
SM_KEY_LEN = 32

_HERE = os.path.dirname(os.path.abspath(__file__))


class PSKTooShortError(ValueError):
    """``ErrPSKTooShort`` (salamander.go:21)."""


def check_psk(psk: bytes) -> None:
    """newSalamanderObfuscator's PSK check (salamander.go:35-37)."""
    if len(psk) < SM_PSK_MIN_LEN:
        raise PSKTooShortError(f"PSK must be at least {SM_PSK_MIN_LEN} bytes")


def key(psk: bytes, salt: bytes) -> bytes:
    """keyLocked (salamander.go:88-91): BLAKE2b-256(PSK || salt[:8])."""
    return hashlib.blake2b(bytes(psk) + bytes(salt[:SM_SALT_LEN]), digest_size=SM_KEY_LEN).digest()


def _xor_key(data: bytes, k: bytes) -> bytes:
    a = np.frombuffer(bytes(data), dtype=np.uint8)
    if a.size == 0:
        return b""
    reps = -(-a.size // SM_KEY_LEN)
    ks = np.frombuffer(k * reps, dtype=np.uint8)[: a.size]
    return (a ^ ks).tobytes()


def obfuscate(psk: bytes, payload: bytes, salt: bytes, out_len: int | None = None) -> bytes:
    """Obfuscate (salamander.go:59-72) with an explicit salt.

    Returns the wire bytes, or ``b""`` where the reference returns 0
    (``len(out) < len(in) + 8``).
    """
    n = len(payload) + SM_SALT_LEN
    if out_len is not None and out_len < n:
        return b""
    return bytes(salt[:SM_SALT_LEN]) + _xor_key(payload, key(psk, salt))


def deobfuscate(psk: bytes, wire: bytes, out_len: int | None = None) -> bytes:
    """Deobfuscate (salamander.go:74-86).  ``b""`` where the reference returns 0."""
    n = len(wire) - SM_SALT_LEN
    if n <= 0 or (out_len is not None and out_len < n):
        return b""
    return _xor_key(wire[SM_SALT_LEN:], key(psk, wire[:SM_SALT_LEN]))


# ------------------------------------------------------------------ seeded inputs
GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def splitmix64_at(seed: int, k: int) -> int:
    """Output k of SplitMix64(seed) in counter form (BASELINE.md 'Synthetic inputs')."""
    z = (seed + (k + 1) * GOLDEN) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def splitmix64_array(seed: int, first: int, n: int) -> np.ndarray:
    """Vectorised splitmix64_at(seed, first..first+n-1) as uint64."""
    with np.errstate(over="ignore"):
        k = np.arange(first + 1, first + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream_bytes(seed: int, start: int, n: int) -> bytes:
    """Bytes [start, start+n) of the little-endian SplitMix64(seed) byte stream."""
    if n <= 0:
        return b""
    w0 = start // 8
    w1 = (start + n + 7) // 8
    words = splitmix64_array(seed, w0, w1 - w0).astype("<u8").tobytes()
    off = start - 8 * w0
    return words[off : off + n]


def bimodal_lengths(seed: int, first: int, n: int) -> np.ndarray:
    """40 % 64 B / 60 % 1350 B, interleaved (BASELINE.json configs[2])."""
    x = splitmix64_array(seed, first, n)
    return np.where(x % np.uint64(5) < np.uint64(2), 64, 1350).astype(np.uint32)


# ------------------------------------------------------------------ C oracle
class COracle:
    """ctypes view of oracle/libsalamander_ref.so (built by oracle/Makefile)."""

    def __init__(self, path: str | None = None):
        path = path or os.path.join(_HERE, "libsalamander_ref.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        u8p = ctypes.c_void_p
        sz = ctypes.c_size_t
        u64 = ctypes.c_uint64
        u32 = ctypes.c_uint32
        lib.oracle_blake2b.argtypes = [u8p, sz, u8p, sz]
        lib.oracle_blake2b.restype = None
        lib.oracle_salamander_key.argtypes = [u8p, sz, u8p, u8p]
        lib.oracle_salamander_key.restype = None
        lib.oracle_salamander_obfuscate.argtypes = [u8p, sz, u8p, sz, u8p, u8p, sz]
        lib.oracle_salamander_obfuscate.restype = sz
        lib.oracle_salamander_deobfuscate.argtypes = [u8p, sz, u8p, sz, u8p, sz]
        lib.oracle_salamander_deobfuscate.restype = sz
        batch_args = [u8p, sz, u64, u8p, u8p, u64, u8p, u32]
        lib.oracle_obfuscate_batch.argtypes = batch_args + [u8p, u8p, u64, u64, u32, u8p, u8p]
        lib.oracle_obfuscate_batch.restype = u64
        lib.oracle_deobfuscate_batch.argtypes = batch_args + [u8p, u64, u64, u32, u8p, u8p]
        lib.oracle_deobfuscate_batch.restype = u64
        lib.oracle_fill_stream.argtypes = [u64, u64, u64, u8p]
        lib.oracle_fill_stream.restype = None
        lib.oracle_fill_salts.argtypes = [u64, u64, u64, u8p]
        lib.oracle_fill_salts.restype = None
        lib.oracle_fill_bimodal_lengths.argtypes = [u64, u64, u64, u8p]
        lib.oracle_fill_bimodal_lengths.restype = None
        lib.oracle_run_uniform_threads.argtypes = [ctypes.c_int, u8p, sz, u64, u8p, u64, u32, u8p, u8p, u64, ctypes.c_int]
        lib.oracle_run_uniform_threads.restype = ctypes.c_int
        self.lib = lib

    @staticmethod
    def _p(a):
        if a is None:
            return None
        if isinstance(a, (bytes, bytearray)):
            a = np.frombuffer(a, dtype=np.uint8)
        return a.ctypes.data

    def blake2b(self, data: bytes, outlen: int) -> bytes:
        out = np.zeros(outlen, np.uint8)
        src = np.frombuffer(bytes(data) or b"\0", np.uint8)
        self.lib.oracle_blake2b(out.ctypes.data, outlen, src.ctypes.data, len(data))
        return out.tobytes()

    def key(self, psk: bytes, salt: bytes) -> bytes:
        out = np.zeros(32, np.uint8)
        p = np.frombuffer(psk, np.uint8)
        s = np.frombuffer(bytes(salt[:8]), np.uint8)
        self.lib.oracle_salamander_key(p.ctypes.data, len(psk), s.ctypes.data, out.ctypes.data)
        return out.tobytes()

    def obfuscate(self, psk: bytes, payload: bytes, salt: bytes, out_len: int) -> bytes:
        out = np.zeros(max(out_len, 1), np.uint8)
        p = np.frombuffer(psk, np.uint8)
        src = np.frombuffer(bytes(payload) or b"\0", np.uint8)
        s = np.frombuffer(bytes(salt[:8]), np.uint8)
        n = self.lib.oracle_salamander_obfuscate(p.ctypes.data, len(psk), src.ctypes.data, len(payload), s.ctypes.data, out.ctypes.data, out_len)
        return out[:n].tobytes()

    def deobfuscate(self, psk: bytes, wire: bytes, out_len: int) -> bytes:
        out = np.zeros(max(out_len, 1), np.uint8)
        p = np.frombuffer(psk, np.uint8)
        src = np.frombuffer(bytes(wire) or b"\0", np.uint8)
        n = self.lib.oracle_salamander_deobfuscate(p.ctypes.data, len(psk), src.ctypes.data, len(wire), out.ctypes.data, out_len)
        return out[:n].tobytes()

    def batch(self, obf: bool, psk: bytes, n: int, inp: np.ndarray, *, in_off=None, in_stride=0,
              in_len=None, len_uniform=0, salts=None, out_cap: int, out_stride=0, pkt_cap=0):
        """Run the batch restatement; returns (out bytes ndarray, out_off, out_len, total)."""
        p = np.frombuffer(psk, np.uint8)
        out = np.zeros(max(out_cap, 1), np.uint8)
        out_off = np.zeros(max(n, 1), np.uint64)
        out_len = np.zeros(max(n, 1), np.uint32)
        args = [p.ctypes.data, len(psk), n, self._p(inp), self._p(in_off), in_stride, self._p(in_len), len_uniform]
        if obf:
            total = self.lib.oracle_obfuscate_batch(*args, self._p(salts), out.ctypes.data, out_cap, out_stride, pkt_cap,
                                                    out_off.ctypes.data, out_len.ctypes.data)
        else:
            total = self.lib.oracle_deobfuscate_batch(*args, out.ctypes.data, out_cap, out_stride, pkt_cap,
                                                      out_off.ctypes.data, out_len.ctypes.data)
        return out[:out_cap], out_off[:n], out_len[:n], int(total)

    def fill_stream(self, seed: int, start: int, n: int) -> np.ndarray:
        a = np.empty(max(n, 1), np.uint8)
        self.lib.oracle_fill_stream(seed, start, n, a.ctypes.data)
        return a[:n]

    def salts(self, seed: int, first: int, n: int) -> np.ndarray:
        a = np.empty(max(n, 1), np.uint64)
        self.lib.oracle_fill_salts(seed, first, n, a.ctypes.data)
        return a[:n]

    def bimodal_lengths(self, seed: int, first: int, n: int) -> np.ndarray:
        a = np.empty(max(n, 1), np.uint32)
        self.lib.oracle_fill_bimodal_lengths(seed, first, n, a.ctypes.data)
        return a[:n]

    def run_uniform(self, obf: bool, psk: bytes, n: int, inp: np.ndarray, in_stride: int, length: int,
                    salts: np.ndarray | None, out: np.ndarray, out_stride: int, nthreads: int) -> None:
        p = np.frombuffer(psk, np.uint8)
        rc = self.lib.oracle_run_uniform_threads(1 if obf else 0, p.ctypes.data, len(psk), n, inp.ctypes.data, in_stride,
                                                 length, self._p(salts), out.ctypes.data, out_stride, nthreads)
        if rc != 0:
            raise RuntimeError("oracle_run_uniform_threads failed")
