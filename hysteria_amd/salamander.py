"""Salamander obfuscator on MI355X -- host-side mirror of the reference interface.

Mirrors ``salamanderObfuscator`` (apernet/hysteria ``extras/obfs/salamander.go:26-91``):

=====================================  ==============================================
reference (Go)                         here
=====================================  ==============================================
``newSalamanderObfuscator(psk)``       ``SalamanderObfuscator(psk, device)`` (:34-46)
``ErrPSKTooShort``                     ``PSKTooShortError`` (:21)
``Obfuscate(in, out []byte) int``      ``SalamanderObfuscator.obfuscate(in_, out)`` (:59-72)
``Deobfuscate(in, out []byte) int``    ``SalamanderObfuscator.deobfuscate(in_, out)`` (:74-86)
``keyLocked(salt)``                    ``SalamanderObfuscator.key(salt)`` (:88-91)
``RandSrc`` (math/rand)                ``seed()`` / ``next_salts()`` or an explicit ``salt=``
=====================================  ==============================================

plus the batch entry points (``obfuscate_batch`` / ``deobfuscate_batch``) that
carry N datagrams per launch.  Every call runs the gfx950 kernels of
``libhyobfs.so`` through its C ABI (``include/hyobfs.h``); there is no CPU path.
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import HyobfsBatch, check

SM_PSK_MIN_LEN = 4    # salamander.go:14
SM_SALT_LEN = 8       # salamander.go:15
SM_KEY_LEN = 32       # salamander.go:16
UDP_BUFFER_SIZE = 2048  # conn.go:10


class PSKTooShortError(ValueError):
    """ErrPSKTooShort (salamander.go:21)."""

    def __init__(self):
        super().__init__(f"PSK must be at least {SM_PSK_MIN_LEN} bytes")


def _cbuf(b, writable=False):
    """(pointer, length, keepalive) for a bytes-like object."""
    if isinstance(b, (bytes,)) and not writable:
        buf = ctypes.create_string_buffer(b, len(b)) if b else ctypes.create_string_buffer(1)
        return ctypes.addressof(buf), len(b), buf
    mv = memoryview(b).cast("B")
    if writable and mv.readonly:
        raise TypeError("out must be writable")
    n = mv.nbytes
    if n == 0:
        buf = ctypes.create_string_buffer(1)
        return ctypes.addressof(buf), 0, buf
    if mv.readonly:
        buf = ctypes.create_string_buffer(bytes(mv), n)
        return ctypes.addressof(buf), n, buf
    arr = (ctypes.c_char * n).from_buffer(mv)
    return ctypes.addressof(arr), n, (arr, mv)


def _ptr(x):
    """Device pointer of a torch tensor / int / None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _hptr(x):
    """Host pointer of a numpy array / CPU torch tensor / int / None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ctypes.data


def _stream(stream, *tensors):
    if stream is not None:
        return stream if isinstance(stream, int) else stream.cuda_stream
    for t in tensors:
        if t is not None and not isinstance(t, int) and getattr(t, "is_cuda", False):
            import torch
            return torch.cuda.current_stream(t.device).cuda_stream
    return None


def _make_batch(*, inp, n, in_off=None, in_stride=0, in_len=None, len_uniform=0, salts=None, out,
                out_cap=None, out_stride=0, pkt_cap=0, out_off=None, out_len=None, out_total=None,
                workspace=None, workspace_bytes=0) -> HyobfsBatch:
    """struct hyobfs_batch from device tensors (layout rules: include/hyobfs.h)."""
    if out_cap is None:
        out_cap = out.numel() * out.element_size() if hasattr(out, "numel") else 0
    return HyobfsBatch(n=n, in_=_ptr(inp), in_off=_ptr(in_off), in_stride=in_stride,
                       in_len=_ptr(in_len), len_uniform=len_uniform, pkt_cap=pkt_cap,
                       salts=_ptr(salts), out=_ptr(out), out_cap=out_cap, out_stride=out_stride,
                       out_off=_ptr(out_off), out_len=_ptr(out_len), out_total=_ptr(out_total),
                       workspace=_ptr(workspace), workspace_bytes=workspace_bytes)


class SalamanderObfuscator:
    """A Salamander obfuscator bound to one MI355X (HIP device ``device``)."""

    def __init__(self, psk: bytes, device: int = 0, lib_path: str | None = None):
        lib = _lib.load(lib_path) if lib_path else _lib.load()
        psk = bytes(psk)
        if len(psk) < SM_PSK_MIN_LEN:
            raise PSKTooShortError()
        h = ctypes.c_void_p()
        pbuf = ctypes.create_string_buffer(psk, len(psk))
        st = lib.hyobfs_salamander_new(pbuf, len(psk), device, ctypes.byref(h))
        if st == _lib.HYOBFS_ERR_PSK_TOO_SHORT:
            raise PSKTooShortError()
        check(st, "hyobfs_salamander_new")
        self._lib = lib
        self._h = h
        self.psk = psk
        self.device = device

    # -------------------------------------------------------------- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.hyobfs_salamander_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    KERNELS = {"auto": 0, "wave": 1, "tile": 2, "flat": 3}

    def set_kernel(self, kernel: str) -> None:
        """Batch kernel of this context: "auto" (the tile kernel where it applies, else the
        wave-group kernel), "wave" (forced), "flat" (the flat kernel on contiguous input
        into packed output, auto elsewhere) or "tile" (= auto; include/hyobfs.h,
        HYOBFS_KERNEL_*)."""
        check(self._lib.hyobfs_salamander_set_kernel(self._h, self.KERNELS[kernel]), "set_kernel")
        self.kernel = kernel

    # ------------------------------------------------------------ salt source
    def seed(self, seed: int) -> None:
        """Make the salt source deterministic (the reference's RandSrc, salamander.go:29)."""
        self._lib.hyobfs_salamander_seed(self._h, seed & ((1 << 64) - 1))

    def next_salts(self, n: int) -> bytes:
        buf = ctypes.create_string_buffer(max(8 * n, 1))
        self._lib.hyobfs_salamander_next_salts(self._h, buf, n)
        return buf.raw[: 8 * n]

    # ------------------------------------------------------------- per packet
    def key(self, salt: bytes) -> bytes:
        """keyLocked (salamander.go:88-91), computed on the GPU."""
        salt = bytes(salt)
        if len(salt) < SM_SALT_LEN:
            raise ValueError("salt must be 8 bytes")
        out = ctypes.create_string_buffer(SM_KEY_LEN)
        check(self._lib.hyobfs_salamander_key(self._h, salt[:8], out), "hyobfs_salamander_key")
        return out.raw

    def obfuscate(self, in_, out, salt: bytes | None = None) -> int:
        """Obfuscate(in, out []byte) int (salamander.go:59-72).

        Writes ``salt || in ^ key`` into ``out`` and returns the byte count, or 0
        when ``len(out) < len(in) + 8``.  ``salt=None`` draws it from the
        context's generator, like the reference's RandSrc.
        """
        ip, il, _k1 = _cbuf(in_)
        op, ol, _k2 = _cbuf(out, writable=True)
        if salt is None:
            return self._lib.hyobfs_salamander_obfuscate_auto(self._h, ip, il, op, ol)
        salt = bytes(salt)
        if len(salt) < SM_SALT_LEN:
            raise ValueError("salt must be 8 bytes")
        return self._lib.hyobfs_salamander_obfuscate(self._h, ip, il, salt[:8], op, ol)

    def deobfuscate(self, in_, out) -> int:
        """Deobfuscate(in, out []byte) int (salamander.go:74-86); 0 = invalid packet."""
        ip, il, _k1 = _cbuf(in_)
        op, ol, _k2 = _cbuf(out, writable=True)
        return self._lib.hyobfs_salamander_deobfuscate(self._h, ip, il, op, ol)

    # ------------------------------------------------------------------ batch
    def _batch(self, obf, *, stream=None, **kw):
        b = _make_batch(**kw)
        s = _stream(stream, kw["inp"], kw["out"])
        f = self._lib.hyobfs_salamander_obfuscate_batch if obf else self._lib.hyobfs_salamander_deobfuscate_batch
        check(f(self._h, ctypes.byref(b), s), "obfuscate_batch" if obf else "deobfuscate_batch")

    def batch_kernel(self, obf: bool, *, inp, n, out, **kw) -> str:
        """The kernel a batch call with these arguments would run ("tile" / "flat" / "wave"; "none"
        for an empty batch): hyobfs_salamander_batch_kernel, no device work."""
        b = _make_batch(inp=inp, n=n, out=out, **kw)
        k = self._lib.hyobfs_salamander_batch_kernel(self._h, ctypes.byref(b), int(bool(obf)))
        check(min(k, 0), "batch_kernel")
        return {0: "none", 1: "wave", 2: "tile", 3: "flat"}[k]

    @staticmethod
    def workspace_bytes(*, inp, n, out, **kw) -> int:
        """hyobfs_batch_workspace_bytes: the device scratch a batch call with these
        arguments needs under any kernel choice (0: none)."""
        b = _make_batch(inp=inp, n=n, out=out, **kw)
        return int(_lib.load().hyobfs_batch_workspace_bytes(ctypes.byref(b)))

    def obfuscate_batch(self, inp, n, *, salts, out, **kw) -> None:
        """Obfuscate n datagrams on the device (layout rules: include/hyobfs.h).

        Tensors are device tensors (torch.uint8 / int64 / int32 views); the call
        enqueues on the current torch stream of ``out`` unless ``stream`` is given.
        """
        self._batch(True, inp=inp, n=n, salts=salts, out=out, **kw)

    def deobfuscate_batch(self, inp, n, *, out, **kw) -> None:
        """Deobfuscate n datagrams on the device; out_len[i] = 0 marks a dropped packet."""
        self._batch(False, inp=inp, n=n, out=out, **kw)

    def _host(self, obf, *, inp, n, in_stride, out, out_stride, in_len=None, len_uniform=0, salts=None,
              out_len=None, pkt_cap=0, chunk=0):
        b = HyobfsBatch(n=n, in_=_hptr(inp), in_stride=in_stride, in_len=_hptr(in_len), len_uniform=len_uniform,
                        pkt_cap=pkt_cap, salts=_hptr(salts), out=_hptr(out), out_cap=n * out_stride,
                        out_stride=out_stride, out_len=_hptr(out_len))
        f = self._lib.hyobfs_salamander_obfuscate_host if obf else self._lib.hyobfs_salamander_deobfuscate_host
        check(f(self._h, ctypes.byref(b), chunk), "obfuscate_host" if obf else "deobfuscate_host")

    def obfuscate_host(self, inp, n, *, in_stride, salts, out, out_stride, **kw) -> None:
        """Obfuscate n datagrams that live in HOST memory (slotted rings, include/hyobfs.h):
        pinned staging, H2D / kernel / D2H overlapped on three streams; synchronous."""
        self._host(True, inp=inp, n=n, in_stride=in_stride, salts=salts, out=out, out_stride=out_stride, **kw)

    def deobfuscate_host(self, inp, n, *, in_stride, out, out_stride, **kw) -> None:
        """Deobfuscate n host-resident datagrams (out_len[i] = 0 marks a dropped one)."""
        self._host(False, inp=inp, n=n, in_stride=in_stride, out=out, out_stride=out_stride, **kw)

    def keys_batch(self, salts, keys, n, stream=None) -> None:
        """keys[32*i:32*i+32] = BLAKE2b-256(PSK || salts[i]) for n device-resident salts."""
        check(self._lib.hyobfs_salamander_keys_batch(self._h, _ptr(salts), _ptr(keys), n,
                                                     _stream(stream, keys)), "keys_batch")


def new_salamander_obfuscator(psk: bytes, device: int = 0) -> SalamanderObfuscator:
    """newSalamanderObfuscator (salamander.go:34-46)."""
    return SalamanderObfuscator(psk, device)


def _sharded(obf, obfuscators, shards) -> None:
    if len(obfuscators) != len(shards):
        raise ValueError("one obfuscator (context) per shard")
    lib = _lib.load()
    arr = (HyobfsBatch * len(shards))(*[_make_batch(**kw) for kw in shards])
    ctxs = (ctypes.c_void_p * len(shards))(*[o._h for o in obfuscators])
    f = lib.hyobfs_salamander_obfuscate_batch_sharded if obf else lib.hyobfs_salamander_deobfuscate_batch_sharded
    check(f(ctxs, arr, len(shards)), "obfuscate_batch_sharded" if obf else "deobfuscate_batch_sharded")


def obfuscate_batch_sharded(obfuscators, shards) -> None:
    """Shard i (keyword dict of obfuscate_batch's arguments, tensors on the device of
    obfuscators[i]) runs on obfuscators[i]'s stream; returns when every shard is done."""
    _sharded(True, obfuscators, shards)


def deobfuscate_batch_sharded(obfuscators, shards) -> None:
    _sharded(False, obfuscators, shards)


def device_count() -> int:
    return _lib.load().hyobfs_device_count()


def device_pci_bus_id(device: int) -> str:
    """hyobfs_device_pci_bus_id: the PCI bus id of HIP device ``device`` (which card)."""
    buf = ctypes.create_string_buffer(64)
    check(_lib.load().hyobfs_device_pci_bus_id(device, buf, 64), "device_pci_bus_id")
    return buf.value.decode()


def workspace_size(n: int) -> int:
    return _lib.load().hyobfs_batch_workspace_size(n)


def build_id() -> str:
    """Kernel-source hash the loaded libhyobfs.so was built from (scripts/src_sha.py)."""
    return _lib.load().hyobfs_build_id().decode()


# ------------------------------------------------------------- synthetic inputs
def synth_stream(dst, nbytes: int, seed: int, start: int = 0, stream=None) -> None:
    """dst[:nbytes] = bytes [start, start+nbytes) of the SplitMix64(seed) stream (device)."""
    check(_lib.load().hyobfs_synth_stream(_ptr(dst), nbytes, seed, start, _stream(stream, dst)), "synth_stream")


def synth_u64(dst, n: int, seed: int, first: int = 0, stream=None) -> None:
    check(_lib.load().hyobfs_synth_u64(_ptr(dst), n, seed, first, _stream(stream, dst)), "synth_u64")


def synth_bimodal_lengths(dst, n: int, seed: int, first: int = 0, stream=None) -> None:
    check(_lib.load().hyobfs_synth_bimodal_lengths(_ptr(dst), n, seed, first, _stream(stream, dst)),
          "synth_bimodal_lengths")
