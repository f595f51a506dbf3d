"""ctypes binding of libhyobfs.so (include/hyobfs.h).

The library holds the gfx950 kernels; there is no CPU fallback.  If the .so is
missing or does not load, importing the product API raises immediately.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HYOBFS_LIB") or os.path.join(_HERE, "libhyobfs.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hyobfs.h")

HYOBFS_OK = 0
HYOBFS_ERR_PSK_TOO_SHORT = -1
HYOBFS_ERR_INVALID = -2
HYOBFS_ERR_HIP = -3
HYOBFS_ERR_NOMEM = -4
HYOBFS_ERR_NO_DEVICE = -5
HYOBFS_ERR_IO = -6
HYOBFS_ERR_CLOSED = -7
ABI_VERSION = 4   # the HYOBFS_ABI_VERSION these bindings are written for (include/hyobfs.h)


class HyobfsBatch(ctypes.Structure):
    """struct hyobfs_batch (include/hyobfs.h)."""

    _fields_ = [
        ("n", ctypes.c_uint64),
        ("in_", ctypes.c_void_p),
        ("in_off", ctypes.c_void_p),
        ("in_stride", ctypes.c_uint64),
        ("in_len", ctypes.c_void_p),
        ("len_uniform", ctypes.c_uint32),
        ("pkt_cap", ctypes.c_uint32),
        ("salts", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("out_cap", ctypes.c_uint64),
        ("out_stride", ctypes.c_uint64),
        ("out_off", ctypes.c_void_p),
        ("out_len", ctypes.c_void_p),
        ("out_total", ctypes.c_void_p),
        ("workspace", ctypes.c_void_p),
        ("workspace_bytes", ctypes.c_uint64),
    ]


class HyobfsDgram(ctypes.Structure):
    """struct hyobfs_dgram (include/hyobfs_conn.h)."""

    _fields_ = [
        ("buf", ctypes.c_void_p),
        ("len", ctypes.c_uint32),
        ("cap", ctypes.c_uint32),
        ("addr", ctypes.c_uint8 * 128),
        ("addrlen", ctypes.c_uint32),
        ("pad_", ctypes.c_uint32),
    ]


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Names of every function declared in include/*.h."""
    names = []
    inc = os.path.dirname(path)
    for fn in sorted(os.listdir(inc)):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(inc, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"\b(hyobfs_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


_lib = None
_variants = {}   # other builds loaded side by side (in-process A/B runs, scripts/ab_variants.py)


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libhyobfs.so and declare the ABI.  Raises OSError if it is missing.
    A different ``path`` loads that build beside the default one (each CDLL keeps
    its own symbols)."""
    global _lib
    if path == LIB_PATH and _lib is not None:
        return _lib
    if path != LIB_PATH and path in _variants:
        return _variants[path]
    if not os.path.exists(path):
        raise OSError(f"{path} is missing: build it with `make -C hysteria_amd/csrc` "
                      "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(path, use_errno=True)
    vp, sz, u64, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    pctx = ctypes.c_void_p
    sig = {
        "hyobfs_abi_version": (i32, []),
        "hyobfs_build_id": (ctypes.c_char_p, []),
        "hyobfs_status_string": (ctypes.c_char_p, [i32]),
        "hyobfs_device_count": (i32, []),
        "hyobfs_device_pci_bus_id": (i32, [i32, ctypes.c_char_p, i32]),
        "hyobfs_salamander_new": (i32, [vp, sz, i32, ctypes.POINTER(ctypes.c_void_p)]),
        "hyobfs_salamander_free": (None, [pctx]),
        "hyobfs_salamander_device": (i32, [pctx]),
        "hyobfs_salamander_set_kernel": (i32, [pctx, i32]),
        "hyobfs_salamander_seed": (None, [pctx, u64]),
        "hyobfs_salamander_next_salts": (None, [pctx, vp, sz]),
        "hyobfs_salamander_key": (i32, [pctx, vp, vp]),
        "hyobfs_salamander_keys_batch": (i32, [pctx, vp, vp, u64, vp]),
        "hyobfs_salamander_obfuscate": (sz, [pctx, vp, sz, vp, vp, sz]),
        "hyobfs_salamander_obfuscate_auto": (sz, [pctx, vp, sz, vp, sz]),
        "hyobfs_salamander_deobfuscate": (sz, [pctx, vp, sz, vp, sz]),
        "hyobfs_batch_workspace_size": (u64, [u64]),
        "hyobfs_batch_workspace_bytes": (u64, [ctypes.POINTER(HyobfsBatch)]),
        "hyobfs_salamander_batch_kernel": (i32, [pctx, ctypes.POINTER(HyobfsBatch), i32]),
        "hyobfs_salamander_obfuscate_batch": (i32, [pctx, ctypes.POINTER(HyobfsBatch), vp]),
        "hyobfs_salamander_deobfuscate_batch": (i32, [pctx, ctypes.POINTER(HyobfsBatch), vp]),
        "hyobfs_salamander_obfuscate_batch_sharded": (i32, [vp, ctypes.POINTER(HyobfsBatch), i32]),
        "hyobfs_salamander_deobfuscate_batch_sharded": (i32, [vp, ctypes.POINTER(HyobfsBatch), i32]),
        "hyobfs_shard_bounds": (i32, [vp, u64, i32, vp]),
        "hyobfs_salamander_obfuscate_host": (i32, [pctx, ctypes.POINTER(HyobfsBatch), u64]),
        "hyobfs_salamander_deobfuscate_host": (i32, [pctx, ctypes.POINTER(HyobfsBatch), u64]),
        "hyobfs_host_alloc": (vp, [sz]),
        "hyobfs_host_free": (None, [vp]),
        "hyobfs_conn_wrap": (i32, [i32, pctx, u32, ctypes.POINTER(ctypes.c_void_p)]),
        "hyobfs_conn_close": (i32, [vp]),
        "hyobfs_conn_free": (None, [vp]),
        "hyobfs_conn_read_from": (ctypes.c_int64, [vp, vp, sz, vp, ctypes.POINTER(u32)]),
        "hyobfs_conn_write_to": (ctypes.c_int64, [vp, vp, sz, vp, u32]),
        "hyobfs_conn_read_batch": (i32, [vp, vp, u32]),
        "hyobfs_conn_write_batch": (i32, [vp, vp, u32]),
        "hyobfs_conn_set_coalescing": (i32, [vp, u32, u32]),
        "hyobfs_conn_flush": (i32, [vp]),
        "hyobfs_conn_set_read_deadline": (i32, [vp, ctypes.c_int64]),
        "hyobfs_conn_set_write_deadline": (i32, [vp, ctypes.c_int64]),
        "hyobfs_conn_stats": (i32, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        "hyobfs_synth_stream": (i32, [vp, u64, u64, u64, vp]),
        "hyobfs_synth_u64": (i32, [vp, u64, u64, u64, vp]),
        "hyobfs_synth_bimodal_lengths": (i32, [vp, u64, u64, u64, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    have = lib.hyobfs_abi_version()
    if have != ABI_VERSION:   # struct layouts and enum values differ between versions
        raise OSError(f"{path}: ABI version {have}, these bindings need {ABI_VERSION}: rebuild the library")
    if path == LIB_PATH:
        _lib = lib
    else:
        _variants[path] = lib
    return lib


def status_string(st: int) -> str:
    return load().hyobfs_status_string(st).decode()


class HyobfsError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {status_string(status)} ({status})" if what else status_string(status))


def check(status: int, what: str = "") -> None:
    if status != HYOBFS_OK:
        raise HyobfsError(status, what)
