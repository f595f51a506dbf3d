"""Builds tests/emu/libhyobfs_emu.so once per source change (test infrastructure).

Every test that loads the emulated build calls ensure_emu_lib(): under an
exclusive file lock (pytest-xdist workers and rank processes share the tree) it
rebuilds when a kernel/ABI source or hip_emu.h is newer than the library, into a
temporary name that is renamed over the old one, so no reader ever sees a
half-linked library.
"""
import fcntl
import glob
import os
import subprocess

EMU = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(EMU))
LIB = os.path.join(EMU, "libhyobfs_emu.so")
_SUFFIXES = (".h", ".hip", ".cpp")


def asan_runtime():
    c = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return c[-1] if c else None


def available():
    return bool(asan_runtime()) and os.path.exists("/opt/rocm/llvm/bin/clang++")


def _stale():
    srcs = [p for p in glob.glob(os.path.join(ROOT, "hysteria_amd", "csrc", "*")) if p.endswith(_SUFFIXES)]
    srcs.append(os.path.join(EMU, "hip_emu.h"))
    return not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(s) for s in srcs)


def ensure_emu_lib():
    with open(os.path.join(EMU, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if _stale():
            tmp = LIB + ".tmp"
            subprocess.run([os.path.join(EMU, "build.sh")], check=True, capture_output=True,
                           env=dict(os.environ, EMU_OUT=tmp))
            os.replace(tmp, LIB)
    return LIB
