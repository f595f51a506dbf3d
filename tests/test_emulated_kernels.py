"""CPU tier: the HIP kernel sources, compiled for the host against tests/emu/hip_emu.h
(CPU emulation of the HIP subset they use) under AddressSanitizer, checked
against the C oracle.  This exercises the kernels' indexing, the packed-layout
scan, chunk ownership, the tile kernel's chunk classes and quad hash, and the
host paths without a GPU, and fails on any out-of-bounds access.  Test infrastructure only: the
product library (hysteria_amd/libhyobfs.so) is never built this way."""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu"))
from emu_build import ensure_emu_lib  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu")
LIB = os.path.join(EMU, "libhyobfs_emu.so")


def _asan_runtime():
    c = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return c[-1] if c else None


@pytest.fixture(scope="module")
def emu_lib():
    if not _asan_runtime() or not os.path.exists("/opt/rocm/llvm/bin/clang++"):
        pytest.skip("clang/ASan runtime not available")
    return ensure_emu_lib()


# Each test's case: (run_case.py arguments, extra environment), from its parameters.
SPECS = {
    "test_emulated_packed_auto": lambda p: (p["which"], p["args"], {"HYEMU_CUS": "2"}),
    "test_emulated_tile_kernel": lambda p: (p["which"], p["args"], {"HYOBFS_KERNEL": "tile", "HYEMU_CUS": "2"}),
    "test_emulated_tile_kernel_exact_input": lambda p: ("slotted", p["args"], {"HYOBFS_KERNEL": "tile", "HYEMU_CUS": "2"}),
    "test_emulated_wave_kernel_forced": lambda p: None if p["which"] in ("conn", "host", "coalesce", "quic",
                                                                         "lifecycle", "deadline", "closerace") else (
        p["which"], p["args"], {"HYEMU_CUS": p["cus"], "HYOBFS_KERNEL": "wave"}),
    "test_emulated_wave_kernel_run_lengths": lambda p: (
        p["which"], p["args"], {"HYOBFS_RUN_LOG2": p["run_log2"], "HYOBFS_KERNEL": "wave"}),
    "test_emulated_wave_kernel_packed_run_lengths": lambda p: (
        p["which"], p["args"], {"HYOBFS_PACKED_RUN_LOG2": p["run_log2"], "HYOBFS_RUN_LOG2": p["run_log2"],
                                "HYOBFS_KERNEL": "wave"}),
    "test_emulated_kernel_vs_oracle": lambda p: (p["which"], p["args"], {"HYEMU_CUS": p["cus"]}),
    "test_emulated_split_launches": lambda p: (p["which"], p["args"], dict(p["env"])),
    "test_emulated_contiguous_input_slotted": lambda p: ("contig", p["args"], {"HYEMU_CUS": "2"}),
    "test_emulated_rx_gpu_failure_reports_eio": lambda p: ("rxfail", "", {"HYEMU_FAIL_EVENTS_FROM": "5"}),
    "test_emulated_tx_gpu_failure_reports_eio": lambda p: ("txfail", "", {"HYEMU_FAIL_EVENTS_FROM": "1"}),
    "test_emulated_contiguous_input_auto": lambda p: ("contig", p["args"], {"HYEMU_CUS": "2"}),
    "test_emulated_contiguous_input_flat": lambda p: ("contig", p["args"], {"HYEMU_CUS": "2", "HYOBFS_KERNEL": "flat",
                                                                           "HYOBFS_FLAT_HASHERS": p["hashers"]}),
    "test_emulated_contiguous_input_prepass_offsets": lambda p: ("contig", p["args"], {
        "HYEMU_CUS": "2", "HYOBFS_PACKED_RUN_LOG2": "3"}),
}


def _spec(item):
    f = SPECS.get(getattr(item, "originalname", None))
    return f(item.callspec.params if hasattr(item, "callspec") else {}) if f else None


def _key(spec):
    return spec[0], spec[1], tuple(sorted(spec[2].items()))


def _launch(emu_lib, spec):
    which, args, extra_env = spec
    env = dict(os.environ, HYOBFS_LIB=emu_lib, LD_PRELOAD=_asan_runtime(), ASAN_OPTIONS="detect_leaks=0",
               **extra_env)
    return subprocess.run([sys.executable, os.path.join(EMU, "run_case.py"), which] + args.split(), env=env,
                          capture_output=True, text=True, timeout=600)


_RESULTS = {}


@pytest.fixture(scope="module", autouse=True)
def emu_prefetch(emu_lib, request):
    """Runs every selected case's subprocess up front, 6 at a time (each is an
    independent emulated run); the tests then check their own result."""
    specs = {_key(sp): sp for it in request.session.items if it.module.__name__ == __name__
             for sp in [_spec(it)] if sp}
    with ThreadPoolExecutor(max_workers=6) as ex:
        futs = {k: ex.submit(_launch, emu_lib, sp) for k, sp in specs.items()}
        for k, f in futs.items():
            _RESULTS[k] = f.result()
    yield


def _run(emu_lib, which, args, extra_env):
    spec = (which, args, extra_env)
    r = _RESULTS.get(_key(spec)) or _launch(emu_lib, spec)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


CASES = [
    ("uniform", "257 1200 1", "1"),
    ("uniform", "600 1200 0", "2"),
    ("bimodal", "3000 1", "3"),
    ("bimodal", "3000 0", "1"),
    ("bimodal", "5000 1", "1"),      # one workgroup, 20 sub-tiles
    ("ragged", "7 2000 2100 1 0", "3"),
    ("ragged", "8 2000 2100 0 0", "4"),
    ("ragged", "9 1500 2100 1 1", "2"),
    ("ragged", "10 1500 40 1 0", "2"),   # tiny datagrams: several per 16-byte chunk
    ("ragged", "11 1500 40 0 1", "2"),
    ("host", "1000 300 96 1", "2"),      # host-resident batch, chunked pipeline
    ("host", "1000 300 96 0", "2"),
    ("host", "600 300 0 1 1", "2"),      # every array mapped (hyobfs_host_alloc): the zero-copy batch
    ("host", "600 300 0 0 1", "2"),
    ("conn", "64 120", "2"),             # UDP loopback through the conn wrapper (conn.go)
    ("coalesce", "8 150 4 32", "2"),     # many threads on one coalescing conn (hyobfs_conn_set_coalescing)
    ("lifecycle", "60 16", "2"),         # close() flushes, wakes blocked callers; deferred send errors
    ("deadline", "", "2"),               # Set{Read,Write}Deadline, both modes
    ("closerace", "8 1500", "2"),        # 8 threads in read_from / write_to while close() runs, under ASan
    ("far", "200 300 15 1", "8"),        # workgroup bases beyond 2^31
    ("far", "200 300 15 0", "8"),
    ("gecko", "40 7", "2"),              # Gecko frame encode + parse kernels (gecko.hip), aligned sweep
    ("gecko", "60 8 1", "2"),            # ... ascending frames with gaps: gap bytes untouched
    ("gecko", "60 9 2", "2"),            # ... shuffled placement: the per-frame path
    ("gecko", "70 10 3", "2"),           # ... tiny frames, several per 16-byte chunk
    ("gecko", "300 11 0", "2"),          # ... many groups
    ("punch", "300 5 3", "2"),           # realm punch matcher (realm.hip)
    ("quic", "2", "2"),                  # QUIC Initial unprotect + ReadCryptoPayload kernels (quic.hip)
]


# The wave kernel (forced for packed layouts too) and its run length (datagrams per run = 2^run_log2, salamander_wave.h):
# single-datagram runs, short runs and whole 64-datagram groups, on ragged
# slotted and packed layouts with tiny datagrams, gaps and zero widths.
RUN_CASES = [
    ("ragged", "9 1500 2100 1 1", "0"),
    ("ragged", "11 1500 40 0 1", "0"),
    ("ragged", "12 700 100 1 0", "1"),
    ("ragged", "13 700 30 0 0", "3"),
    ("ragged", "14 700 200 0 1", "3"),
    ("ragged", "15 700 19 1 1", "6"),
    ("uniform", "300 1200 1", "6"),
    ("uniform", "300 1200 0", "0"),
]


# Packed batches under AUTO (the wave kernel): tiny datagrams (several per 16-byte
# chunk, empty ones), ragged 1-6 KiB, out_cap cutting the batch, deobfuscate of real
# wire with drops (wire of 8 bytes), PSK lengths across salt words.
PACKED_CASES = [
    ("pcap", "1 300 40 1 100 16"), ("pcap", "2 300 40 0 100 16"), ("pcap", "3 400 2100 1 100 9"),
    ("pcap", "4 400 2100 0 100 121"), ("pcap", "5 200 6000 1 100 16"), ("pcap", "6 200 6000 0 100 33"),
    ("pcap", "7 500 1400 1 60 16"), ("pcap", "8 500 1400 0 70 127"), ("pcap", "9 17 3 1 100 4"),
    ("bimodal", "1000 1"), ("bimodal", "1000 0"),
]


# Contiguous input (in_off NULL, in_stride 0; tests/emu/run_case.py case_contig:
# seed n dist obf cap% psk_len [pkt_cap misalign out_stride]).  Packed output under
# AUTO: the wave kernel taking its input offsets from the scan of the lengths, or,
# with packed runs of 8, the prepass's input offsets (in_offsets_kernel); under
# HYOBFS_KERNEL=flat from 16-byte aligned input the flat kernel (16 KiB output tiles,
# salamander_flat.h), its keys from the hasher workgroups (4 hashers: published key
# records) or, with none, hashed by each tile after its poll gives up (the fallback).
# Bimodal, 0..2100 B, tiny (several datagrams per chunk, tiles of several passes),
# 1-5 KB, zero-length datagrams; out_cap cuts, pkt_cap drops (dropped input inside a
# tile's window), real wire with 8-byte datagrams, PSKs across salt words and the
# two-block case, a misaligned input (the wave kernel).  The flat kernel's emulation
# costs a 256-thread workgroup per 16 KiB of output, so its cases are a few hundred KB.
CONTIG_CASES = [
    "1 3000 0 1 100 16", "2 3000 0 0 100 16", "3 2000 1 1 100 16", "4 2000 1 0 100 33", "5 3000 2 1 100 16",
    "6 3000 2 0 100 121", "7 300 3 1 100 16", "8 300 3 0 100 4", "9 3000 4 1 100 16", "10 3000 4 0 100 16",
    "11 2000 1 1 60 16", "12 2000 1 0 70 127", "13 2000 1 1 100 16 1000", "14 2000 1 0 100 16 900",
    "15 3000 0 1 100 16 0 1", "16 3000 0 0 100 16 0 1", "17 3000 2 1 50 16",
]
FLAT_CASES = [
    "1 600 0 1 100 16", "2 600 0 0 100 16", "3 500 1 1 100 16", "4 500 1 0 100 33", "5 3000 2 1 100 16",
    "6 3000 2 0 100 121", "7 100 3 1 100 16", "8 100 3 0 100 4", "9 600 4 1 100 16", "10 600 4 0 100 16",
    "11 500 1 1 60 16", "12 500 1 0 70 127", "13 500 1 1 100 16 1000", "14 500 1 0 100 16 900",
    "15 600 0 1 100 16 0 1", "16 600 0 0 100 16 0 1", "17 3000 2 1 50 16", "18 600 0 1 100 9",
    "19 600 0 0 100 128",
]


@pytest.mark.parametrize("args", CONTIG_CASES)
def test_emulated_contiguous_input_auto(emu_lib, args):
    _run(emu_lib, "contig", args, {"HYEMU_CUS": "2"})


@pytest.mark.parametrize("hashers", ["4", "0"])
@pytest.mark.parametrize("args", FLAT_CASES)
def test_emulated_contiguous_input_flat(emu_lib, args, hashers):
    _run(emu_lib, "contig", args, {"HYEMU_CUS": "2", "HYOBFS_KERNEL": "flat", "HYOBFS_FLAT_HASHERS": hashers})


@pytest.mark.parametrize("args", [CONTIG_CASES[i] for i in (1, 2, 10)])
def test_emulated_contiguous_input_prepass_offsets(emu_lib, args):
    _run(emu_lib, "contig", args, {"HYEMU_CUS": "2", "HYOBFS_PACKED_RUN_LOG2": "3"})


# Contiguous input into SLOTS (out_stride > 0): the prepass writes the input offsets
# into the caller's workspace (8 B per datagram after the two sum arrays), the wave
# kernel reads them.  Bimodal into 1358/1350-byte slots (everything fits), 0..2100 B
# into 1200-byte slots (the slot drops the long ones), out_cap cutting the slots,
# pkt_cap drops, a misaligned input, a two-block PSK, tiny datagrams in 48-byte slots.
CONTIG_SLOTTED = [
    "21 1000 0 1 100 16 0 0 1358", "22 1000 0 0 100 16 0 0 1350", "23 800 1 1 100 16 0 0 1200",
    "24 800 1 0 100 33 0 0 1200", "25 800 1 1 60 16 0 0 2112", "26 800 1 0 70 127 0 0 2104",
    "27 800 1 1 100 16 900 0 1208", "28 800 1 0 100 16 700 1 2104", "29 1000 2 1 100 121 0 0 48",
    "30 1000 4 0 100 16 0 0 1350",
]


@pytest.mark.parametrize("args", CONTIG_SLOTTED)
def test_emulated_contiguous_input_slotted(emu_lib, args):
    _run(emu_lib, "contig", args, {"HYEMU_CUS": "2"})


@pytest.mark.parametrize("which,args", PACKED_CASES)
def test_emulated_packed_auto(emu_lib, which, args):
    _run(emu_lib, which, args, {"HYEMU_CUS": "2"})


# The tile kernel (salamander_tile.h): slotted batches whose region edges are all
# multiples of 8.  Dense slots of 8 mod 16 (obfuscate 1200 -> 1208, deobfuscate
# 1216 -> 1208) and 0 mod 16, gapped slots (gap bytes untouched), input strides with
# padding, partial last tiles, slots needing several compose passes (9000 B), every
# salt-word position of the PSK (lengths 4..127, including the two-block case
# 121..127), and layouts that do not qualify (odd lengths, inputs over 4 KiB: the
# wave kernel).
from tile_cases import TILE_CASES  # noqa: E402  (the tile kernel's layout grid, shared with the GPU tier)


@pytest.mark.parametrize("which,args", TILE_CASES)
def test_emulated_tile_kernel(emu_lib, which, args):
    _run(emu_lib, which, args, {"HYOBFS_KERNEL": "tile", "HYEMU_CUS": "2"})


# Short datagrams in long input slots, the input buffer ending right after the last
# datagram's L bytes ((n-1) x stride + L, all the API promises): the tile kernel's
# obfuscate prefetch loads (salamander_tile.h, HY_TILE_PREFETCH) stay inside each
# datagram, ASan reports any byte read past the buffer.
@pytest.mark.parametrize("args", ["40 16 1 8 4080 16 1", "40 24 0 8 4072 16 1", "33 1200 1 0 2896 16 1"])
def test_emulated_tile_kernel_exact_input(emu_lib, args):
    _run(emu_lib, "slotted", args, {"HYOBFS_KERNEL": "tile", "HYEMU_CUS": "2"})


# A batch split into several launches (salamander_tile.h launch_tile_sw: big batches
# go out as launches of at most HYOBFS_TILE_LAUNCH_TILES tiles; salamander_wave.h
# launch_wave_sw: HYOBFS_WAVE_LAUNCH_BLOCKS workgroups for packed batches): tiny limits
# so every case spans several launches, partial last launches included.
SPLIT_CASES = [
    ("uniform", "257 1200 1", (("HYOBFS_KERNEL", "tile"), ("HYOBFS_TILE_LAUNCH_TILES", "3"))),
    ("uniform", "301 1192 0", (("HYOBFS_KERNEL", "tile"), ("HYOBFS_TILE_LAUNCH_TILES", "5"))),
    ("slotted", "70 1208 0 8 0 16", (("HYOBFS_KERNEL", "tile"), ("HYOBFS_TILE_LAUNCH_TILES", "1"))),
    ("bimodal", "3000 1", (("HYOBFS_WAVE_LAUNCH_BLOCKS", "3"),)),
    ("bimodal", "3000 0", (("HYOBFS_WAVE_LAUNCH_BLOCKS", "2"),)),
    ("pcap", "4 400 2100 0 100 121", (("HYOBFS_WAVE_LAUNCH_BLOCKS", "1"),)),
]


@pytest.mark.parametrize("which,args,env", SPLIT_CASES)
def test_emulated_split_launches(emu_lib, which, args, env):
    _run(emu_lib, which, args, dict(env))


@pytest.mark.parametrize("which,args,run_log2", RUN_CASES)
def test_emulated_wave_kernel_run_lengths(emu_lib, which, args, run_log2):
    _run(emu_lib, which, args, {"HYOBFS_RUN_LOG2": run_log2, "HYOBFS_KERNEL": "wave"})


@pytest.mark.parametrize("which,args,run_log2", RUN_CASES + [("bimodal", "3000 1", "3"), ("bimodal", "5000 0", "2")])
def test_emulated_wave_kernel_packed_run_lengths(emu_lib, which, args, run_log2):
    """Packed layouts with runs shorter than the 64-datagram group: each run's output
    base is the tile prefix plus the widths of the tile's earlier datagrams."""
    _run(emu_lib, which, args, {"HYOBFS_PACKED_RUN_LOG2": run_log2, "HYOBFS_RUN_LOG2": run_log2,
                                "HYOBFS_KERNEL": "wave"})


@pytest.mark.parametrize("which,args,cus", CASES)
def test_emulated_wave_kernel_forced(emu_lib, which, args, cus):
    """The wave-group kernel (HYOBFS_KERNEL=wave) on every case, also where AUTO runs the tile kernel."""
    if which in ("conn", "host", "coalesce", "quic", "lifecycle", "deadline", "closerace"):
        pytest.skip("kernel-independent host paths run once, under the default kernel")
    _run(emu_lib, which, args, {"HYEMU_CUS": cus, "HYOBFS_KERNEL": "wave"})


@pytest.mark.parametrize("which,args,cus", CASES)
def test_emulated_kernel_vs_oracle(emu_lib, which, args, cus):
    _run(emu_lib, which, args, {"HYEMU_CUS": cus})


def test_emulated_rx_gpu_failure_reports_eio(emu_lib):
    """A coalescing connection's receive batch whose GPU step fails: ReadFrom raises EIO
    (once per failed batch) and nothing is counted as an invalid datagram (rx_dropped 0);
    the emulation fails every wait of the receive queue (HYEMU_FAIL_EVENTS_FROM=5)."""
    _run(emu_lib, "rxfail", "", {"HYEMU_FAIL_EVENTS_FROM": "5"})


def test_emulated_tx_gpu_failure_reports_eio(emu_lib):
    """A coalescing connection's send batch whose GPU step fails: the datagram is not
    sent, it counts as a tx error, and the next WriteTo raises EIO once (every event of
    the connection fails, HYEMU_FAIL_EVENTS_FROM=1)."""
    _run(emu_lib, "txfail", "", {"HYEMU_FAIL_EVENTS_FROM": "1"})
