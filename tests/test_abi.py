"""CPU tests of the drop-in boundary: libhyobfs.so loads, exports every symbol
declared in include/*.h, and its struct layout matches the header (checked
by compiling a probe against the header with gcc).  No compute without a GPU."""
import ctypes
import os
import subprocess

import pytest

from hysteria_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = _lib.header_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(names) <= exported


def test_abi_basics():
    lib = _lib.load()
    assert lib.hyobfs_abi_version() == _lib.ABI_VERSION == 4
    assert _lib.status_string(_lib.HYOBFS_ERR_PSK_TOO_SHORT) == "PSK must be at least 4 bytes"
    assert _lib.status_string(_lib.HYOBFS_ERR_CLOSED) == "use of closed connection"
    assert lib.hyobfs_batch_workspace_size(0) == 8
    assert lib.hyobfs_batch_workspace_size(257) == 3 * 8


def test_psk_too_short_before_device_check():
    """ErrPSKTooShort comes from the constructor (salamander.go:35-37) on any machine."""
    import hysteria_amd
    with pytest.raises(hysteria_amd.PSKTooShortError):
        hysteria_amd.SalamanderObfuscator(b"abc")


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import hysteria_amd
    with pytest.raises(_lib.HyobfsError) as e:
        hysteria_amd.SalamanderObfuscator(b"average_password")
    assert e.value.status == _lib.HYOBFS_ERR_NO_DEVICE


def test_batch_struct_layout_matches_header(tmp_path):
    fields = [f[0] for f in _lib.HyobfsBatch._fields_]
    cnames = ["n", "in", "in_off", "in_stride", "in_len", "len_uniform", "pkt_cap", "salts", "out",
              "out_cap", "out_stride", "out_off", "out_len", "out_total", "workspace", "workspace_bytes"]
    assert len(fields) == len(cnames)
    src = tmp_path / "probe.c"
    body = "\n".join(f'printf("%zu\\n", offsetof(hyobfs_batch, {c}));' for c in cnames)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "hyobfs.h"\nint main(void){\n'
                   + body + '\nprintf("%zu\\n", sizeof(hyobfs_batch));return 0;}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    py = [getattr(_lib.HyobfsBatch, f).offset for f in fields] + [ctypes.sizeof(_lib.HyobfsBatch)]
    assert vals == py


def _c_layout(tmp_path, header, ctype, cfields):
    src = tmp_path / f"probe_{ctype}.c"
    body = "\n".join(f'printf("%zu\\n", offsetof({ctype}, {c}));' for c in cfields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{header}"\nint main(void){{\n'
                   + body + f'\nprintf("%zu\\n", sizeof({ctype}));return 0;}}\n')
    exe = tmp_path / f"probe_{ctype}"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    return [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]


def test_gecko_and_realm_struct_layouts_match_headers(tmp_path):
    """The Python mirrors of hyobfs_gecko.h / hyobfs_realm.h structs (ctypes and numpy
    records) have the C offsets and sizes."""
    from hysteria_amd import gecko, realm
    for ct, cls in (("hyobfs_gecko_header", gecko.HyobfsGeckoHeader), ("hyobfs_gecko_batch", gecko.HyobfsGeckoBatch),
                    ("hyobfs_punch_attempt", realm.HyobfsPunchAttempt)):
        names = [f[0] for f in cls._fields_]
        header = "hyobfs_realm.h" if ct.startswith("hyobfs_punch") else "hyobfs_gecko.h"
        vals = _c_layout(tmp_path, header, ct, names)
        assert vals == [getattr(cls, f).offset for f in names] + [ctypes.sizeof(cls)], ct
    for ct, dt in (("hyobfs_gecko_frame", gecko.FRAME_DTYPE), ("hyobfs_gecko_parsed", gecko.PARSED_DTYPE),
                   ("hyobfs_punch_attempt", realm.ATTEMPT_DTYPE)):
        header = "hyobfs_realm.h" if ct.startswith("hyobfs_punch") else "hyobfs_gecko.h"
        vals = _c_layout(tmp_path, header, ct, list(dt.names))
        assert vals == [dt.fields[n][1] for n in dt.names] + [dt.itemsize], ct


def test_header_abi_version_matches_bindings():
    """HYOBFS_ABI_VERSION in the header, the library and the Python bindings agree."""
    import re
    text = open(os.path.join(ROOT, "include", "hyobfs.h")).read()
    assert int(re.search(r"#define HYOBFS_ABI_VERSION (\d+)", text).group(1)) == _lib.ABI_VERSION
    assert int(re.search(r"#define HYOBFS_ERR_CLOSED \((-\d+)\)", text).group(1)) == _lib.HYOBFS_ERR_CLOSED
    from hysteria_amd.salamander import SalamanderObfuscator
    kernels = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"HYOBFS_KERNEL_(\w+) = (\d+)", text)}
    assert kernels == SalamanderObfuscator.KERNELS   # auto, wave, tile


def test_load_refuses_other_abi_version(tmp_path):
    """_lib.load() refuses a library built for another ABI version (struct layouts and
    enum values differ between versions, include/hyobfs.h)."""
    src = tmp_path / "old.c"
    names = [n for n in _lib.header_functions()]
    body = "\n".join(f"void {n}(void) {{}}" for n in names if n != "hyobfs_abi_version")
    src.write_text(body + "\nint hyobfs_abi_version(void) { return 1; }\n")
    so = tmp_path / "libold.so"
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    with pytest.raises(OSError, match="ABI version 1"):
        _lib.load(str(so))
