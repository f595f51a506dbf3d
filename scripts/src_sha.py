"""sha256 over the kernel sources (hysteria_amd/csrc: *.h, *.hip, *.cpp, Makefile),
16 hex digits.  The Makefile compiles it into libhyobfs.so (hyobfs_build_id());
bench.py compares it with the loaded library's id and keys the committed PMC
traffic figures (profiles/pmc_traffic.json) by it."""
import glob
import hashlib
import os

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hysteria_amd", "csrc")


def src_sha(csrc: str = CSRC) -> str:
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(csrc, "*"))):
        if os.path.isfile(p) and p.endswith((".h", ".hip", ".cpp", "Makefile")):
            h.update(os.path.basename(p).encode())
            h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_sha())
