"""Where a library build's configs[2] wire differs from the shipped build's (a store
cache-policy experiment, tools/ab_patches/stream_store_ntsc1.patch): both builds run the
same contiguous bimodal batch under each kernel; for every kernel the number of differing
bytes and, for the first differing 16-byte chunks, their offset in the 16 KiB flat tile
and in the 128-byte line, and whether a datagram edge (salt or payload boundary) lies in
the chunk's line.  Prints one JSON object.

  python scripts/diag_store_policy.py ab_builds/libhyobfs_X.so [P=65536]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hysteria_amd  # noqa: E402

variant = os.path.abspath(sys.argv[1])
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
dev = torch.device("cuda:0")
lens = torch.empty(P, dtype=torch.int32, device=dev)
hysteria_amd.synth_bimodal_lengths(lens, P, 3, 0)
total_in = int(lens.to(torch.int64).sum())
inp = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(inp, total_in, 1, 0)
salts = torch.empty(P, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, P, 2, 0)
cap = total_in + 8 * P
SO = hysteria_amd.SalamanderObfuscator
nws = 4 * SO.workspace_bytes(inp=inp, n=P, in_len=lens, out=torch.empty(16, dtype=torch.uint8, device=dev),
                             out_cap=cap) + 40 * P + (1 << 20)
ws = torch.empty(nws, dtype=torch.uint8, device=dev)
out_len = torch.empty(P, dtype=torch.int32, device=dev)
out_off = torch.empty(P, dtype=torch.int64, device=dev)


def wire(lib, kernel):
    o = SO(b"average_password", 0, lib_path=lib)
    o.set_kernel(kernel)
    w = torch.full((cap + 256,), 0xA5, dtype=torch.uint8, device=dev)
    o.obfuscate_batch(inp, P, in_len=lens, salts=salts, out=w, out_cap=cap, out_off=out_off, out_len=out_len,
                      workspace=ws, workspace_bytes=ws.numel())
    torch.cuda.synchronize()
    return w


res = {"P": P, "variant": os.path.basename(variant)}
for kernel in ("wave", "flat"):
    a = wire(hysteria_amd._lib.LIB_PATH, kernel)
    b = wire(variant, kernel)
    d = torch.cat([((a[i:i + (1 << 28)] != b[i:i + (1 << 28)]).nonzero().flatten() + i)
                   for i in range(0, a.numel(), 1 << 28)])
    r = {"diff_bytes": int(d.numel())}
    if d.numel():
        offs = out_off.cpu().tolist()
        edges = sorted(set(offs) | {x + 8 for x in offs})   # salt starts and payload starts
        import bisect
        chunks = sorted(set((d // 16).cpu().tolist()))
        r["diff_chunks"] = len(chunks)
        ex = []
        for c in chunks[:12]:
            a0 = 16 * c
            line = a0 & ~127
            i = bisect.bisect_left(edges, line)
            edge_in_line = i < len(edges) and edges[i] < line + 128
            ex.append({"chunk_off": a0, "in_tile": a0 % 16384, "in_line": a0 % 128, "edge_in_line": edge_in_line,
                       "bytes": int(((d >= a0) & (d < a0 + 16)).sum())})
        r["first"] = ex
        lines = sorted(set((16 * c) & ~127 for c in chunks))
        with_edge = 0
        for line in lines:
            i = bisect.bisect_left(edges, line)
            with_edge += i < len(edges) and edges[i] < line + 128
        r["diff_lines"] = len(lines)
        r["diff_lines_with_edge"] = with_edge
    res[kernel] = r
print(json.dumps(res))
