"""Why is the tile kernel slower per byte on big batches?  On an 8M x 1200 B batch (the
configs[3] per-GPU shard), time: one 8M launch; eight 1M launches over consecutive
sub-ranges; 1M launches over the first / the last sub-range only.  Same buffers, same
process, medians of interleaved rounds."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hysteria_amd  # noqa: E402

L, S = 1200, 1 << 20
NS = int(sys.argv[1]) if len(sys.argv) > 1 else 8
P = NS * S
dev = torch.device("cuda:0")
inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(inp, P * L, 1, 0)
salts = torch.empty(P, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, P, 2, 0)
wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)


def sub(i, n=S):
    return lambda: o.obfuscate_batch(inp[i * S * L:], n, in_stride=L, len_uniform=L, salts=salts[i * S:],
                                     out=wire[i * S * (L + 8):], out_stride=L + 8)


cases = {
    f"one launch of {NS}M": ([sub(0, P)], P),
    f"{NS} launches of 1M, consecutive": ([sub(i) for i in range(NS)], P),
    "1M launches on the first 1M": ([sub(0)] * NS, P),
    "1M launches on the last 1M": ([sub(NS - 1)] * NS, P),
}
res = {k: [] for k in cases}
for r in range(7):
    for k, (fns, n) in cases.items():
        for f in fns:
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            for f in fns:
                f()
        e1.record()
        torch.cuda.synchronize()
        if r:
            res[k].append(e0.elapsed_time(e1) / 3)
for k, (fns, n) in cases.items():
    ms = statistics.median(res[k])
    gbs = n * (2 * L + 16) / (ms * 1e-3) / 1e9
    print(f"{k:40s} {ms:8.4f} ms  {gbs:7.1f} GB/s  ({gbs / 80:5.1f} % of 8 TB/s)")
