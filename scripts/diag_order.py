"""Diagnostic: obfuscate/deobfuscate launch times (HIP events, 20 launches each)
in different orders and with different buffers, bench.py's setup (1M x 1200)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hysteria_amd  # noqa: E402

dev = torch.device("cuda:0")
P, L = 1 << 20, 1200
o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)
inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(inp, P * L, 1, 0)
salts = torch.empty(P, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, P, 2, 0)
wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
wire2 = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
back = torch.empty(P * L, dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream()


def obf(out=wire, src=inp):
    o.obfuscate_batch(src, P, in_stride=L, len_uniform=L, salts=salts, out=out, out_stride=L + 8)


def deobf(src=wire, out=back):
    o.deobfuscate_batch(src, P, in_stride=L + 8, len_uniform=L + 8, out=out, out_stride=L)


def t(fn, k=20, w=5):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / k, 4)


res = []
res.append(("obf", t(obf)))
res.append(("deobf", t(deobf)))
res.append(("obf again", t(obf)))
res.append(("deobf again", t(deobf)))
res.append(("obf -> wire2", t(lambda: obf(out=wire2))))
res.append(("deobf wire2 -> back", t(lambda: deobf(src=wire2))))
res.append(("obf from back (same bytes)", t(lambda: obf(src=back))))
res.append(("alternating obf,deobf pairs /2", round(t(lambda: (obf(), deobf())) / 2, 4)))
res.append(("obf null stream", t(lambda: o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire,
                                                          out_stride=L + 8, stream=0))))
res.append(("deobf null stream", t(lambda: o.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back,
                                                              out_stride=L, stream=0))))
for k, v in res:
    print(f"{k:34s} {v:.4f} ms")
