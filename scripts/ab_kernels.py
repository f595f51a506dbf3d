"""In-process interleaved A/B of the batch kernels on one workload (methodology:
one process, interleaved rounds, medians).  One context per kernel choice;
a torch device copy of the same bytes is the calibration line.

  python scripts/ab_kernels.py [kernels=wave,uniform] [L=1200] [P=1048576]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hysteria_amd  # noqa: E402

kernels = (sys.argv[1] if len(sys.argv) > 1 else "wave,uniform").split(",")
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
P = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
K = int(os.environ.get("AB_STEPS", "10"))
R = int(os.environ.get("AB_ROUNDS", "6"))
dev = torch.device("cuda:0")
inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(inp, P * L, 1, 0)
salts = torch.empty(P, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, P, 2, 0)
wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
back = torch.empty(P * L, dtype=torch.uint8, device=dev)
ctxs = {}
for k in kernels:
    o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)
    o.set_kernel(k)
    ctxs[k] = o
obf_bytes, deobf_bytes = P * (2 * L + 16), P * (2 * L + 8)


def ob(o):
    return lambda: o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)


def de(o):
    return lambda: o.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)


keys = torch.empty(32 * P, dtype=torch.uint8, device=dev)
o0 = next(iter(ctxs.values()))
cases = [("copy", "obf", lambda: wire[:P * L].copy_(inp), 2 * P * L),
         ("keys_only", "obf", lambda: o0.keys_batch(salts, keys, P), 40 * P)]
for k, o in ctxs.items():
    cases += [(k, "obf", ob(o), obf_bytes), (k, "deobf", de(o), deobf_bytes)]
# every kernel's output must agree before timing
ref = None
for k, o in ({} if os.environ.get("AB_NOCHECK") else ctxs).items():   # AB_NOCHECK: ablation builds (wrong output)
    ob(o)()
    de(o)()
    torch.cuda.synchronize()
    assert torch.equal(back, inp), f"{k}: round trip"
    h = wire[: 1 << 26].clone()
    if ref is None:
        ref = h
    assert torch.equal(h, ref), f"{k}: wire differs from {kernels[0]}"
res = {(k, d): [] for k, d, _, _ in cases}
for r in range(R + 1):
    for k, d, fn, nbytes in cases:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            res[(k, d)].append(e0.elapsed_time(e1) / K)
print(f"P={P} L={L} steps={K} rounds={R}")
for k, d, _, nbytes in cases:
    v = res[(k, d)]
    med = statistics.median(v)
    print(f"{k:12s} {d:6s} {med:.4f} ms  {nbytes / med / 1e6:7.1f} GB/s  ({nbytes / med / 1e6 / 8000 * 100:5.1f} % of 8 TB/s)"
          f"  min {min(v):.4f}")
