"""In-process A/B of library BUILDS (compile-time variants) and kernel choices on
one workload: every variant runs in the same process on the same buffers, in
interleaved rounds, medians reported -- buffer placement, which moves a
streaming kernel by up to +-5 % between processes, is shared.

  AB_LIBS="main=hysteria_amd/libhyobfs.so,align!=build_variants/libhyobfs_align.so" \
      python scripts/ab_variants.py [kernels=tile] [L=1200] [P=1048576]

A name ending in "!" is an ablation build (wrong output): its wire is not checked.
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hysteria_amd  # noqa: E402

kernels = (sys.argv[1] if len(sys.argv) > 1 else "tile").split(",")
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
P = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
K = int(os.environ.get("AB_STEPS", "10"))
R = int(os.environ.get("AB_ROUNDS", "6"))
libs = [kv.split("=", 1) for kv in os.environ.get("AB_LIBS", "main=" + hysteria_amd._lib.LIB_PATH).split(",")]
dev = torch.device("cuda:0")
inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(inp, P * L, 1, 0)
salts = torch.empty(P, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, P, 2, 0)
wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
back = torch.empty(P * L, dtype=torch.uint8, device=dev)
obf_bytes, deobf_bytes = P * (2 * L + 16), P * (2 * L + 8)
ctxs = {}
for name, path in libs:
    for k in kernels:
        o = hysteria_amd.SalamanderObfuscator(b"average_password", 0, lib_path=os.path.abspath(path))
        o.set_kernel(k)
        ctxs[f"{name}/{k}"] = (o, name.endswith("!"))


def ob(o):
    return lambda: o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)


def de(o):
    return lambda: o.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)


ref = None
for name, (o, nocheck) in ctxs.items():   # every checked variant's output must agree before timing
    if nocheck:
        continue
    ob(o)()
    de(o)()
    torch.cuda.synchronize()
    assert torch.equal(back, inp), f"{name}: round trip"
    h = wire[: 1 << 26].clone()
    if ref is None:
        ref = h
    assert torch.equal(h, ref), f"{name}: wire differs"
cases = [("copy", "obf", lambda: wire[:P * L].copy_(inp), 2 * P * L)]
for name, (o, _) in ctxs.items():
    cases += [(name, "obf", ob(o), obf_bytes), (name, "deobf", de(o), deobf_bytes)]
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
    print(f"{k:22s} {d:6s} {med:.4f} ms  {nbytes / med / 1e6:7.1f} GB/s  ({nbytes / med / 1e6 / 8000 * 100:5.1f} % of 8 TB/s)"
          f"  min {min(v):.4f}")
