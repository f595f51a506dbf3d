"""In-process A/B of library BUILDS (compile-time variants) and kernel choices on
one workload: every variant runs in the same process on the same buffers, in
interleaved rounds, medians reported -- buffer placement, which moves a
streaming kernel by up to +-5 % between processes, is shared.

  AB_LIBS="main=hysteria_amd/libhyobfs.so,align!=ab_builds/libhyobfs_align.so" \
      python scripts/ab_variants.py [kernels=tile] [L=1200] [P=1048576]

A name ending in "!" is an ablation build (wrong output): its wire is not checked.
AB_WORKLOAD=bimodal runs BASELINE configs[2] instead (P datagrams of the 40 % 64 B /
60 % 1350 B mix, default 4M, packed output).  Bimodal input is contiguous (in_off NULL,
as bench.py); a kernel name with "@off" passes explicit in_off / out_off arrays instead.
AB_LEN_MAP="1350:1344" replaces lengths (alignment studies).  The first variant of a run
measures ~1.5 % slow (profiles/r04_ab_wave_wu_order_control.txt): put a throw-away
copy of a build first when differences of that size matter.
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
WL = os.environ.get("AB_WORKLOAD", "uniform")
salts = None
if WL == "bimodal":
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 22
    lens = torch.empty(P, dtype=torch.int32, device=dev)
    hysteria_amd.synth_bimodal_lengths(lens, P, 3, 0)
    for kv in filter(None, os.environ.get("AB_LEN_MAP", "").split(",")):   # e.g. 1350:1352 (alignment study)
        x, y = (int(v) for v in kv.split(":"))
        lens[lens == x] = y
    in_off = torch.zeros(P, dtype=torch.int64, device=dev)
    in_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
    total_in = int(lens.to(torch.int64).sum())
    inp = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    hysteria_amd.synth_stream(inp, total_in, 1, 0)
    salts = torch.empty(P, dtype=torch.int64, device=dev)
    hysteria_amd.synth_u64(salts, P, 2, 0)
    cap = total_in + 8 * P
    wire = torch.empty(cap, dtype=torch.uint8, device=dev)
    out_off = torch.empty(P, dtype=torch.int64, device=dev)
    out_len = torch.empty(P, dtype=torch.int32, device=dev)
    back = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    SO = hysteria_amd.SalamanderObfuscator
    nws = max(hysteria_amd.workspace_size(P), SO.workspace_bytes(inp=inp, n=P, in_len=lens, out=wire, out_cap=cap),
              SO.workspace_bytes(inp=wire, n=P, in_len=out_len, out=back, out_cap=total_in))
    ws = torch.empty(4 * nws + 40 * P, dtype=torch.uint8, device=dev)   # room for builds with smaller tiles or key arrays
    obf_bytes, deobf_bytes = 2 * total_in + 16 * P, 2 * total_in + 8 * P
    PL = total_in
else:
    inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
    hysteria_amd.synth_stream(inp, P * L, 1, 0)
    salts = torch.empty(P, dtype=torch.int64, device=dev)
    hysteria_amd.synth_u64(salts, P, 2, 0)
    wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
    back = torch.empty(P * L, dtype=torch.uint8, device=dev)
    obf_bytes, deobf_bytes = P * (2 * L + 16), P * (2 * L + 8)
    PL = P * L
ctxs = {}
for name, path in libs:
    for k in kernels:
        o = hysteria_amd.SalamanderObfuscator(b"average_password", 0, lib_path=os.path.abspath(path))
        o.set_kernel(k.split("@")[0])
        o.ab_offsets = k.endswith("@off")
        ctxs[f"{name}/{k}"] = (o, name.endswith("!"))


def ob(o):
    if WL == "bimodal":
        off = dict(in_off=in_off) if o.ab_offsets else {}
        return lambda: o.obfuscate_batch(inp, P, in_len=lens, salts=salts, out=wire, out_cap=cap, out_off=out_off,
                                         out_len=out_len, workspace=ws, workspace_bytes=ws.numel(), **off)
    return lambda: o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)


def de(o):
    if WL == "bimodal":
        off = dict(in_off=out_off) if o.ab_offsets else {}
        return lambda: o.deobfuscate_batch(wire, P, in_len=out_len, out=back, out_cap=total_in,
                                           workspace=ws, workspace_bytes=ws.numel(), **off)
    return lambda: o.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)


ref = None
for name, (o, nocheck) in ctxs.items():   # every checked variant's output must agree before timing
    if nocheck:
        continue
    ob(o)()
    de(o)()
    torch.cuda.synchronize()
    assert torch.equal(back[:PL], inp[:PL]), f"{name}: round trip"
    h = wire[: 1 << 26].clone()
    if ref is None:
        ref = h
    assert torch.equal(h, ref), f"{name}: wire differs"
cases = [("copy", "obf", lambda: wire[:PL].copy_(inp[:PL]), 2 * PL)]
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
print(f"workload={WL} P={P} L={L if WL != 'bimodal' else 'bimodal'} steps={K} rounds={R}")
for k, d, _, nbytes in cases:
    v = res[(k, d)]
    med = statistics.median(v)
    print(f"{k:22s} {d:6s} {med:.4f} ms  {nbytes / med / 1e6:7.1f} GB/s  ({nbytes / med / 1e6 / 8000 * 100:5.1f} % of 8 TB/s)"
          f"  min {min(v):.4f}")
