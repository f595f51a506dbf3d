"""Minimal driver for rocprofv3 counter passes: K obfuscate + K deobfuscate launches
of the uniform 1M x 1200 B batch (BASELINE configs[1]), or of the 4M bimodal
batch (configs[2], packed output) with 'bimodal'; 'uniform8m': the 8M x 1200 B shard of
configs[3] (one rank at N > 1) (contiguous input, as bench.py) or
'bimodal_off' (explicit offsets); 'bimodal_alt': 20 warm-up obfuscate launches, then
K of each layout alternating (obfuscate only).  Optional 3rd argument: the context's
kernel (auto|wave|tile).  PROF_PRETOUCH=1 writes zeros over every output buffer (and
the workspace) before the first launch (the first-touch study).
'uniform_rev': the uniform batch with the K deobfuscate launches first (a wire made by
one obfuscate launch), then the K obfuscate launches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, hysteria_amd
wl = sys.argv[1] if len(sys.argv) > 1 else "uniform"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
kern = sys.argv[3] if len(sys.argv) > 3 else "auto"
if wl not in ("uniform", "uniform8m", "uniform_rev", "bimodal", "bimodal_off", "bimodal_alt"):
    sys.exit(f"unknown workload {wl!r}: uniform | uniform8m | uniform_rev | bimodal | bimodal_off | bimodal_alt")
dev = torch.device("cuda:0")
o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)
o.set_kernel(kern)
if wl == "uniform_rev":
    P, L = 1 << 20, 1200
    inp = torch.empty(P * L, dtype=torch.uint8, device=dev); hysteria_amd.synth_stream(inp, P * L, 1, 0)
    salts = torch.empty(P, dtype=torch.int64, device=dev); hysteria_amd.synth_u64(salts, P, 2, 0)
    wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev); back = torch.empty(P * L, dtype=torch.uint8, device=dev)
    o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)
    for _ in range(K):
        o.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)
    for _ in range(K):
        o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)
elif wl in ("uniform", "uniform8m"):   # uniform8m: the 8M-datagram shard a rank runs at N > 1
    P, L = (1 << 20) if wl == "uniform" else (1 << 23), 1200
    inp = torch.empty(P * L, dtype=torch.uint8, device=dev); hysteria_amd.synth_stream(inp, P * L, 1, 0)
    salts = torch.empty(P, dtype=torch.int64, device=dev); hysteria_amd.synth_u64(salts, P, 2, 0)
    wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev); back = torch.empty(P * L, dtype=torch.uint8, device=dev)
    for _ in range(K):
        o.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)
    for _ in range(K):
        o.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)
else:
    P = 1 << 22
    lens = torch.empty(P, dtype=torch.int32, device=dev); hysteria_amd.synth_bimodal_lengths(lens, P, 3, 0)
    in_off = None
    if wl in ("bimodal_off", "bimodal_alt"):
        in_off = torch.zeros(P, dtype=torch.int64, device=dev); in_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
    total_in = int(lens.to(torch.int64).sum())
    inp = torch.empty(total_in + 16, dtype=torch.uint8, device=dev); hysteria_amd.synth_stream(inp, total_in, 1, 0)
    salts = torch.empty(P, dtype=torch.int64, device=dev); hysteria_amd.synth_u64(salts, P, 2, 0)
    cap = total_in + 8 * P
    wire = torch.empty(cap, dtype=torch.uint8, device=dev)
    out_off = torch.empty(P, dtype=torch.int64, device=dev)
    out_len = torch.empty(P, dtype=torch.int32, device=dev)
    back = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    nws = max(o.workspace_bytes(inp=inp, n=P, in_off=in_off, in_len=lens, out=wire, out_cap=cap),
              o.workspace_bytes(inp=inp, n=P, in_len=lens, out=wire, out_cap=cap),   # bimodal_alt: both layouts
              o.workspace_bytes(inp=wire, n=P, in_off=None if in_off is None else out_off, in_len=out_len, out=back, out_cap=total_in))
    ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=dev)
    if os.environ.get("PROF_PRETOUCH") == "1":
        for t in (wire, out_off, out_len, back, ws):
            t.zero_()
        torch.cuda.synchronize()
    if wl == "bimodal_alt":   # 20 warm-up launches, then contiguous and explicit offsets alternating
        for i in range(20 + 2 * K):
            o.obfuscate_batch(inp, P, in_off=in_off if i % 2 else None, in_len=lens, salts=salts, out=wire,
                              out_cap=cap, out_off=out_off, out_len=out_len, workspace=ws, workspace_bytes=ws.numel())
        K = 0
    for _ in range(K):
        o.obfuscate_batch(inp, P, in_off=in_off, in_len=lens, salts=salts, out=wire, out_cap=cap,
                          out_off=out_off, out_len=out_len, workspace=ws, workspace_bytes=ws.numel())
    for _ in range(K):
        o.deobfuscate_batch(wire, P, in_off=None if in_off is None else out_off, in_len=out_len, out=back, out_cap=total_in,
                            workspace=ws, workspace_bytes=ws.numel())
torch.cuda.synchronize()
print("done", wl, K, kern)
