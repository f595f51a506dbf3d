"""In-process interleaved A/B of kernel variants (methodology rule: one process,
interleaved rounds).  Loads every library given (ctypes, separate handles),
prepares the uniform 1M x 1200 workload once, and times obfuscate/deobfuscate
launches of each variant round-robin.  Prints median/min per variant."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hysteria_amd import _lib  # noqa: E402

# each argument: path/to/lib.so[:kernel[:VAR=value,...]]  (kernel = auto|wave|persistent|uniform|stream|pipe;
# the variables are set for that variant's launches only: per-launch knobs such as HYOBFS_PERSIST_ORDER)
KERNELS = {"auto": 0, "wave": 1, "persistent": 2, "uniform": 3, "stream": 4, "pipe": 5, "flat": 6}
specs = [a.split(":") for a in (sys.argv[1:] or ["hysteria_amd/libhyobfs.so"])]
libs = [x[0] for x in specs]
P, L = 1 << 20, int(os.environ.get("AB_LEN", "1200"))
workload = os.environ.get("AB_WORKLOAD", "uniform")
dev = torch.device("cuda:0")
main = _lib.load(os.path.abspath(libs[0]))
handles = []
for spec in specs:
    path = spec[0]
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.hyobfs_salamander_new.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p)]
    lib.hyobfs_salamander_obfuscate_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(_lib.HyobfsBatch), ctypes.c_void_p]
    lib.hyobfs_salamander_deobfuscate_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(_lib.HyobfsBatch), ctypes.c_void_p]
    h = ctypes.c_void_p()
    psk = b"average_password"
    assert lib.hyobfs_salamander_new(psk, len(psk), 0, ctypes.byref(h)) == 0
    kern = spec[1] if len(spec) > 1 else "auto"
    assert lib.hyobfs_salamander_set_kernel(h, KERNELS[kern]) == 0
    env = dict(kv.split("=", 1) for kv in spec[2].split(",")) if len(spec) > 2 else {}
    name = os.path.basename(path).replace("libhyobfs_", "").replace(".so", "") + ":" + kern
    name += (":" + ",".join(f"{k}={v}" for k, v in env.items())) if env else ""
    handles.append((name, lib, h, env))
ENV_KEYS = {k for x in handles for k in x[3]}


def use_env(env):
    for k in ENV_KEYS:
        os.environ.pop(k, None)
    os.environ.update(env)

if workload == "uniform":
    inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
    main.hyobfs_synth_stream(inp.data_ptr(), P * L, 1, 0, None)
    salts = torch.empty(P, dtype=torch.int64, device=dev)
    main.hyobfs_synth_u64(salts.data_ptr(), P, 2, 0, None)
    wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
    back = torch.empty(P * L, dtype=torch.uint8, device=dev)
    bo = _lib.HyobfsBatch(n=P, in_=inp.data_ptr(), in_stride=L, len_uniform=L, salts=salts.data_ptr(),
                          out=wire.data_ptr(), out_cap=P * (L + 8), out_stride=L + 8)
    bd = _lib.HyobfsBatch(n=P, in_=wire.data_ptr(), in_stride=L + 8, len_uniform=L + 8, out=back.data_ptr(),
                          out_cap=P * L, out_stride=L)
    obf_bytes, deobf_bytes = P * (2 * L + 16), P * (2 * L + 8)
else:
    P = 1 << 22
    lens = torch.empty(P, dtype=torch.int32, device=dev)
    main.hyobfs_synth_bimodal_lengths(lens.data_ptr(), P, 3, 0, None)
    in_off = torch.zeros(P, dtype=torch.int64, device=dev)
    in_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
    total_in = int(lens.to(torch.int64).sum())
    inp = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    main.hyobfs_synth_stream(inp.data_ptr(), total_in, 1, 0, None)
    salts = torch.empty(P, dtype=torch.int64, device=dev)
    main.hyobfs_synth_u64(salts.data_ptr(), P, 2, 0, None)
    cap = total_in + 8 * P
    wire = torch.empty(cap, dtype=torch.uint8, device=dev)
    out_off = torch.empty(P, dtype=torch.int64, device=dev)
    out_len = torch.empty(P, dtype=torch.int32, device=dev)
    back = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    ws = torch.empty(main.hyobfs_batch_workspace_size(P), dtype=torch.uint8, device=dev)
    bo = _lib.HyobfsBatch(n=P, in_=inp.data_ptr(), in_off=in_off.data_ptr(), in_len=lens.data_ptr(),
                          salts=salts.data_ptr(), out=wire.data_ptr(), out_cap=cap, out_off=out_off.data_ptr(),
                          out_len=out_len.data_ptr(), workspace=ws.data_ptr(), workspace_bytes=ws.numel())
    bd = _lib.HyobfsBatch(n=P, in_=wire.data_ptr(), in_off=out_off.data_ptr(), in_len=out_len.data_ptr(),
                          out=back.data_ptr(), out_cap=total_in, workspace=ws.data_ptr(), workspace_bytes=ws.numel())
    obf_bytes, deobf_bytes = 2 * total_in + 16 * P, 2 * total_in + 8 * P

K = int(os.environ.get("AB_STEPS", "10"))
R = int(os.environ.get("AB_ROUNDS", "6"))
res = {name: {"obf": [], "deobf": []} for name, _, _, _ in handles}
# every variant's wire must equal the first one's before timing
ref = None
for name, lib, h, env in handles:
    use_env(env)
    wire.zero_()
    lib.hyobfs_salamander_obfuscate_batch(h, ctypes.byref(bo), None)
    torch.cuda.synchronize()
    if ref is None:
        ref = wire.clone()
    assert torch.equal(wire, ref), f"{name}: wire differs from {handles[0][0]}"
del ref
print("wire identical across variants")
for r in range(R + 1):
    for name, lib, h, env in handles:
        use_env(env)
        for kind, fn, b in (("obf", lib.hyobfs_salamander_obfuscate_batch, bo),
                            ("deobf", lib.hyobfs_salamander_deobfuscate_batch, bd)):
            fn(h, ctypes.byref(b), None)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                fn(h, ctypes.byref(b), None)
            e1.record()
            torch.cuda.synchronize()
            if r:   # round 0 = warmup
                res[name][kind].append(e0.elapsed_time(e1) / K)
for name, d in res.items():
    mo, md = statistics.median(d["obf"]), statistics.median(d["deobf"])
    print(f"{name:28s} obf {mo:.4f} ms ({obf_bytes / mo / 1e6:7.1f} GB/s, min {min(d['obf']):.4f})  "
          f"deobf {md:.4f} ms ({deobf_bytes / md / 1e6:7.1f} GB/s, min {min(d['deobf']):.4f})")
