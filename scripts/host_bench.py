"""Host-to-host rate (BASELINE configs[4], PCIe-inclusive): 1M x 1200 B datagrams
in host memory -> obfuscate through the H2D / kernel / D2H pipeline -> host.
Prints one JSON line; DESIGN.md quotes it.  Also measures the raw pinned copy
rates the pipeline is bounded by, one zero-copy batch call on mapped pinned buffers,
and checks the output digests (configs[1])."""
import hashlib, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, hysteria_amd
P, L = 1 << 20, 1200
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)
d_in = torch.empty(P * L, dtype=torch.uint8, device=dev); hysteria_amd.synth_stream(d_in, P * L, 1, 0)
d_s = torch.empty(P, dtype=torch.int64, device=dev); hysteria_amd.synth_u64(d_s, P, 2, 0)
h_in = d_in.cpu().pin_memory(); h_s = d_s.cpu()
h_out = torch.empty(P * (L + 8), dtype=torch.uint8).pin_memory()
del d_in
res = {"workload": f"{P} x {L} B datagrams, host memory in and out", "reps": reps}

def timeit(fn):
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]

for chunk in (16384, 65536, 262144):
    t = timeit(lambda: o.obfuscate_host(h_in, P, in_stride=L, len_uniform=L, salts=h_s, out=h_out,
                                        out_stride=L + 8, chunk=chunk))
    res[f"pinned_chunk{chunk}_GiBps"] = round(P * L / t / 2**30, 2)
    res[f"pinned_chunk{chunk}_ms"] = round(t * 1e3, 2)
want = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "tests/golden/batch_digests.json")))["config2_1M_x_1200"]["obf_sha256"]
res["digest_match"] = hashlib.sha256(h_out.numpy().tobytes()).hexdigest() == want
# zero-copy: one batch call whose input and output are mapped pinned host buffers
# (hyobfs_host_alloc: hipHostMallocMapped, device-accessible): the tile kernel reads
# and writes across PCIe in place, no staging copies
import ctypes
lib = hysteria_amd._lib.load()
z_in, z_out, z_s = lib.hyobfs_host_alloc(P * L), lib.hyobfs_host_alloc(P * (L + 8)), lib.hyobfs_host_alloc(P * 8)
if z_in and z_out and z_s:
    a_in = np.ctypeslib.as_array(ctypes.cast(z_in, ctypes.POINTER(ctypes.c_uint8)), (P * L,))
    a_out = np.ctypeslib.as_array(ctypes.cast(z_out, ctypes.POINTER(ctypes.c_uint8)), (P * (L + 8),))
    a_s = np.ctypeslib.as_array(ctypes.cast(z_s, ctypes.POINTER(ctypes.c_uint8)), (P * 8,))
    a_in[:] = h_in.numpy()
    a_s[:] = h_s.numpy().view(np.uint8)
    a_out[:] = 0
    st = torch.cuda.current_stream().cuda_stream
    t = timeit(lambda: o.obfuscate_batch(z_in, P, in_stride=L, len_uniform=L, salts=z_s, out=z_out,
                                         out_cap=P * (L + 8), out_stride=L + 8, stream=st))
    res["zerocopy_mapped_GiBps"] = round(P * L / t / 2**30, 2)
    res["zerocopy_mapped_ms"] = round(t * 1e3, 2)
    res["zerocopy_digest_match"] = hashlib.sha256(a_out.tobytes()).hexdigest() == want
    del a_in, a_out, a_s
for z in (z_in, z_out, z_s):
    lib.hyobfs_host_free(z)
# pageable host memory
p_in, p_out = h_in.numpy().copy(), np.empty(P * (L + 8), np.uint8)
t = timeit(lambda: o.obfuscate_host(p_in, P, in_stride=L, len_uniform=L, salts=h_s, out=p_out, out_stride=L + 8,
                                    chunk=65536))
res["pageable_chunk65536_GiBps"] = round(P * L / t / 2**30, 2)
# raw pinned copy rates (the bound): H2D of the input, D2H of the output, and both at once
d_a = torch.empty(P * L, dtype=torch.uint8, device=dev); d_b = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
t = timeit(lambda: d_a.copy_(h_in, non_blocking=True)); res["h2d_pinned_GBps"] = round(P * L / t / 1e9, 1)
t = timeit(lambda: h_out.copy_(d_b, non_blocking=True)); res["d2h_pinned_GBps"] = round(P * (L + 8) / t / 1e9, 1)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def both():
    with torch.cuda.stream(s1): d_a.copy_(h_in, non_blocking=True)
    with torch.cuda.stream(s2): h_out.copy_(d_b, non_blocking=True)
t = timeit(both); res["h2d_plus_d2h_concurrent_GBps_each"] = round(P * L / t / 1e9, 1)
print(json.dumps(res))
