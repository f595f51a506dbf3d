"""Host-to-host rate (BASELINE configs[4], PCIe-inclusive): 1M x 1200 B datagrams
in host memory -> obfuscate through the H2D / kernel / D2H pipeline -> host.
Prints one JSON line; DESIGN.md quotes it.  Also measures the raw pinned copy
rates the pipeline is bounded by, and checks the output digest (configs[1])."""
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
