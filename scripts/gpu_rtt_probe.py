"""Latency of one small synchronous GPU call (hyobfs_salamander_obfuscate: H2D, one batch
kernel, D2H) when calls are spaced out: are the coalescing connection's millisecond
tails the GPU's own wake-up after idle gaps?  Prints percentiles per gap (JSON)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import hysteria_amd

o = hysteria_amd.SalamanderObfuscator(b"probe_password", 0)
p = bytes(1200)
out = bytearray(1208)
res = {}
for gap_us in (0, 20, 100, 500, 2000):
    lat = []
    n = 3000 if gap_us < 500 else 800
    for i in range(n):
        if gap_us:
            t_end = time.perf_counter() + gap_us * 1e-6
            while time.perf_counter() < t_end:
                pass
        t0 = time.perf_counter()
        o.obfuscate(p, out, salt=b"12345678")
        lat.append((time.perf_counter() - t0) * 1e6)
    a = np.array(lat[50:])
    res[gap_us] = {"p50_us": round(float(np.percentile(a, 50)), 1), "p99_us": round(float(np.percentile(a, 99)), 1),
                   "p999_us": round(float(np.percentile(a, 99.9)), 1), "max_us": round(float(a.max()), 1), "n": int(a.size)}
print(json.dumps(res))
