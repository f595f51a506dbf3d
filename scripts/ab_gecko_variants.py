"""In-process A/B of library builds on the Gecko encode (scripts/aux_bench.py's
workload: 262144 messages of 1200 B, default 512..1200 band, ~1.31 M frames).
Every build runs in the same process on the same buffers, interleaved rounds,
medians reported (placement moves a streaming kernel by +-5 %
between processes).

  AB_LIBS="main=hysteria_amd/libhyobfs.so,wave=ab_builds/libhyobfs_gkwave.so,nopad!=..." \
      python scripts/ab_gecko_variants.py

A name ending in "!" is an ablation build (wrong output): its wire is not checked
against the first build's."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hysteria_amd  # noqa: E402
from hysteria_amd import gecko  # noqa: E402

K = int(os.environ.get("AB_STEPS", "10"))
R = int(os.environ.get("AB_ROUNDS", "6"))
libs = [kv.split("=", 1) for kv in os.environ.get("AB_LIBS", "main=" + hysteria_amd._lib.LIB_PATH).split(",")]
dev = torch.device("cuda:0")
M, L = int(os.environ.get("AB_MSGS", "262144")), 1200
rng = np.random.default_rng(1)
fr, off, total = gecko.plan_fragments(np.full(M, L), rand32=lambda k: rng.integers(0, 2**32, k, dtype=np.uint64))
nf = len(fr)
msg = torch.empty(M * L, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(msg, M * L, 1, 0)
salts = torch.empty(nf, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, nf, 2, 0)
out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
dfr = torch.from_numpy(fr.view(np.uint8)).to(dev)
doff = torch.from_numpy(off.view(np.uint8)).to(dev)
alg = M * L + total
modes = ["wave"]
obs = {}
for name, path in libs:
    for m in modes:
        o = hysteria_amd.SalamanderObfuscator(b"average_password", 0, lib_path=path)
        obs[f"{name}/{m}"] = o
libs = [(f"{name}/{m}", path) for name, path in libs for m in modes]


def run(name):
    gecko.encode_batch(obs[name], msg=msg, frames=dfr, salts=salts, pad_key=bytes(range(32)), pad_nonce=bytes(12),
                       out=out, out_off=doff, n=nf)


ref = None
for name, _ in libs:
    out.fill_(0)
    run(name)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    elif "!" not in name:
        assert torch.equal(out, ref), f"{name}: wire differs from {libs[0][0]}"
times = {name: [] for name, _ in libs}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(R):
    for name, _ in libs:
        run(name)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(K):
            run(name)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / K)
print(f"gecko encode: {M} x {L} B messages, {nf} frames, {total} wire bytes, steps={K} rounds={R}")
for name, _ in libs:
    ms = statistics.median(times[name])
    print(f"{name:14s} {ms:.4f} ms  {alg / ms / 1e6:7.1f} GB/s ({alg / ms / 1e6 / 8000 * 100:5.1f} % of 8 TB/s)  "
          f"min {min(times[name]):.4f}")
for o in set(obs.values()):
    o.close()
