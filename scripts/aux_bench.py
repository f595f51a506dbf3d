"""Device rates of the §8(f) rows beside the headline path:

* Gecko: hyobfs_gecko_encode_batch over 262144 long-header messages of 1200 B
  (~1.2M frames, default 512..1200 band): frames/s and wire GB/s, keys kernel
  included; parse kernel over the same datagrams after deobfuscation.
* Realm: hyobfs_punch_match_batch, 1M received datagrams x 8 registered attempts.

Prints one JSON line.  Timing: HIP events around K launches after a warmup."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hysteria_amd  # noqa: E402
from hysteria_amd import gecko, realm  # noqa: E402

dev = torch.device("cuda:0")
K = 20


def timed(fn, warmup=20, rounds=5):
    """Steady state: `warmup` untimed calls first (the shader clock ramps up over the first
    launches), then the median over `rounds` of K back-to-back calls."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(rounds):
        e0.record()
        for _ in range(K):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / K)
    return sorted(ts)[len(ts) // 2]


def d(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)


res = {}
# ---- Gecko encode / parse
M, L = 262144, 1200
rng = np.random.default_rng(1)
fr, off, total = gecko.plan_fragments(np.full(M, L), rand32=lambda k: rng.integers(0, 2**32, k, dtype=np.uint64))
nf = len(fr)
msg = torch.empty(M * L, dtype=torch.uint8, device=dev)
hysteria_amd.synth_stream(msg, M * L, 1, 0)
salts = torch.empty(nf, dtype=torch.int64, device=dev)
hysteria_amd.synth_u64(salts, nf, 2, 0)
out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)
dfr, doff = d(fr), d(off)
ms = timed(lambda: gecko.encode_batch(o, msg=msg, frames=dfr, salts=salts, pad_key=bytes(range(1, 33)), pad_nonce=bytes(12), out=out, out_off=doff,
                                      n=nf))
alg = M * L + total   # chunk bytes read + wire bytes written (pad generated on device)
res["gecko_encode"] = {"messages": M, "msg_len": L, "frames": nf, "wire_bytes": total, "ms": round(ms, 4),
                       "frames_per_s": round(nf / ms * 1e3), "alg_GBs": round(alg / ms / 1e6, 1),
                       "frac_of_8TBs": round(alg / ms / 1e6 / 8000, 4)}
wl = torch.from_numpy((13 + fr["chunk_len"].astype(np.uint32) + fr["pad_len"]).astype(np.int32)).to(dev)
plain = torch.empty(total + 16, dtype=torch.uint8, device=dev)
poff = torch.empty(nf, dtype=torch.int64, device=dev)
plen = torch.empty(nf, dtype=torch.int32, device=dev)
ws2 = torch.empty(hysteria_amd.workspace_size(nf), dtype=torch.uint8, device=dev)
o.deobfuscate_batch(out, nf, in_off=doff.view(torch.int64), in_len=wl, out=plain, out_cap=total, out_off=poff,
                    out_len=plen, workspace=ws2, workspace_bytes=ws2.numel())
parsed = torch.empty(nf * 16, dtype=torch.uint8, device=dev)
ms = timed(lambda: gecko.parse_batch(plain, poff, plen, nf, parsed))
pr = parsed.cpu().numpy().view(gecko.PARSED_DTYPE)
res["gecko_parse"] = {"datagrams": nf, "ms": round(ms, 4), "datagrams_per_s": round(nf / ms * 1e3),
                      "all_fragments": bool((pr["status"] == gecko.FRAGMENT).all())}
o.close()
del msg, out, plain
# ---- realm punch matcher
N, A = 1 << 20, 8
metas = [realm.new_punch_metadata() for _ in range(A)]
mt = realm.PunchMatcher(metas)
pk = [realm.encode_punch_packet(1 + (i & 1), metas[i % A]) for i in range(4096)]
lens = np.array([len(x) for x in pk], np.uint32)
buf = np.frombuffer(b"".join(pk), np.uint8)
offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
idx = np.arange(N) % len(pk)          # 1M datagrams cycling over 4096 distinct packets
dbuf, doffs, dlens = d(buf), d(offs[idx]), d(lens[idx])
match = torch.empty(N, dtype=torch.int32, device=dev)
datt = d(mt.attempts)
ms = timed(lambda: mt.match_batch(dbuf, doffs, dlens, N, match, attempts=datt))
hm = match.cpu().numpy()
res["punch_match"] = {"datagrams": N, "attempts": A, "ms": round(ms, 4), "datagrams_per_s": round(N / ms * 1e3),
                      "sha256_per_s": round(float((idx % A + 1).sum()) / ms * 1e3),   # attempts tried until the match
                      "all_matched_expected": bool((hm == (idx % A)).all())}
print(json.dumps(res))
