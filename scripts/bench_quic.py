"""Throughput of the QUIC Initial sniff path (hyobfs_quic_read_crypto_payload_batch)
on one GPU: N client Initial packets of ~1200 bytes (64 oracle-made templates,
V1 and V2, split CRYPTO frames + PADDING), device resident.  Prints one JSON
line: packets/s, packet GB/s, per-kernel split (HIP events), and the pure-Python
oracle's rate on a few packets for scale.

  python scripts/bench_quic.py [--n 262144] [--steps 20] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def templates(k=64, seed=11):
    import quic_cases as qc
    from oracle import quic_ref as ref
    rng = np.random.default_rng(seed)
    out = []
    for t in range(k):
        ch = qc.client_hello_like(rng, int(rng.integers(250, 600)))
        cut = int(rng.integers(1, len(ch)))
        frames = qc._crypto(cut, ch[cut:]) + b"\x00" * int(rng.integers(0, 40)) + qc._crypto(0, ch[:cut])
        dcid = rng.integers(0, 256, int(rng.integers(8, 21)), dtype=np.uint8).tobytes()
        version = ref.V2 if t % 2 else ref.V1
        pad = 1200 - (len(frames) + 30 + len(dcid))
        out.append(ref.client_initial(dcid, b"", version, b"", 2, 4, frames + b"\x00" * max(pad, 0)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import torch
    from hysteria_amd import quic
    from oracle import quic_ref as ref
    dev = torch.device("cuda", 0)
    temps = templates()
    n = args.n
    pick = np.random.default_rng(5).integers(0, len(temps), n)
    lens = np.array([len(temps[i]) for i in pick], np.uint32)
    off = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], out=off[1:])
    src = torch.from_numpy(np.concatenate([np.frombuffer(temps[i], np.uint8) for i in pick] +
                                          [np.zeros(64, np.uint8)])).to(dev)
    buf = torch.empty_like(src)
    d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens).to(dev)
    cap = 1024
    d_out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(np.arange(n, dtype=np.uint64) * np.uint64(cap)).to(dev)
    d_cap = torch.full((n,), cap, dtype=torch.int32, device=dev)
    d_res = torch.empty(n * 24, dtype=torch.uint8, device=dev)
    ws = torch.empty(quic.workspace_size(n), dtype=torch.uint8, device=dev)

    def step():
        buf.copy_(src)   # the path works in place: restore the protected packets (timed separately)
        quic.read_crypto_payload_batch(buf, d_off, d_len, n, d_out, d_oo, d_cap, d_res, ws)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    copy_ms = total_ms = 0.0
    for _ in range(args.steps):
        e[0].record()
        buf.copy_(src)
        e[1].record()
        quic.read_crypto_payload_batch(buf, d_off, d_len, n, d_out, d_oo, d_cap, d_res, ws)
        e[2].record()
        torch.cuda.synchronize()
        copy_ms += e[0].elapsed_time(e[1])
        total_ms += e[1].elapsed_time(e[2])
    ms = total_ms / args.steps
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), quic.RESULT_DTYPE)
    assert (res["status"] == 0).all(), np.unique(res["status"])
    # CPU scale: the pure-Python oracle on a few packets (1 thread)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 5.0 and k < len(temps):
        ref.read_crypto_payload(temps[k])
        k += 1
    cpu_pps = k / (time.perf_counter() - t0)
    byts = int(lens.astype(np.uint64).sum())
    print(json.dumps({
        "metric": "QUIC Initial ReadCryptoPayload packets/s (device resident, ~1200 B client Initials)",
        "value": round(n / (ms / 1e3)), "unit": "packets/s", "n_packets": n, "steps": args.steps,
        "ms_per_batch": round(ms, 4), "packet_GBs": round(byts / (ms / 1e3) / 1e9, 2),
        "restore_copy_ms": round(copy_ms / args.steps, 4),
        "cpu_oracle": {"value": round(cpu_pps, 2), "unit": "packets/s", "cores": 1, "kind": "port",
                       "sample": f"{k} packets through oracle/quic_ref.py (pure Python)"}}))


if __name__ == "__main__":
    main()
