"""Throughput of the QUIC Initial sniff path (hyobfs_quic_read_crypto_payload_batch)
on one GPU: N client Initial packets of ~1200 bytes (64 oracle-made templates,
V1 and V2, split CRYPTO frames + PADDING), device resident.  Prints one JSON
line: packets/s, packet GB/s, and the C restatement's rate on the host's cores
(oracle/quic_ref.c, the CPU baseline).

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
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline (counter passes)")
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
    # CPU baseline: the C restatement (oracle/quic_ref.c) on the same packets, host
    # threads, a bounded sample (~5 s per thread count)
    host = src.cpu().numpy()
    co = ref.CQuicOracle()
    cpu = {}
    for th in (() if args.no_cpu else (1, args.cpu_threads)):
        m = min(n, 4096 * th)
        t0 = time.perf_counter()
        reps = 0
        while True:
            st, _, _ = co.read_batch(host, off[:m], lens[:m], m, cap, threads=th)
            reps += 1
            if time.perf_counter() - t0 > 5.0:
                break
        assert (st == 0).all()
        cpu[th] = (m * reps / (time.perf_counter() - t0), m * reps)
    byts = int(lens.astype(np.uint64).sum())
    print(json.dumps({
        "metric": "QUIC Initial ReadCryptoPayload packets/s (device resident, ~1200 B client Initials)",
        "value": round(n / (ms / 1e3)), "unit": "packets/s", "n_packets": n, "steps": args.steps,
        "ms_per_batch": round(ms, 4), "packet_GBs": round(byts / (ms / 1e3) / 1e9, 2),
        "restore_copy_ms": round(copy_ms / args.steps, 4),
        "cpu_baseline": None if args.no_cpu else {
            "value": round(cpu[args.cpu_threads][0]), "unit": "packets/s", "cores": args.cpu_threads,
            "kind": "port", "single_thread_value": round(cpu[1][0]),
            "sample": f"{cpu[args.cpu_threads][1]} packets on {args.cpu_threads} threads + {cpu[1][1]} on 1 "
                      "through oracle/quic_ref.c (AES T-tables, 4-bit GHASH), ~5 s each"}}))


if __name__ == "__main__":
    main()
