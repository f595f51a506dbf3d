#!/usr/bin/env python3
"""bench.py -- device-resident Salamander obfuscation throughput on MI355X.

Metric (BASELINE.json): "device-resident packet-obfs GiB/s @ 1200B datagrams,
1/2/4/8 MI355X".  One step = one obfuscate pass (salamander.go:59-72 per
datagram) over the whole synthetic batch, inputs already resident in HBM.

  * N = 1: BASELINE.json configs[1] -- 1,048,576 x 1200 B datagrams, one batch.
  * N > 1: one process per GPU (torch.distributed.run); rank r owns packets
    [r*P, (r+1)*P) of the global synthetic batch (weak scaling, P per GPU,
    no collective on the data path; gloo only for the timing barrier/max).

value = sum over ranks of plaintext payload bytes / max-over-ranks wall time
of the K timed steps / 2^30 (Go's b.SetBytes numerator).  The roofline is for
the obfuscate kernel: 2L+16 algorithmic HBM bytes per datagram / its average
launch time from HIP events on the launch stream.  cpu_baseline times the C
restatement in oracle/ (a port: no Go toolchain exists on the box) on host
cores.  --workload bimodal runs BASELINE configs[2] (ragged, packed output).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured float4 copy
PSK = b"average_password"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["uniform", "bimodal"], default="uniform")
    ap.add_argument("--packets-per-gpu", type=int, default=None)
    ap.add_argument("--len", type=int, default=1200)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads() -> int:
    n = os.cpu_count() or 1
    for var in ("OMP_NUM_THREADS",):
        if os.environ.get(var, "").isdigit():
            n = min(n, int(os.environ[var]))
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    return max(1, n)


def cpu_baseline(L: int, seconds: float) -> dict:
    """Oracle C restatement, per-packet Obfuscate calls, bounded sample."""
    import numpy as np
    from oracle.salamander_ref import COracle
    co = COracle()
    n = 65536
    inp = co.fill_stream(1, 0, n * L)
    salts = co.salts(2, 0, n)
    out = np.empty(n * (L + 8), np.uint8)

    def rate(threads, budget):
        passes, t0 = 0, time.perf_counter()
        while True:
            co.run_uniform(True, PSK, n, inp, L, L, salts, out, L + 8, threads)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return passes * n * L / dt / 2**30, passes

    threads = cpu_threads()
    single, p1 = rate(1, seconds / 2)
    multi, pm = rate(threads, seconds / 2)
    return {"value": round(multi, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n} x {L} B datagrams, per-packet Obfuscate (oracle/salamander_ref.c), "
                      f"{pm} passes on {threads} threads + {p1} passes on 1 thread, ~{seconds:.0f} s",
            "single_thread_value": round(single, 3), "cpu_model": cpu_model(),
            "go_reference": "unavailable: no Go toolchain on the box"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import hysteria_amd
    from hysteria_amd.shard import weak_shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    # one process per GPU; modulo the visible devices so N > 1 can be rehearsed on one card
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    def barrier():
        if world > 1:
            dist.barrier()

    def allmax(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    obfs = hysteria_amd.SalamanderObfuscator(PSK, local)
    stream = torch.cuda.current_stream(dev)
    L = args.len

    if args.workload == "uniform":
        P = args.packets_per_gpu or (1 << 20)
        first, P = weak_shard(P, rank)
        inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
        hysteria_amd.synth_stream(inp, P * L, 1, first * L)
        salts = torch.empty(P, dtype=torch.int64, device=dev)
        hysteria_amd.synth_u64(salts, P, 2, first)
        wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
        back = torch.empty(P * L, dtype=torch.uint8, device=dev)
        payload_bytes = P * L
        obf_bytes = P * (2 * L + 16)      # algorithmic HBM bytes / launch
        deobf_bytes = P * (2 * L + 8)

        def step_obf():
            obfs.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire,
                                 out_stride=L + 8)

        def step_deobf():
            obfs.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)
        config = {"workload": f"uniform {P} x {L} B datagrams per GPU, slotted (= packed) output",
                  "datagrams_per_gpu": P, "datagram_len": L, "global_datagrams": P * world,
                  "psk": PSK.decode(), "parallelism": f"packet-index shards x{world}"}
    else:
        P = args.packets_per_gpu or (1 << 22)
        first, P = weak_shard(P, rank)
        lens = torch.empty(P, dtype=torch.int32, device=dev)
        hysteria_amd.synth_bimodal_lengths(lens, P, 3, first)
        in_off = torch.zeros(P, dtype=torch.int64, device=dev)
        in_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
        total_in = int(lens.to(torch.int64).sum())
        inp = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
        # stream offset of this rank's shard (global packed input): computed from the lengths
        # of every earlier packet, generated on device in chunks
        start = 0
        if first:
            tmp = torch.empty(min(first, 1 << 24), dtype=torch.int32, device=dev)
            done = 0
            while done < first:
                k = min(first - done, tmp.numel())
                hysteria_amd.synth_bimodal_lengths(tmp, k, 3, done)
                start += int(tmp[:k].to(torch.int64).sum())
                done += k
        hysteria_amd.synth_stream(inp, total_in, 1, start)
        salts = torch.empty(P, dtype=torch.int64, device=dev)
        hysteria_amd.synth_u64(salts, P, 2, first)
        cap = total_in + 8 * P
        wire = torch.empty(cap, dtype=torch.uint8, device=dev)
        out_off = torch.empty(P, dtype=torch.int64, device=dev)
        out_len = torch.empty(P, dtype=torch.int32, device=dev)
        back = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
        ws = torch.empty(hysteria_amd.workspace_size(P), dtype=torch.uint8, device=dev)
        payload_bytes = total_in
        obf_bytes = 2 * total_in + 16 * P
        deobf_bytes = 2 * total_in + 8 * P

        def step_obf():
            obfs.obfuscate_batch(inp, P, in_off=in_off, in_len=lens, salts=salts, out=wire, out_cap=cap,
                                 out_off=out_off, out_len=out_len, workspace=ws,
                                 workspace_bytes=ws.numel())

        def step_deobf():
            obfs.deobfuscate_batch(wire, P, in_off=out_off, in_len=out_len, out=back, out_cap=total_in,
                                   workspace=ws, workspace_bytes=ws.numel())
        config = {"workload": f"bimodal 40% 64 B / 60% 1350 B, {P} datagrams per GPU, packed output",
                  "datagrams_per_gpu": P, "global_datagrams": P * world, "psk": PSK.decode(),
                  "parallelism": f"packet-index shards x{world}"}

    torch.cuda.synchronize()

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        barrier()
        wall = time.perf_counter() - t0
        return allmax(wall), ev0.elapsed_time(ev1) / 1e3 / steps

    wall_obf, ev_obf = timed(step_obf, args.steps, args.warmup)
    wall_deobf, ev_deobf = timed(step_deobf, args.steps, args.warmup)

    parity = None
    if rank == 0 and not args.no_parity and args.workload == "uniform" and P == (1 << 20) and L == 1200:
        with open(os.path.join(ROOT, "tests", "golden", "batch_digests.json")) as f:
            want = json.load(f)["config2_1M_x_1200"]["obf_sha256"]
        torch.cuda.synchronize()
        got = hashlib.sha256(wire.cpu().numpy().tobytes()).hexdigest()
        rt = bool(torch.equal(back, inp))
        parity = {"sha256_match_config2": got == want, "roundtrip_identity": rt}
    elif rank == 0 and not args.no_parity:
        torch.cuda.synchronize()
        parity = {"roundtrip_identity": bool(torch.equal(back[:payload_bytes], inp[:payload_bytes]))}

    # wall_* cover all K timed steps: every step processes the whole batch once
    total_payload = payload_bytes * world * args.steps
    value = total_payload / wall_obf / 2**30
    achieved = obf_bytes / ev_obf / 1e9
    res = {
        "metric": "device-resident packet-obfs GiB/s @ 1200B datagrams, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_obf / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SplitMix64 seeds 1/2/3, generated on device; PSK average_password)",
        "config": config,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": ("salamander_wave_kernel<obfuscate, slotted>" if args.workload == "uniform"
                                else "salamander_kernel<obfuscate, packed> (+ tile-sum scan)"),
                     "algorithmic_bytes_per_launch": obf_bytes, "avg_launch_ms": round(ev_obf * 1e3, 4)},
        "deobfuscate": {"value": round(total_payload / wall_deobf / 2**30, 2), "unit": "GiB/s",
                        "ms_per_step": round(wall_deobf / args.steps * 1e3, 4),
                        "achieved_GBs": round(deobf_bytes / ev_deobf / 1e9, 1),
                        "frac": round(deobf_bytes / ev_deobf / 1e9 / HBM_PEAK_GBS, 4)},
        "parity": parity,
    }
    traffic_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(traffic_file) and args.workload == "uniform":
        try:
            tj = json.load(open(traffic_file))
            if tj.get("datagrams") == P and tj.get("len") == L:
                res["roofline"]["traffic"] = tj["hbm_bytes_per_launch"]
                res["roofline"]["traffic_source"] = tj.get("source", traffic_file)
        except (ValueError, KeyError):
            pass
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(1200, args.cpu_seconds)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    obfs.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
