#!/usr/bin/env python3
"""bench.py -- device-resident Salamander obfuscation throughput on MI355X.

Metric (BASELINE.json): "device-resident packet-obfs GiB/s @ 1200B datagrams,
1/2/4/8 MI355X".  One step = one obfuscate pass (salamander.go:59-72 per
datagram) over the whole synthetic batch, inputs already resident in HBM.

  * N = 1: BASELINE.json configs[1] -- 1,048,576 x 1200 B datagrams, one batch.
    The line also carries a `bimodal` object: configs[2], 4M datagrams of the
    40 % 64 B / 60 % 1350 B mix, packed output.
  * N > 1: BASELINE.json configs[3] -- 8,388,608 x 1200 B datagrams per GPU
    (64M over 8 GPUs), one process per GPU; rank r owns datagrams
    [r*P, (r+1)*P) of the global synthetic batch (weak scaling, no collective
    on the data path; gloo only for the timing barrier and the max).
    `python bench.py --gpus N` starts the N rank processes itself (this process
    never touches the GPU); under torch.distributed.run it is one rank.

value = sum over ranks of plaintext payload bytes / max-over-ranks wall time
of the K timed steps / 2^30 (Go's b.SetBytes numerator).  The roofline is for
the obfuscate kernel: 2L+16 algorithmic HBM bytes per datagram / its average
launch time from HIP events on the launch stream.  `traffic` is the PMC
figure from profiles/pmc_traffic.json, used only when its entry was measured
on the same kernel sources (sha256 of hysteria_amd/csrc/*, see
scripts/collect_profiles.sh).  cpu_baseline times the C restatement in oracle/
(a port: no Go toolchain exists on the box) on host cores.

Warm load: whatever runs in a cold GPU's first ~10 ms of sustained load slows by
up to 12 % (a GPU power-state transient: per-call kernel traces with either
direction first, profiles/r05_transient/).  Each workload therefore first runs a
fixed warm load -- alternating obfuscate and deobfuscate steps for at least
WARM_LOAD_MS of wall time -- and then times its deobfuscate pass and its obfuscate
pass (the headline), each after the same W warm-up steps: both directions are
measured at the rate a busy serving GPU sustains.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured float4 copy
PSK = b"average_password"
METRIC = "device-resident packet-obfs GiB/s @ 1200B datagrams, 1/2/4/8 MI355X"
BIMODAL_MIN_WARMUP = 20
WARM_LOAD_MS = 60.0   # the fixed warm load before a workload's timed legs (>= 20 ms, see above)
KERNEL_NAMES = {   # keyed by the kernel the library reports for the batch (hyobfs_salamander_batch_kernel)
    "uniform": {"tile": "salamander_tile_kernel<obfuscate> (salamander_tile.h)",
                "wave": "salamander_wave_kernel<obfuscate, slotted> (salamander_wave.h)"},
    "bimodal": {"wave": "salamander_wave_kernel<obfuscate, packed> (salamander_wave.h) + width/length sums and scan (3 launches)",
                "flat": "salamander_flat_kernel<obfuscate> (salamander_flat.h) + width/length sums, scan and locate (4 launches)"},
}


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
    ap.add_argument("--no-bimodal", action="store_true", help="N=1: skip the configs[2] sub-object")
    ap.add_argument("--kernel", choices=["auto", "wave", "tile", "flat"], default="auto")
    ap.add_argument("--warm-load-ms", type=float, default=WARM_LOAD_MS)
    return ap.parse_args()


def kernel_src_sha() -> str:
    """sha256 over the kernel sources: keys the committed PMC traffic figures (scripts/src_sha.py)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from src_sha import src_sha
    return src_sha()


def pmc_traffic(workload: str, direction: str, datagrams: int, length, kernel: str) -> dict | None:
    """The committed PMC traffic entry for this batch, if one was measured on these kernel
    sources with the same kernel choice (kernel = "tile" / "wave" / "flat")."""
    f = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        entries = json.load(open(f)).get("entries", [])
    except (OSError, ValueError, AttributeError):
        return None
    sha = kernel_src_sha()
    import hysteria_amd
    if hysteria_amd.build_id() != sha:   # the loaded library was not built from these sources
        return None
    for e in entries:
        if (e.get("src_sha") == sha and e.get("workload") == workload and e.get("direction") == direction
                and e.get("datagrams") == datagrams and e.get("len") == length
                and f"salamander_{kernel}_kernel<" in e.get("kernel", "")):
            return e
    return None


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


def spawn_ranks(args) -> int:
    """--gpus N without an external launcher: one child process per rank (this
    parent never initialises HIP), rank 0 prints the line.  If a rank fails the
    others are stopped (by their own PIDs) and its exit code is returned."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc, pending = 0, set(range(len(procs)))
    while pending:
        for i in sorted(pending):
            r = procs[i].poll()
            if r is None:
                continue
            pending.discard(i)
            if r != 0 and rc == 0:
                rc = r
                for j in pending:
                    procs[j].kill()
        time.sleep(0.1)
    return rc


# ------------------------------------------------------------------ workloads
def setup_uniform(hy, obfs, dev, P, L, first):
    import torch
    inp = torch.empty(P * L, dtype=torch.uint8, device=dev)
    hy.synth_stream(inp, P * L, 1, first * L)
    salts = torch.empty(P, dtype=torch.int64, device=dev)
    hy.synth_u64(salts, P, 2, first)
    wire = torch.empty(P * (L + 8), dtype=torch.uint8, device=dev)
    back = torch.empty(P * L, dtype=torch.uint8, device=dev)

    def step_obf():
        obfs.obfuscate_batch(inp, P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)

    def step_deobf():
        obfs.deobfuscate_batch(wire, P, in_stride=L + 8, len_uniform=L + 8, out=back, out_stride=L)

    kernel = obfs.batch_kernel(True, inp=inp, n=P, in_stride=L, len_uniform=L, salts=salts, out=wire, out_stride=L + 8)
    return dict(obf=step_obf, deobf=step_deobf, payload=P * L, obf_bytes=P * (2 * L + 16),
                deobf_bytes=P * (2 * L + 8), inp=inp, wire=wire, back=back, n=P, len=L, kernel=kernel)


def setup_bimodal(hy, obfs, dev, P, first):
    """configs[2]: the datagrams back to back in one buffer (contiguous input: in_off
    NULL, in_stride 0, include/hyobfs.h), packed output; the wire, contiguous too, is
    the deobfuscate step's input."""
    import torch
    lens = torch.empty(P, dtype=torch.int32, device=dev)
    hy.synth_bimodal_lengths(lens, P, 3, first)
    total_in = int(lens.to(torch.int64).sum())
    inp = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    # stream offset of this rank's shard (global packed input): the lengths of
    # every earlier datagram, generated on device in chunks
    start = 0
    if first:
        tmp = torch.empty(min(first, 1 << 24), dtype=torch.int32, device=dev)
        done = 0
        while done < first:
            k = min(first - done, tmp.numel())
            hy.synth_bimodal_lengths(tmp, k, 3, done)
            start += int(tmp[:k].to(torch.int64).sum())
            done += k
    hy.synth_stream(inp, total_in, 1, start)
    salts = torch.empty(P, dtype=torch.int64, device=dev)
    hy.synth_u64(salts, P, 2, first)
    cap = total_in + 8 * P
    wire = torch.empty(cap, dtype=torch.uint8, device=dev)
    out_off = torch.empty(P, dtype=torch.int64, device=dev)
    out_len = torch.empty(P, dtype=torch.int32, device=dev)
    back = torch.empty(total_in + 16, dtype=torch.uint8, device=dev)
    nws = max(obfs.workspace_bytes(inp=inp, n=P, in_len=lens, out=wire, out_cap=cap),
              obfs.workspace_bytes(inp=wire, n=P, in_len=out_len, out=back, out_cap=total_in))
    ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=dev)

    def step_obf():
        obfs.obfuscate_batch(inp, P, in_len=lens, salts=salts, out=wire, out_cap=cap,
                             out_off=out_off, out_len=out_len, workspace=ws, workspace_bytes=ws.numel())

    def step_deobf():
        obfs.deobfuscate_batch(wire, P, in_len=out_len, out=back, out_cap=total_in,
                               workspace=ws, workspace_bytes=ws.numel())

    kernel = obfs.batch_kernel(True, inp=inp, n=P, in_len=lens, salts=salts, out=wire, out_cap=cap,
                               out_off=out_off, out_len=out_len, workspace=ws, workspace_bytes=ws.numel())
    return dict(obf=step_obf, deobf=step_deobf, payload=total_in, obf_bytes=2 * total_in + 16 * P,
                deobf_bytes=2 * total_in + 8 * P, inp=inp, wire=wire, back=back, n=P, len="bimodal",
                kernel=kernel)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))

    # stdout carries exactly one JSON line: whatever libraries print (gloo's "Rank r is
    # connected to ..." lines) goes to stderr until the line is printed
    sys.stdout.flush()
    real_stdout = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    import hysteria_amd as hy
    from hysteria_amd.shard import check_rank_devices, weak_shard

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

    def allgather(x: float) -> list:
        if world == 1:
            return [x]
        out = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(out, torch.tensor([x], dtype=torch.float64))
        return [float(t[0]) for t in out]

    # which card each rank bound: rank setup fails if two ranks share one while the
    # node has a card per rank (hysteria_amd/shard.py check_rank_devices)
    bus_id = hy.device_pci_bus_id(local)
    if world > 1:
        bus_ids = [None] * world
        dist.all_gather_object(bus_ids, bus_id)
    else:
        bus_ids = [bus_id]
    shared = check_rank_devices(bus_ids, torch.cuda.device_count())
    obfs = hy.SalamanderObfuscator(PSK, local)
    obfs.set_kernel(args.kernel)
    stream = torch.cuda.current_stream(dev)
    L = args.len

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
        mine = time.perf_counter() - t0
        return allmax(mine), mine, ev0.elapsed_time(ev1) / 1e3 / steps

    def warm_load(w):
        """The fixed warm load ("Warm load" above): obfuscate + deobfuscate steps for at
        least --warm-load-ms of wall time, synchronised every 8 pairs."""
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < args.warm_load_ms:
            for _ in range(8):
                w["obf"]()
                w["deobf"]()
            torch.cuda.synchronize()

    def measure(w, workload, warmup):
        """Timed deobfuscate and obfuscate passes of one workload, after the warm load:
        the line's fields.  The deobfuscate pass reads the wire the warm-up obfuscate
        steps wrote."""
        w["obf"]()
        warm_load(w)
        wall_deobf, _, ev_deobf = timed(w["deobf"], args.steps, warmup)
        wall_obf, mine_obf, ev_obf = timed(w["obf"], args.steps, warmup)
        total_payload = w["payload"] * world * args.steps   # every step processes the whole batch
        achieved = w["obf_bytes"] / ev_obf / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": KERNEL_NAMES[workload].get(w["kernel"], w["kernel"]),
                "algorithmic_bytes_per_launch": w["obf_bytes"], "avg_launch_ms": round(ev_obf * 1e3, 4),
                "kernel_src_sha": kernel_src_sha(), "lib_build_id": hy.build_id()}
        t = pmc_traffic(workload, "obfuscate", w["n"], w["len"], w["kernel"])
        if t:
            roof["traffic"] = t["hbm_bytes_per_launch"]
            roof["traffic_over_algorithmic"] = round(t["hbm_bytes_per_launch"] / w["obf_bytes"], 4)
            roof["traffic_source"] = t.get("source")
        deob = {"value": round(total_payload / wall_deobf / 2**30, 2), "unit": "GiB/s",
                "ms_per_step": round(wall_deobf / args.steps * 1e3, 4),
                "achieved_GBs": round(w["deobf_bytes"] / ev_deobf / 1e9, 1),
                "frac": round(w["deobf_bytes"] / ev_deobf / 1e9 / HBM_PEAK_GBS, 4),
                "avg_launch_ms": round(ev_deobf * 1e3, 4), "algorithmic_bytes_per_launch": w["deobf_bytes"]}
        t = pmc_traffic(workload, "deobfuscate", w["n"], w["len"], w["kernel"])
        if t:
            deob["traffic"] = t["hbm_bytes_per_launch"]
            deob["traffic_over_algorithmic"] = round(t["hbm_bytes_per_launch"] / w["deobf_bytes"], 4)
        per_gpu = [round(w["payload"] * args.steps / x / 2**30, 2) for x in allgather(mine_obf)]
        launch_ms = [round(x * 1e3, 4) for x in allgather(ev_obf)]
        return dict(value=total_payload / wall_obf / 2**30, ms=wall_obf / args.steps * 1e3, roofline=roof,
                    deobfuscate=deob, per_gpu=per_gpu, launch_ms=launch_ms)

    if args.workload == "uniform":
        P = args.packets_per_gpu or ((1 << 20) if world == 1 else (1 << 23))
        first, P = weak_shard(P, rank)
        w = setup_uniform(hy, obfs, dev, P, L, first)
        cfg_name = "configs[1]" if world == 1 else "configs[3] shard"
        config = {"workload": f"uniform {P} x {L} B datagrams per GPU ({cfg_name}), dense slotted output",
                  "datagrams_per_gpu": P, "datagram_len": L, "global_datagrams": P * world,
                  "psk": PSK.decode(), "parallelism": f"packet-index shards x{world}"}
    else:
        P = args.packets_per_gpu or (1 << 22)
        first, P = weak_shard(P, rank)
        w = setup_bimodal(hy, obfs, dev, P, first)
        config = {"workload": f"bimodal 40% 64 B / 60% 1350 B, {P} datagrams per GPU, contiguous input, packed output",
                  "datagrams_per_gpu": P, "global_datagrams": P * world, "psk": PSK.decode(),
                  "parallelism": f"packet-index shards x{world}"}
    torch.cuda.synchronize()
    m = measure(w, args.workload, args.warmup)

    parity = None
    if rank == 0 and not args.no_parity:
        torch.cuda.synchronize()
        parity = {"roundtrip_identity": bool(torch.equal(w["back"][:w["payload"]], w["inp"][:w["payload"]]))}
        if args.workload == "uniform" and P == (1 << 20) and L == 1200 and first == 0:
            with open(os.path.join(ROOT, "tests", "golden", "batch_digests.json")) as f:
                want = json.load(f)["config2_1M_x_1200"]["obf_sha256"]
            parity["sha256_match_config2"] = hashlib.sha256(w["wire"].cpu().numpy().tobytes()).hexdigest() == want
    del w

    res = {
        "metric": METRIC,
        "value": round(m["value"], 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warm_load_ms": args.warm_load_ms,
        "ms_per_step": round(m["ms"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SplitMix64 seeds 1/2/3, generated on device; PSK average_password)",
        "config": config,
        "roofline": m["roofline"],
        "per_gpu_GiBs": m["per_gpu"],
        "ranks": [{"rank": r, "pci_bus_id": bus_ids[r], "obf_call_ms": m["launch_ms"][r]} for r in range(world)],
        "devices_shared": shared,
        "deobfuscate": m["deobfuscate"],
        "parity": parity,
    }

    # configs[2] beside the headline (N = 1 only): the ragged mix with packed output
    if world == 1 and args.workload == "uniform" and not args.no_bimodal:
        torch.cuda.empty_cache()
        wb = setup_bimodal(hy, obfs, dev, 1 << 22, 0)
        torch.cuda.synchronize()
        # the first ~15 packed obfuscate launches after the switch from the uniform
        # batch run up to 30 % slow before settling (a per-launch kernel trace,
        # profiles/r04_trace_bimodal_obf40.txt), so this leg warms up for at least 20
        bw = max(args.warmup, BIMODAL_MIN_WARMUP)
        mb = measure(wb, "bimodal", bw)
        torch.cuda.synchronize()
        rt = bool(torch.equal(wb["back"][:wb["payload"]], wb["inp"][:wb["payload"]]))
        res["bimodal"] = {"workload": "configs[2]: 4194304 datagrams, 40% 64 B / 60% 1350 B, contiguous input, "
                                      "packed output",
                          "value": round(mb["value"], 2), "unit": "GiB/s", "ms_per_step": round(mb["ms"], 4),
                          "roofline": mb["roofline"], "deobfuscate": mb["deobfuscate"],
                          "warmup": bw, "parity": {"roundtrip_identity": rt}}
        del wb

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(1200, args.cpu_seconds)
    elif rank == 0:
        res["cpu_baseline"] = None
    sys.stdout.flush()
    os.dup2(real_stdout, 1)
    os.close(real_stdout)
    if rank == 0:
        print(json.dumps(res), flush=True)
    obfs.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
