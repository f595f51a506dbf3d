"""Per batch CALL durations from a rocprofv3 --kernel-trace CSV of bench.py.

One batch call can be several kernel launches: the tile kernel goes out in launches
of 512K datagrams (salamander_tile.h launch_tile_sw: 2 per 1M-datagram call), the
bimodal call is the width/length sums, their scan and (flat kernel) the locate
prepass followed by the main kernel's launch(es).  bench.py's roofline times the whole
call with HIP events on its stream; this sums each call's dispatches so that the
rocprofv3 figure describes the same thing.

  python scripts/rocprof_per_call.py <dir with *kernel_trace.csv> [uniform launches per call = 2]

Uniform calls are cut every K tile-kernel dispatches of one direction; bimodal calls
start at their tile_sums_kernel dispatch and take every dispatch up to the next one."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    us = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    calls = {}

    def add(g, v, n):
        calls.setdefault(g, []).append((v, n))

    # uniform: tile kernel dispatches per direction, K per call
    for obf in (True, False):
        seq = [us(r) for r in rows if f"salamander_tile_kernel<{'true' if obf else 'false'}" in r["Kernel_Name"]]
        for i in range(0, len(seq) - len(seq) % K, K):
            add(f"uniform_{'obfuscate' if obf else 'deobfuscate'}", sum(seq[i:i + K]), K)
    # bimodal: from a tile_sums_kernel dispatch to the next one (or a non-bimodal kernel)
    bim = ("tile_sums_kernel", "scan_tiles_kernel", "flat_locate_kernel", "salamander_flat_kernel",
           "salamander_wave_kernel")
    cur = None
    for r in rows:
        name = r["Kernel_Name"]
        if "tile_sums_kernel" in name:
            if cur:
                add(*cur)
            cur = [f"bimodal_{'obfuscate' if '<true' in name else 'deobfuscate'}", 0.0, 0]
        if cur and any(k in name for k in bim):
            cur[1] += us(r)
            cur[2] += 1
        elif cur:
            add(*cur)
            cur = None
    if cur:
        add(*cur)
    out = {}
    for g, cs in calls.items():
        v = [c[0] for c in cs]
        out[g] = {"calls": len(cs), "launches_per_call": statistics.mode([c[1] for c in cs]),
                  "mean_us": round(statistics.mean(v), 1), "median_us": round(statistics.median(v), 1),
                  "min_us": round(min(v), 1), "max_us": round(max(v), 1)}
    print(json.dumps({"source": os.path.relpath(f[0]), "per_call": out}, indent=1))


if __name__ == "__main__":
    main()
