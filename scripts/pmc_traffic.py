"""HBM bytes per batch call ("launch" in bench.py's roofline) of the obfuscate and deobfuscate kernels of one workload
from rocprofv3 FETCH_SIZE and WRITE_SIZE passes (units: KiB), merged into a
pmc_traffic.json keyed by the kernel-source hash bench.py computes.

  python scripts/pmc_traffic.py <pmc dir> <uniform|bimodal> <in.json> <out.json> [source label]

<pmc dir> holds pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/ (scripts/collect_profiles.sh).
gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts exactly half the
bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16-byte-per-lane streaming stores."""
import csv, glob, json, os, re, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_src_sha  # noqa: E402

root, wl, src, dst = sys.argv[1:5]
label = sys.argv[5] if len(sys.argv) > 5 else root
MAIN = {True: re.compile(r"salamander_(tile_kernel|wave_kernel|flat_kernel)<true"),
        False: re.compile(r"salamander_(tile_kernel|wave_kernel|flat_kernel)<false")}


def per_batch(counter, obf):
    """Counter value of one batch call: the dispatches of the run in issue order, cut
    into BATCHES equal groups (scripts/prof_one.py issues BATCHES calls per direction;
    a tile-kernel batch is several launches, launch_tile_sw), summed per group, median
    group."""
    vals, names = {}, set()
    for f in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter or not MAIN[obf].search(row["Kernel_Name"]):
                continue
            names.add(row["Kernel_Name"])
            d = int(row["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    if not vals:
        return None, names, 0
    order = [vals[d] for d in sorted(vals)]
    m = max(1, len(order) // BATCHES)   # launches per batch call
    groups = [sum(order[i:i + m]) for i in range(0, m * (len(order) // m), m)]
    groups.sort()
    return groups[len(groups) // 2], names, m


BATCHES = int(os.environ.get("PMC_BATCHES", "5"))
if wl in ("uniform", "uniform8m"):   # uniform8m: configs[3]'s 8M shard, stored as workload "uniform"
    P, L = (1 << 20) if wl == "uniform" else (1 << 23), 1200
    alg = {True: P * (2 * L + 16), False: P * (2 * L + 8)}
    wl = "uniform"
else:
    from oracle.salamander_ref import COracle
    P, L = 1 << 22, "bimodal"
    total_in = int(COracle().bimodal_lengths(3, 0, P).sum(dtype="uint64"))
    alg = {True: 2 * total_in + 16 * P, False: 2 * total_in + 8 * P}
sha = kernel_src_sha()
try:
    entries = json.load(open(src)).get("entries", [])
except (OSError, ValueError, AttributeError):
    entries = []
for obf in (True, False):
    direction = "obfuscate" if obf else "deobfuscate"
    fetch_kib, n1, m1 = per_batch("FETCH_SIZE", obf)
    write_kib, n2, m2 = per_batch("WRITE_SIZE", obf)
    if fetch_kib is None or write_kib is None:
        print(f"no {direction} dispatches in {root}", file=sys.stderr)
        continue
    fetch, write = 2 * fetch_kib * 1024, write_kib * 1024
    entries = [e for e in entries if not (e.get("src_sha") == sha and e.get("workload") == wl
                                          and e.get("direction") == direction and e.get("datagrams") == P)]
    entries.append({
        "src_sha": sha, "workload": wl, "direction": direction, "datagrams": P, "len": L,
        "kernel": " | ".join(sorted(n1 | n2)), "fetch_size_kib_raw": fetch_kib, "write_size_kib": write_kib,
        "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": alg[obf],
        "traffic_over_algorithmic": round((fetch + write) / alg[obf], 4),
        # algorithmic reads: obfuscate L + 8 (payload, salt), deobfuscate L + 8 (wire)
        "read_over_algorithmic_read": round(fetch / ((alg[obf] + (0 if obf else 8 * P)) / 2), 4),
        "write_over_algorithmic_write": round(write / ((alg[obf] - (0 if obf else 8 * P)) / 2), 4),
        "launches_per_batch": m1,
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median batch call "
                  f"({m1} launch(es) each), FETCH_SIZE x2 (gfx950); {label}"})
json.dump({"note": "HBM bytes per launch keyed by kernel_src_sha (bench.py); regenerate with "
                   "scripts/collect_profiles.sh on the tree being measured", "entries": entries},
          open(dst, "w"), indent=1)
print(json.dumps(entries[-2:], indent=1))
