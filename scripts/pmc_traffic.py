"""HBM bytes per launch of the obfuscate kernel from rocprofv3 FETCH_SIZE and
WRITE_SIZE passes (units: KiB).  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE counts exactly half the bytes of a wide coalesced streaming read, so
it is doubled; WRITE_SIZE is exact for 16-byte-per-lane streaming stores."""
import csv, glob, json, os, sys
root = sys.argv[1]
names = set()
def per_dispatch(counter):
    vals = {}
    for f in glob.glob(os.path.join(root, f"pmc_{counter}", "run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if not ("salamander_kernel<true" in row["Kernel_Name"] or "salamander_wave_kernel<true" in row["Kernel_Name"]) or row["Counter_Name"] != counter:
                continue
            names.add(row["Kernel_Name"])
            vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    v = sorted(vals.values())
    return v[len(v) // 2] if v else None
fetch_kib, write_kib = per_dispatch("FETCH_SIZE"), per_dispatch("WRITE_SIZE")
P, L = 1 << 20, 1200
fetch = 2 * fetch_kib * 1024
write = write_kib * 1024
alg = P * (2 * L + 16)
print(json.dumps({
    "kernel": " | ".join(sorted(names)), "datagrams": P, "len": L,
    "fetch_size_kib_raw": fetch_kib, "write_size_kib": write_kib,
    "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
    "hbm_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": (fetch + write) / alg,
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median dispatch, FETCH_SIZE x2 (gfx950)",
}, indent=1))
