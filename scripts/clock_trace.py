"""Per-dispatch GPU clock from a rocprofv3 counter pass (scripts/gpu_session.sh clk:...).

GRBM_GUI_ACTIVE counts the GPU's busy cycles during a dispatch, GRBM_COUNT all of
its cycles; divided by the dispatch's duration (Start/End_Timestamp, ns) they give
the shader clock the dispatch ran at.  rocprofv3 sums the counter over the 8 XCDs
(each has its own GRBM): the per-XCD clock is the sum / 8 (2.0-2.3 GHz measured,
against the 2.4 GHz peak engine clock).  If a run of slow dispatches ran at the same
clock as the fast ones, the slowdown is on the memory side, not the clock.

  python scripts/clock_trace.py gpurun_out/TAG/clk_bimodal_40_0 [kernel-substring]
Prints one CSV line per matching dispatch: kind, index, duration_us, MHz."""
import csv
import glob
import os
import sys


def rows(d: str, match: str):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        sys.exit(f"no counter_collection.csv under {d}")
    per = {}
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if match not in k or not ("wave_kernel" in k or "tile_kernel" in k):
            continue
        e = per.setdefault(int(r["Dispatch_Id"]), {"name": k, "t0": int(r["Start_Timestamp"]),
                                                   "t1": int(r["End_Timestamp"])})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return [per[i] for i in sorted(per)]


def main():
    d = sys.argv[1]
    match = sys.argv[2] if len(sys.argv) > 2 else "salamander"
    print("kind,index,duration_us,gui_active_MHz_sum8,grbm_count_MHz_sum8,clock_MHz_per_xcd")
    idx = {}
    for e in rows(d, match):
        kind = "obfuscate" if "<true" in e["name"] else "deobfuscate"
        i = idx.get(kind, 0)
        idx[kind] = i + 1
        us = (e["t1"] - e["t0"]) / 1e3
        ga = e.get("GRBM_GUI_ACTIVE", 0.0) / us
        gc = e.get("GRBM_COUNT", 0.0) / us
        print(f"{kind},{i},{us:.1f},{ga:.0f},{gc:.0f},{gc / 8:.0f}")


if __name__ == "__main__":
    main()
