"""VALU issue fraction per kernel from one rocprofv3 --pmc pass of
SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / SQ_WAVES / SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE
(scripts/gpu_r03n.sh, gpu_r03fin.sh: the aux_bench.py run), median dispatch per kernel:
  valu_issue_fraction = SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8 cycles / 2 cycles per wave64 VALU instruction)
  python scripts/valu_fraction.py <run_counter_collection.csv> [out.json]"""
import csv
import json
import statistics
import sys
from collections import defaultdict

src = sys.argv[1]
per = defaultdict(dict)   # dispatch -> counter -> value
meta = {}
for row in csv.DictReader(open(src)):
    d = row["Dispatch_Id"]
    per[d][row["Counter_Name"]] = per[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    meta[d] = (row["Kernel_Name"].split("(")[0].removeprefix("void "), row["VGPR_Count"],
               (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
by = defaultdict(list)
for d, cs in per.items():
    by[meta[d][0]].append((d, cs))
out = {"note": "median dispatch; valu_issue_fraction = SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8 cycles / "
               "2 cycles per wave64 VALU instruction); scripts/valu_fraction.py", "kernels": {}}
for name, ds in sorted(by.items()):
    if not name.startswith("hyobfs::") or "synth" in name:
        continue
    ds.sort(key=lambda x: x[1].get("GRBM_GUI_ACTIVE", 0.0))
    d, cs = ds[len(ds) // 2]
    insts, grbm = cs.get("SQ_INSTS_VALU", 0.0), cs.get("GRBM_GUI_ACTIVE", 0.0)
    cyc = grbm / 8
    out["kernels"][name] = {
        "SQ_INSTS_VALU": insts, "SQ_WAVES": cs.get("SQ_WAVES"), "GRBM_GUI_ACTIVE": grbm, "cycles_per_xcd": cyc,
        "valu_issue_fraction": round(insts / (1024 * cyc / 2), 3) if cyc else None,
        "valu_insts_per_wave": round(insts / cs["SQ_WAVES"]) if cs.get("SQ_WAVES") else None,
        "ms_under_pmc": round(meta[d][2], 4), "vgpr": meta[d][1], "dispatches": len(ds)}
text = json.dumps(out, indent=1)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(text + "\n")
print(text)
