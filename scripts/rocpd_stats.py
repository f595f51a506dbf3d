"""Per-kernel duration stats (and the gaps between consecutive dispatches) from a
rocprofv3 rocpd database: python scripts/rocpd_stats.py <run_results.db> [name-filter]"""
import sqlite3
import statistics
import sys

db = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
rows = c.execute("select k.start, k.end, s.kernel_name from rocpd_kernel_dispatch k "
                 "join rocpd_info_kernel_symbol s on k.kernel_id = s.id order by k.start").fetchall()
by = {}
for st, en, nm in rows:
    by.setdefault(nm, []).append((en - st) / 1000.0)
print(f"{'kernel':90s} {'n':>4s} {'avg_us':>9s} {'med_us':>9s} {'min_us':>9s}")
for nm, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    if filt in nm:
        print(f"{nm[:90]:90s} {len(d):4d} {statistics.mean(d):9.2f} {statistics.median(d):9.2f} {min(d):9.2f}")
gaps = [(rows[i + 1][0] - rows[i][1]) / 1000.0 for i in range(len(rows) - 1)]
if gaps:
    print(f"gaps between consecutive dispatches: median {statistics.median(gaps):.2f} us")
