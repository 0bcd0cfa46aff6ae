"""Per-step kernel table from a rocprofv3 --stats kernel_stats.csv (steps = AdamW launches / 3)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
grep = sys.argv[3] if len(sys.argv) > 3 else ""
nsteps = sum(int(r["Calls"]) for r in rows if "adamw" in r["Name"]) / 3
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"steps ~{nsteps:.0f}  kernel ms/step {tot / nsteps / 1e6:.3f}")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    if grep and grep not in r["Name"]:
        continue
    print(f"{float(r['TotalDurationNs']) / nsteps / 1e3:8.1f} us/step {int(r['Calls']) / nsteps:5.1f}x "
          f"{float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:110]}")
