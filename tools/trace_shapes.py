"""Per (kernel, grid) timing table from a rocprofv3 kernel_trace.csv: which GEMM
shape each instantiation runs, per step (steps = AdamW launches / 3)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
grep = sys.argv[2] if len(sys.argv) > 2 else ""
steps = sum(1 for r in rows if "adamw" in r["Kernel_Name"]) / 3
agg = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if grep and grep not in n:
        continue
    key = (n.replace("hvit::", "").replace("unsigned short", "u16")[:150],
           (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])),
           int(r["Workgroup_Size_X"]), r["VGPR_Count"], r["LDS_Block_Size"])
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    tot += sum(v) / steps
    print(f"{sum(v) / steps:8.1f} us/step {len(v) / steps:5.1f}x med {v[len(v) // 2]:7.1f}us grid {k[1]} wg {k[2]} "
          f"vgpr {k[3]} lds {k[4]}  {k[0]}")
print(f"total {tot:.1f} us/step over {steps:.0f} steps")
