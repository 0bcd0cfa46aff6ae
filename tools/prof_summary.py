"""Summarise a rocprofv3 --kernel-trace --stats output directory (csv or
rocpd SQLite): top kernels by total time, per bench step.
Usage: prof_summary.py DIR [steps] [top] [--grid]   (--grid: split by launch grid)"""

import csv
import glob
import os
import re
import sys


def short(name):
    grid = re.search(r" grid=\S+", name)
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("hvit::", "").replace("unsigned short", "bf16")
    return name[:100] + (grid.group(0) if grid else "")


def main():
    d = sys.argv[1]
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[1]) if len(args) > 1 else 13
    top = int(args[2]) if len(args) > 2 else 40
    by_grid = "--grid" in sys.argv
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if f and not by_grid:
        rows = list(csv.DictReader(open(f[0])))
    elif tr:
        agg = {}
        for r in csv.DictReader(open(tr[0])):
            wg = int(r["Workgroup_Size_X"]) or 1
            key = r["Kernel_Name"] + (f" grid={int(r['Grid_Size_X']) // wg}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
                                      if by_grid else "")
            a = agg.setdefault(key, [0, 0.0])
            a[0] += 1
            a[1] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        rows = [dict(Name=k, Calls=v[0], TotalDurationNs=v[1], AverageNs=v[1] / v[0]) for k, v in agg.items()]
    else:
        import sqlite3
        db = sqlite3.connect(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0])
        key = "name || ' grid=' || grid_x || 'x' || grid_y || 'x' || grid_z" if by_grid else "name"
        rows = [dict(Name=r[0], Calls=r[1], TotalDurationNs=r[2], AverageNs=r[3]) for r in db.execute(
            f"select {key}, count(*), sum(duration), avg(duration) from kernels group by {key}")]
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total GPU kernel time {tot / 1e6:.2f} ms over {steps} steps = {tot / 1e6 / steps:.3f} ms/step")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e3 / steps:9.1f} us/step {int(r['Calls']) / steps:6.1f} calls "
              f"{float(r['AverageNs']) / 1e3:8.1f} us avg  {100 * t / tot:5.1f}%  {short(r['Name'])}")


if __name__ == "__main__":
    main()
