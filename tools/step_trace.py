"""One training step's kernel sequence from a rocprofv3 kernel trace
(--kernel-trace, csv): the dispatches between the last two wgrad_group
launches (or another marker kernel), with duration, grid and the gap before
each.  Shows per-call times where kernel_stats only has class averages.

    python tools/step_trace.py DIR [marker_regex] [min_us]
"""
import csv
import glob
import re
import sys


def main():
    d = sys.argv[1]
    marker = re.compile(sys.argv[2] if len(sys.argv) > 2 else "adamw_kernel")
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    rows = list(csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker.search(r["Kernel_Name"])]
    # a step = from just after one marker group to the last marker of the next group
    if len(idx) < 4:
        print("not enough markers")
        return
    a, b = idx[-4], idx[-2]
    seg = rows[a + 1:b + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    prev_end = int(rows[a]["End_Timestamp"])
    tot = 0.0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        us = (e - s) / 1e3
        tot += us
        if us >= min_us:
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:90]
            grid = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}'
            print(f"{(s - t0) / 1e3:9.1f} {us:8.1f} gap {(s - prev_end) / 1e3:6.1f}  {grid:>22s}  {name}")
        prev_end = e
    print(f"kernels {len(seg)}, busy {tot:.1f} us, span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
