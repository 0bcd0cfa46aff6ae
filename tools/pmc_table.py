"""Per-kernel PMC table of a short train step (tools/pmc_pass.sh over
``bench.py --steps 2 --warmup 2``), for profiles/: launches, HBM bytes per
launch (2 * FETCH_SIZE + WRITE_SIZE, the gfx950 FETCH correction), MFMA-busy
cycles, LDS issue stalls and bank conflicts, grouped by kernel and grid.

    python tools/pmc_table.py OUT_PREFIX DIR [DIR ...]

Writes OUT_PREFIX.json and OUT_PREFIX.md (top kernels by launches x bytes)."""

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("hvit::", "").replace("unsigned short", "bf16")
    return name[:110]


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                g = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
                vals[(short(r["Kernel_Name"]), g)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for (k, g), cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        row = {"kernel": k, "grid_threads": g, "launches": max(len(v) for v in cs.values()), "mean": m}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            row["hbm_bytes"] = round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024)
        rows.append(row)
    rows.sort(key=lambda r: -r.get("hbm_bytes", 0) * r["launches"])
    with open(out + ".json", "w") as f:
        json.dump(rows, f, indent=1)
    with open(out + ".md", "w") as f:
        f.write("| kernel | grid (threads) | launches | HBM MB/launch | MFMA busy Mcyc | LDS issue stall Mcyc | "
                "LDS bank conflict Mcyc | wave Mcyc |\n|---|---|---|---|---|---|---|---|\n")
        for r in rows[:40]:
            m = r["mean"]
            f.write(f"| {r['kernel']} | {r['grid_threads']} | {r['launches']} | "
                    f"{r.get('hbm_bytes', 0) / 1e6:.1f} | {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1e6:.2f} | "
                    f"{m.get('SQ_WAIT_INST_LDS', 0) / 1e6:.2f} | {m.get('SQ_LDS_BANK_CONFLICT', 0) / 1e6:.2f} | "
                    f"{m.get('SQ_WAVE_CYCLES', 0) / 1e6:.2f} |\n")
    print(open(out + ".md").read())


if __name__ == "__main__":
    main()
