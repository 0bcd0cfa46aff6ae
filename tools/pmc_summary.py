"""Per-kernel PMC summary from rocprofv3 --pmc csv passes (tools/pmc_pass.sh).

    python tools/pmc_summary.py OUT.json DIR [DIR ...] [--op NAME --match REGEX --oplaunches N]

Kernels are grouped by (short name, grid); per group: launches and the mean
per-launch counters.  HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes):
on gfx950 FETCH_SIZE counts half of the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section).  SQ_VALU_MFMA_BUSY_CYCLES is summed over
the chip; mfma_busy_frac = it / (SQ_BUSY_CYCLES * 4 SIMDs * ... ) is not
derived here (no gfx950 derived-counter formulas ship with ROCm 7.2): the raw
per-launch values are kept.  With --op NAME (the bench's dominant op class),
hbm_bytes_per_launch of the whole op (all of its kernels per op launch) is
also written for bench.py's roofline ``traffic``."""

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("hvit::", "").replace("unsigned short", "bf16")
    return name[:150]


def main():
    argv = sys.argv[1:]
    def opt(flag, cast=str):
        nonlocal argv
        if flag in argv:
            i = argv.index(flag)
            v = cast(argv[i + 1])
            argv = argv[:i] + argv[i + 2:]
            return v
        return None

    op = opt("--op")
    match = opt("--match")
    oplaunches = opt("--oplaunches", int)
    out, dirs = argv[0], argv[1:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                g = f"{r.get('Grid_Size', r.get('Grid_Size_X', '?'))}"
                key = f"{short(r['Kernel_Name'])} grid={g}"
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, cs in vals.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        row = {"launches": max(len(v) for v in cs.values()), "counters_mean_per_launch": mean}
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            row["hbm_bytes_per_launch"] = round((2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024)
        kernels[k] = row
    summary = {"kernels": dict(sorted(kernels.items(), key=lambda kv: -kv[1].get("hbm_bytes_per_launch", 0)))}
    if op:
        # the roofline loop's op = one split-K GEMM + its slab reduction per launch
        # --match: regex of the op's kernel names; --oplaunches: op launches in the
        # run (every kernel launch of the op counts toward its bytes)
        pat = re.compile(match or r"^(gemm_kernel|sum_slabs)")
        mine = {k: r for k, r in kernels.items() if pat.search(k)}
        tot = sum(r.get("hbm_bytes_per_launch", 0) * r["launches"] for r in mine.values())
        nops = oplaunches or sum(r["launches"] for k, r in mine.items() if k.startswith("gemm_kernel"))
        summary["op_kernels"] = sorted(mine)
        summary["op_launches"] = nops
        summary["op"] = op
        summary["hbm_bytes_per_launch"] = round(tot / max(nops, 1))
    with open(out, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
