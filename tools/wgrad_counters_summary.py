"""Summarise tools/r6_wgrad_counters.sh: per train step (the class's launches of
one step), the SQ / TCC counters of the ViT weight-gradient kernels in the
per-Linear (round 5) and grouped (round 6) forms.

    python tools/wgrad_counters_summary.py TAG OUT.json
"""
import csv
import json
import re
import sys
from collections import defaultdict

PAT = {0: re.compile(r"gemm_ring_kernel<.*false, false, 2>|gemm_kernel<.*LdDense<unsigned short, false>, "
                     r"hvit::LdDense<unsigned short, false>"),
       1: re.compile(r"wgrad_group_kernel")}
PER_STEP = {0: 24, 1: 1}


def main():
    tag, out = sys.argv[1], sys.argv[2]
    res = {"how": "tools/r6_wgrad_counters.sh: bench.py --roofline-only --roofline-op vit_linear_wgrad (B = 32 "
                  "default model) under rocprofv3 --pmc, HF.WGRAD_GROUP = 0 (round 5's per-Linear split-K GEMMs; "
                  "their slab sums ride on other launches and are not counted) and 1 (the grouped launch); "
                  "counters summed over the class's kernels and divided by the steps' worth of launches",
           "modes": {}}
    for g in (0, 1):
        tot, disp = defaultdict(float), set()
        for kind in ("sq", "tcc"):
            for r in csv.DictReader(open(f"gpurun_out/{tag}_g{g}_{kind}/run_counter_collection.csv")):
                if PAT[g].search(r["Kernel_Name"]):
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
                    disp.add((kind, r["Dispatch_Id"]))
        n = len([d for d in disp if d[0] == "sq"])
        steps = n / PER_STEP[g]
        ps = {k: v / steps for k, v in tot.items()}
        ps["mfma_busy_over_busy_cycles"] = ps["SQ_VALU_MFMA_BUSY_CYCLES"] / max(ps["SQ_BUSY_CYCLES"], 1)
        ps["wait_inst_any_over_wave_cycles"] = ps["SQ_WAIT_INST_ANY"] / max(ps["SQ_WAVE_CYCLES"], 1)
        ps["tcc_hit_rate"] = ps["TCC_HIT_sum"] / max(ps["TCC_HIT_sum"] + ps["TCC_MISS_sum"], 1)
        res["modes"]["grouped" if g else "per_linear"] = {"dispatches": n, "steps": steps,
                                                         "per_step": {k: round(v, 4) for k, v in ps.items()}}
    json.dump(res, open(out, "w"), indent=1)
    for m, v in res["modes"].items():
        p = v["per_step"]
        print(m, v["dispatches"], {k: p[k] for k in ("mfma_busy_over_busy_cycles", "wait_inst_any_over_wave_cycles",
                                                      "tcc_hit_rate", "TCC_EA0_RDREQ_sum", "SQ_BUSY_CYCLES")})


if __name__ == "__main__":
    main()
