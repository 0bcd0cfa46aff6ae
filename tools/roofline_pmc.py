"""profiles/roofline_pmc.json for the ViT linear op classes (multi-op form
read by bench.py's measured_traffic): HBM bytes per op launch from rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) over
``bench.py --roofline-only --roofline-op OP`` (tools/gpu_session.sh roof:OP).
HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB; the gfx950 FETCH_SIZE
correction, MI355X_MICROARCH.md HBM section).  Per op launch = the op's
per-step launch mix of its kernels (mean bytes per launch of each kernel over
every launch of it in the run) / the op's launches per step.

    python tools/roofline_pmc.py OUT OP:FETCH_DIR:WRITE_DIR [OP:FETCH_DIR:WRITE_DIR ...]
"""

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

# op -> [(kernel-name regex, grid size, launches per step, what)], B = 32 default model, 6 blocks
MIX = {
    "vit_linear_fwd": [(r"gemm_kernel<.*128, 128, .*LdDense<.*true>, .*LdDense<.*true>, 1,", 196608, 6, "qkv"),
                       (r"gemm_kernel<.*128, 64, .*LdDense<.*true>, .*LdDense<.*true>, 4,", 131072, 12,
                        "proj + fc2 (residual)"),
                       (r"gemm_ring_kernel<256, 256, 2, 4, 2, true, true, 3>", 131072, 6, "fc1 (GELU_DUAL)")],
    "vit_linear_dgrad": [(r"gemm_ring_kernel<256, 256, 2, 4, 2, true, false, 5>", 131072, 6, "fc2 dgrad (GELU backward)"),
                         (r"gemm_kernel<.*128, 64, .*LdDense<.*true>, .*LdDense<.*false>, 1,", 131072, 18,
                          "fc1 / proj / qkv dgrad")],
}
ALGO = {  # algorithmic bytes per op launch (bf16 operands / activations, f32 residual rows), B = 32, D = 512
    "vit_linear_fwd": (56.2e6, "mean of qkv 35.2 MB (xn1 8.4 + W 1.6 in, qkv 25.2 out), proj 42.5 (o 8.4 + W 0.5 + "
                               "f32 residual 16.8 in, f32 x1 16.8 out), fc1 77.7 (xn2 8.4 + W 2.1 in, gelu'(h) and "
                               "gelu(h) 33.6 each out), fc2 69.3 (a 33.6 + W 2.1 + residual 16.8 in, x2 16.8 out)"),
    "vit_linear_dgrad": (43.6e6, "mean of fc2 dgrad 77.7 MB (dy 8.4 + W 2.1 + gelu'(h) 33.6 in, dh 33.6 out), fc1 "
                                 "dgrad 44.1 (dh 33.6 + W 2.1 in, bf16 dxn2 8.4 out), proj dgrad 17.3, qkv dgrad 35.2 "
                                 "(dqkv 25.2 + W 1.6 in, bf16 dxn1 8.4 out)"),
}


def counters(d, name):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                out[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def main():
    out = sys.argv[1]
    res = {"variant": "default", "mode": "train", "batch": 32, "round": 6, "ops": {}}
    for spec in sys.argv[2:]:
        op, fd, wd = spec.split(":")
        fe, wr = counters(fd, "FETCH_SIZE"), counters(wd, "WRITE_SIZE")
        kern, tot, n = {}, 0.0, 0
        for pat, grid, per_step, what in MIX[op]:
            rx = re.compile(pat)
            fk = [v for (k, g), vs in fe.items() if rx.search(k) and g == grid for v in vs]
            wk = [v for (k, g), vs in wr.items() if rx.search(k) and g == grid for v in vs]
            if not fk or not wk:
                raise SystemExit(f"{op}: no launches of {pat}")
            b = (2 * sum(fk) / len(fk) + sum(wk) / len(wk)) * 1024
            kern[what] = {"launches": len(fk), "hbm_bytes_per_launch": round(b)}
            tot += b * per_step
            n += per_step
        algo, note = ALGO[op]
        res["ops"][op] = {"hbm_bytes_per_launch": round(tot / n), "kernels": kern,
                          "algorithmic_bytes_per_launch": round(algo), "algorithmic_note": note,
                          "traffic_over_algorithmic": round(tot / n / algo, 3),
                          "how": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over bench.py --roofline-only "
                                 f"--roofline-op {op} ({fd}, {wd})"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v["hbm_bytes_per_launch"] for k, v in res["ops"].items()}))


if __name__ == "__main__":
    main()
