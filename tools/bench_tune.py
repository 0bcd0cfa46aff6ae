"""bench.py with library tuning knobs set first (same-process A/B of a
hvit_gemm_tune form or a functional.py path switch):
    python tools/bench_tune.py 6=1 HF.LN_DY_LOW=0 -- --no-cpu-baseline
(``what=value`` / ``HF.NAME=int`` before ``--``, bench.py's arguments after)."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    import hvit_amd_loader

    hv = hvit_amd_loader.load()
    HF = sys.modules["hvit_amd.functional"]
    knobs = []
    for a in argv[:cut]:
        k, v = a.split("=")
        if k.startswith("HF."):
            setattr(HF, k[3:], type(getattr(HF, k[3:]))(int(v)))
            print(f"functional.{k[3:]} = {getattr(HF, k[3:])}", file=sys.stderr)
        else:
            knobs.append((int(k), int(v)))
    for what, value in knobs:
        old = hv._lib.lib().hvit_gemm_tune(what, value)
        print(f"hvit_gemm_tune({what}, {value}) (was {old})", file=sys.stderr)
    import bench

    sys.argv = [os.path.join(ROOT, "bench.py")] + argv[cut + 1:]
    bench.main()


if __name__ == "__main__":
    main()
