"""Print the op table of a bench.py JSON line: tools/opt.py LOG [LOG2] (side by side)."""
import json
import sys


def load(p):
    return json.loads([x for x in open(p) if x.startswith("{")][-1])


ds = [load(p) for p in sys.argv[1:]]
print("ms/step", *[d["ms_per_step"] for d in ds], " host", *[d.get("host_enqueue_ms_per_step") for d in ds])
for k in ds[0]["op_table"]:
    print(f"{k:18s}", *[f"{d['op_table'].get(k, {}).get('ms_per_step', 0):7.3f}" for d in ds])
