"""Per-kernel mean of every counter in rocprofv3 --pmc counter_collection.csv files.

  python tools/pmc_diag.py gpurun_out/pmc_a/*counter_collection.csv ... [--json out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(vm_stage_kernel<\d>|rows_fwd_kernel<\d+>|cols_kernel<\d+>|"
                  r"rows_inv_kernel<\d+>|\w+_kernel(<\d+>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    paths = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    vals = defaultdict(lambda: defaultdict(list))
    for p in paths:
        if out and p == out:
            continue
        for r in csv.DictReader(open(p)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}
    for k, d in sorted(res.items()):
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:32s} {v:16.4g}")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
