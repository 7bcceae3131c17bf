"""Aggregate a rocprofv3 *_kernel_trace.csv by (kernel, grid size): calls, mean us."""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: [0, 0.0])
for row in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"cfdj::\(anonymous namespace\)::|HIP_vector_type<double, 2u>", "",
                  row["Kernel_Name"]).split("(")[0][:60]
    grid = int(row.get("Grid_Size_X", row.get("Grid_Size", 0)) or 0) * \
        int(row.get("Grid_Size_Y", 1) or 1)
    wg = int(row.get("Workgroup_Size_X", 1) or 1) * int(row.get("Workgroup_Size_Y", 1) or 1)
    a = acc[(name, grid // max(wg, 1), wg)]
    a[0] += 1
    a[1] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in acc.values())
for (name, wgs, wg), (n, us) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print(f"{name:60s} wgs {wgs:6d} x {wg:4d}  calls {n:6d}  mean {us / n:8.2f} us  {100 * us / tot:5.1f} %")
