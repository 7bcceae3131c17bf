"""Print name / calls / average us of a rocprofv3 *_kernel_stats.csv (names shortened)."""
import csv
import re
import sys

for row in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"cfdj::\(anonymous namespace\)::|HIP_vector_type<double, 2u>", "", row["Name"])
    name = name.split("(")[0][:70]
    print(f'{name:70s} {int(row["Calls"]):6d} {float(row["AverageNs"]) / 1e3:9.2f} us '
          f'{float(row["Percentage"]):6.2f} %')
