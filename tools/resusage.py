"""Summarise a -Rpass-analysis=kernel-resource-usage log: name, VGPRs, spills, occupancy, LDS."""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
OCC = r"Occupancy \[waves/SIMD\]"
LDS = r"LDS Size \[bytes/block\]"
for b in re.split(r"remark: Function Name: ", txt)[1:]:
    name = b.split(" ")[0]
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    dem = re.sub(r"cfdj::\(anonymous namespace\)::|HIP_vector_type<double, 2u>", "", dem).split("(")[0]

    def g(k):
        return re.search(k + r": (\d+)", b).group(1)

    print(f"{dem[:64]:64s} VGPR {g('VGPRs'):>3s} spill {g('VGPRs Spill'):>3s} occ {g(OCC)} LDS {g(LDS)}")
