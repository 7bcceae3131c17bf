"""Launch cfdj_vm_kernel_bench ids ($KB_IDS) a few times each at 4096^2 -- a short program
for rocprofv3 --pmc passes on single kernels."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cfd_julia_amd import VortexMerger
from cfd_julia_amd.common import vm_ic
n = 4096; dx = 2 * math.pi / n
h = VortexMerger(n, n, dx, dx, 1000.0, device=0)
x = dx * np.arange(n + 1)
wn = np.zeros((n + 2, n + 2), order="F"); vm_ic(n, n, x, x, wn); h.upload(wn)
h.step(5e-4, 1)
for k in [int(i) for i in os.environ.get("KB_IDS", "1,2,3,4,5,6").split(",")]:
    print(k, round(h.kernel_bench(k, 5e-4, int(os.environ.get("KB_N", "3"))) * 1e3, 1))
