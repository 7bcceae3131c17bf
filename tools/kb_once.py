"""Launch cfdj_vm_kernel_bench ids ($KB_IDS) a few times each at $KB_NX x $KB_NY (4096^2) -- a short program
for rocprofv3 --pmc passes on single kernels."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cfd_julia_amd import VortexMerger
from cfd_julia_amd.common import vm_ic
n = int(os.environ.get("KB_NX", "4096")); ny = int(os.environ.get("KB_NY", str(n)))
dx = 2 * math.pi / n; dy = 2 * math.pi / ny
h = VortexMerger(n, ny, dx, dy, 1000.0, device=0)
x = dx * np.arange(n + 1); y = dy * np.arange(ny + 1)
wn = np.zeros((n + 2, ny + 2), order="F"); vm_ic(n, ny, x, y, wn); h.upload(wn)
h.step(5e-4, 1)
for k in [int(i) for i in os.environ.get("KB_IDS", "1,2,3,4,5,6").split(",")]:
    print(k, round(h.kernel_bench(k, 5e-4, int(os.environ.get("KB_N", "3"))) * 1e3, 1))
