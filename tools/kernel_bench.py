import math, os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
from cfd_julia_amd import VortexMerger, _lib
from cfd_julia_amd.common import vm_ic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dx = 2 * math.pi / n
h = VortexMerger(n, n, dx, dx, 1000.0, device=0)
x = dx * np.arange(n + 1)
wn = np.zeros((n + 2, n + 2), order="F"); vm_ic(n, n, x, x, wn); h.upload(wn)
h.step(5e-4, 2)
res = {name: round(h.kernel_bench(k, 5e-4, 30) * 1e3, 2) for k, name in _lib.KB_NAMES.items()}
print(os.environ.get("TAG", ""), json.dumps(res))
