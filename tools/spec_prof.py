import math, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cfd_julia_amd.spectral import SpectralNS2D
from cfd_julia_amd.common import vm_ic
n = 4096; dx = 2 * math.pi / n
x = dx * np.arange(n + 1)
wn = np.zeros((n + 2, n + 2), order="F"); vm_ic(n, n, x, x, wn)
kind = sys.argv[1] if len(sys.argv) > 1 else "hybrid"
with SpectralNS2D(n, n, dx, dx, 1000.0, kind) as h:
    h.upload(wn); h.step(1e-4, 1); h.step(1e-4, 3)
