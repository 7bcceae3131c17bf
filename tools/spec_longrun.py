"""500 vortex-merger steps at 1024^2: half-spectrum state against full spectra (max |dw|)."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cfd_julia_amd.spectral import SpectralNS2D
from oracle import vm_oracle as vo
n = 1024
dx, dy, x, y = vo.vm_grid(n, n)
w0 = vo.vm_ic(n, n, x, y)
for kind in ("hybrid", "2/3"):
    out = {}
    for half in ("1", "0"):
        os.environ["CFDJ_SPEC_HALF"] = half
        with SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
            h.upload_interior(w0)
            h.step(2e-3, 500)
            out[half] = h.download()
    d = np.abs(out["1"] - out["0"]).max()
    print(kind, "500 steps: max|w|", np.abs(out["0"]).max(), "half vs full", d, flush=True)
