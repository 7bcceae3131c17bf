"""Spectral solvers at 8192^2: half-spectrum path against the library transforms."""
import math, sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cfd_julia_amd.spectral import SpectralNS2D
from cfd_julia_amd.common import vm_ic
n = 8192; dx = 2 * math.pi / n
x = dx * np.arange(n + 1)
wn = np.zeros((n + 2, n + 2), order="F"); vm_ic(n, n, x, x, wn)
for kind in ("hybrid", "2/3"):
    for env in (None, "rocfft"):
        os.environ.pop("CFDJ_SPEC_FFT", None)
        if env: os.environ["CFDJ_SPEC_FFT"] = env
        with SpectralNS2D(n, n, dx, dx, 1000.0, kind) as h:
            h.upload(wn); h.step(1e-4, 1)
            t0 = time.perf_counter(); h.step(1e-4, 3); t = (time.perf_counter() - t0) / 3
        print(kind, env or "half", f"{t*1e3:.2f} ms/step", f"{n*n/t/1e6:.0f} MLUPS", flush=True)
