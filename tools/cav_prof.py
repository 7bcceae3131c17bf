"""One short cavity run for rocprofv3: python tools/cav_prof.py [dst|mg] [n]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cfd_julia_amd.cavity import Cavity  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
dx = 1.0 / n
kind = sys.argv[1] if len(sys.argv) > 1 else "dst"
with Cavity(n, n, dx, dx, 100.0, poisson=kind, tol=1e-6) as h:
    h.step(5e-6, 2)
    h.step(5e-6, 20)
    if kind == "mg":
        print("vcycles", h.mg_iterations())
