import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cfd_julia_amd.cavity import Cavity
n = 2048; dx = 1.0 / n
with Cavity(n, n, dx, dx, 100.0, poisson="dst", tol=1e-6) as h:
    h.step(5e-6, 2); h.step(5e-6, 20)
