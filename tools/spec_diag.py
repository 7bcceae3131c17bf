"""Where the spectral Jacobian of the half-spectrum path differs from the oracle.
usage: tools/spec_diag.py [n] [kind ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import spectral_oracle as so, vm_oracle as vo
from tests.golden.make_golden import smooth_field
from cfd_julia_amd import spectral
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
kinds = sys.argv[2:] or ["hybrid", "2/3", "3/2"]
KID = {"hybrid": so.HYBRID, "2/3": so.PS23, "3/2": so.PS32}
dx, dy, _, _ = vo.vm_grid(n, n)
f = smooth_field(n, n, 6, n) + 0.01 * np.random.default_rng(n).standard_normal((n, n))
wf = so.to_spectral(f)
k2 = so.wavespace(n, n, dx, dy)
for kind in kinds:
    ref = so.JACOBIANS[KID[kind]](wf, k2, dx, dy)
    for half in ("1", "0"):
        os.environ["CFDJ_SPEC_HALF"] = half
        with spectral.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
            got = h.jacobian(wf)
        d = np.abs(got - ref) / np.abs(ref).max()
        i, j = np.unravel_index(d.argmax(), d.shape)
        print(kind, "half", half, "max err", d.max(), "at", i, j, "ref", ref[i, j], "got", got[i, j])
        bad = d > 1e-11
        print("   entries above 1e-11:", int(bad.sum()), "first-index values:",
              sorted(set(np.nonzero(bad)[0].tolist()))[:12], "second-index values:",
              sorted(set(np.nonzero(bad)[1].tolist()))[:12], flush=True)
