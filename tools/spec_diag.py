"""Where the spectral Jacobian of the half-spectrum path differs from the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import spectral_oracle as so, vm_oracle as vo
from tests.golden.make_golden import smooth_field
from cfd_julia_amd import spectral
n = 1024
dx, dy, _, _ = vo.vm_grid(n, n)
f = smooth_field(n, n, 6, n) + 0.01 * np.random.default_rng(n).standard_normal((n, n))
wf = so.to_spectral(f)
k2 = so.wavespace(n, n, dx, dy)
for kind, kid in (("hybrid", so.HYBRID), ("2/3", so.PS23)):
    ref = so.JACOBIANS[kid](wf, k2, dx, dy)
    for half in ("1", "0"):
        os.environ["CFDJ_SPEC_HALF"] = half
        with spectral.SpectralNS2D(n, n, dx, dy, 1000.0, kind) as h:
            got = h.jacobian(wf)
        d = np.abs(got - ref)
        i, j = np.unravel_index(d.argmax(), d.shape)
        print(kind, "half", half, "max err", d.max() / np.abs(ref).max(), "at", i, j,
              "ref", ref[i, j], "got", got[i, j])
        srt = np.argsort(d.ravel())[::-1][:8]
        print("   worst:", [(int(t % n), int(t // n), float(d.ravel(order='F')[t]) if False else 0) for t in srt][:0],
              [tuple(int(x) for x in np.unravel_index(t, d.shape)) for t in srt])
