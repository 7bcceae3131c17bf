"""CPU tests of config 1 (01_Heat_Equation_FTCS/ftcs.jl): the C ABI's host FTCS against
the NumPy oracle (bit-exact) and the analytic decay (ftcs.jl:26, 44-52)."""
import math

import numpy as np
import pytest

from oracle import misc_oracle as mo


def test_ftcs_bit_exact_vs_oracle():
    from cfd_julia_amd import ftcs

    nx, nt, beta, x, u0, ue = mo.ftcs_setup()
    un = ftcs.ftcs(u0, nt, beta)
    assert np.array_equal(un, mo.ftcs(u0, nt, beta))


@pytest.mark.parametrize("dx,dt", [(0.025, 0.0025), (2.0 / 1024, 2.0 ** -16)])
def test_ftcs_analytic_decay(dx, dt):
    # C1: nx = 1024 needs beta <= 0.5; dt = 2^-16 gives beta = 0.405
    from cfd_julia_amd import ftcs

    l2, linf = ftcs.main(dx=dx, dt=dt, t=1.0 if dx > 0.01 else 0.05)
    assert linf < 5e-3 and l2 < 5e-3


def test_ftcs_argument_errors():
    from cfd_julia_amd import _lib

    with pytest.raises(_lib.ArgumentError):
        _lib.check(_lib.load().cfdj_ftcs(1, 1, 0.4, None, None, 2), "cfdj_ftcs")
