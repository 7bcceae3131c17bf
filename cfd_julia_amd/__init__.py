"""cfd_julia_amd -- MI355X-native (gfx950) implementation of the t-bltg/CFD_Julia 2D
vorticity-streamfunction Navier-Stokes hot path (Arakawa Jacobian + 5-point Laplacian +
SSP-RK3 + FD-FFT Poisson), exposed through the C ABI of `libcfdj.so` (include/cfdj.h).

Modules mirror the reference files they replace:
  common  -- Common.jl (fps, vm_rhs, vm_ic, compute_l2norm*)
  vm      -- 19_NS2D_Vortex_Merger/vm.jl (numerical, main)
  fft_p   -- 12_Poisson_Solver_FFT/fft_p.jl (ps_fft, main)
  fft_s   -- 13_Poisson_Solver_FFT_Spectral/fft_s.jl (ps_spectral)
  fft_d   -- 14_Poisson_Solver_FST/fft_d.jl (ps_fst, main)
  cavity  -- 18_NS2D_Lid_Driven_Cavity/lid_driven_cavity.jl (fps_sine, numerical, main)
  mg      -- 17_Poisson_Solver_Multigrid/mg_N.jl and mg.jl
  solver  -- handle objects (VortexMerger, PoissonFFT)
  dist    -- one-process-per-GPU y-slab driver over RCCL
"""
from ._lib import ArgumentError, CfdjError, load  # noqa: F401
from .solver import PoissonFFT, VortexMerger  # noqa: F401

__version__ = "0.1.0"
