// The vortex-merger RHS arithmetic shared by the marching and the row-group stage kernels
// (vm_kernels.hip) and the spectral solvers' Arakawa kernel (spectral.hip): Arakawa Jacobian
// + 5-point Laplacian (Common.jl:148-181) and the SSP-RK3 stage combinations (vm.jl:28,
// 43-47, 62-66).
//
// Every function body pins `fp contract(off)`: the expressions are evaluated in the
// reference's written order without FMA, so given the same streamfunction the output is
// bit-identical to the CPU oracle (oracle/vm_oracle.py: arakawa_rhs, rk3_step) even inside
// translation units that enable contraction for their FFT code.
#pragma once
#include "cfdj_internal.hpp"

namespace cfdj {

namespace {

constexpr int kWave = 64;

// Four values of one row around a lane's point pair: l = x-1, a = x, b = x+1, r = x+2.
struct Win {
  double l, a, b, r;
};
// A lane's 16-B load of (x, x+1) plus the wave-edge values it alone fetches.
struct Raw {
  double2 c;
  double el, er;
};

__device__ __forceinline__ Raw fetch(const double* row, int xs, int xl, int xr, bool is_l,
                                     bool is_r) {
  Raw r;
  r.c = *reinterpret_cast<const double2*>(row + xs);
  r.el = 0.0;
  r.er = 0.0;
  if (is_l) r.el = row[xl];
  if (is_r) r.er = row[xr];
  return r;
}

// x-1 / x+2 from the neighbouring lanes (the wave edges from the lane's own loads).
__device__ __forceinline__ Win expand(const Raw& raw, bool is_l, bool is_r) {
  Win w;
  w.a = raw.c.x;
  w.b = raw.c.y;
  const double up = __shfl_up(raw.c.y, 1, kWave);    // lane-1's x+1 == my x-1
  const double dn = __shfl_down(raw.c.x, 1, kWave);  // lane+1's x   == my x+2
  w.l = is_l ? raw.el : up;
  w.r = is_r ? raw.er : dn;
  return w;
}

// r = -J(w, s) + (1/re) lap(w) at one point; the argument names are compass directions
// (E = i+1, N = j+1).  Float order of Common.jl:155-180.
__device__ __forceinline__ double arakawa_rhs(double wc, double wE, double wW, double wN,
                                              double wS, double wNE, double wSW, double wNW,
                                              double wSE, double sE, double sW, double sN,
                                              double sS, double sNE, double sSW,
                                              double sNW, double sSE, const StageCoef& k) {
#pragma clang fp contract(off)
  const double j1 = (wE - wW) * (sN - sS) - (wN - wS) * (sE - sW);
  const double j2 =
      wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW);
  const double j3 =
      wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS);
  const double jac = k.gg * (j1 + j2 + j3) * k.hh;
  return -jac + (k.aa * (wE - 2.0 * wc + wW) + k.bb * (wN - 2.0 * wc + wS));
}

template <int STAGE>
__device__ __forceinline__ double stage_update(double r, double wc, double wn,
                                               const StageCoef& k) {
#pragma clang fp contract(off)
  if constexpr (STAGE == 0) {
    return r;
  } else if constexpr (STAGE == 1) {
    return wc + k.dt * r;  // vm.jl:28 (wc is wn here)
  } else if constexpr (STAGE == 2) {
    return (0.75 * wn + 0.25 * wc) + k.c25dt * r;  // vm.jl:43-47
  } else {
    return (wn / 3.0 + k.c23 * wc) + k.c23dt * r;  // vm.jl:62-66
  }
}

// The two outputs of a lane's point pair (x, x+1) of row y from the 3-row windows of omega
// (m = y-1, c = y, p = y+1) and psi.  point x: W = l, C = a, E = b; point x+1: W = a,
// C = b, E = r.
__device__ __forceinline__ void pair_rhs(const Win& wm, const Win& wc, const Win& wp,
                                         const Win& sm, const Win& sc, const Win& sp,
                                         const StageCoef& k, double& r0, double& r1) {
  r0 = arakawa_rhs(wc.a, wc.b, wc.l, wp.a, wm.a, wp.b, wm.l, wp.l, wm.b, sc.b, sc.l, sp.a,
                   sm.a, sp.b, sm.l, sp.l, sm.b, k);
  r1 = arakawa_rhs(wc.b, wc.r, wc.a, wp.b, wm.b, wp.r, wm.a, wp.a, wm.r, sc.r, sc.a, sp.b,
                   sm.b, sp.r, sm.a, sp.a, sm.r, k);
}

}  // namespace

}  // namespace cfdj
