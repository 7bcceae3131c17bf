// Spectral-space NS2D solvers of the reference:
//   20_NS2D_Hybrid_Solver/hybrid.jl                         (CFDJ_SPEC_HYBRID)
//   22_NS2D_PseudoSpectral_23_Rule/pseudospectral_23_rule.jl (CFDJ_SPEC_PS23)
//   21_NS2D_PseudoSpectral_32_Rule/pseudospectral_32_rule.jl (CFDJ_SPEC_PS32)
//
// All three advance the vorticity spectrum w_f with the same low-storage RK3 /
// Crank-Nicolson loop (hybrid.jl:41-67) and differ in the Jacobian jf = fft(-J(w, psi)).
//
// The reference holds full complex nx x ny spectra and never assumes Hermitian symmetry (its
// kx[1] = eps and its Nyquist derivatives are not odd, the 2/3 rule's zero band is not
// symmetric) but takes real(ifft(.)) of everything, which keeps exactly the Hermitian part.
// Three transform paths, the same results to FFT round-off:
//   * square power-of-two grids of 1024..8192, hybrid and 2/3 rule: the state is the HALF
//     spectrum (kx index 0..nx/2, ky contiguous) and the transforms are real (fft2d_r2c.hip;
//     its column pass forms that Hermitian part from the half spectrum);
//   * other power-of-two grids of 256..4096 (or CFDJ_SPEC_HALF=0): full spectra, the
//     hand-written two-pass complex transform (fft2d_c2c.hip), real physical-space fields;
//   * the 3/2 rule's padded product grid: rocFFT REAL transforms on the half spectrum of the
//     padded grid (any even grid; CFDJ_SPEC_REAL=0: complex);
//   * everything else: rocFFT complex-to-complex.
// The C interface always speaks the reference's layout: complex nx x ny, kx contiguous.
//
// Per Jacobian evaluation (one RK3 substep):
//   hybrid: [w_f, w_f / k2] -> batch-2 inverse c2c -> Arakawa stencil on the real parts
//           (hybrid.jl:129-150, per-term gg) -> forward c2c;
//   2/3:    psi_x, w_y, psi_y, w_x spectra with the 2/3-rule modes zeroed -> batch-4
//           inverse c2c -> psi_x w_y - psi_y w_x -> forward c2c;
//   3/2:    the same four spectra zero-padded to (3nx/2) x (3ny/2) by quadrant copies,
//           scaled by (nxe nye)/(nx ny) -> batch-4 inverse c2c -> product -> forward c2c
//           -> quadrants back, scaled by (nx ny)/(nxe nye).
// Elementwise arithmetic follows the source order (Julia Real*Complex and Complex/Real
// act componentwise), built with -ffp-contract=off like the rest of the library.
#include <cmath>
#include <memory>

#include "host_common.hpp"
#include "stencil.hpp"

namespace cfdj {

namespace {

struct SpecDims {
  int nx, ny;        // spectral grid
  int px, py;        // transform grid of the products (padded for the 3/2 rule)
  double inv_n;      // 1 / (nx ny)      (real(ifft) scale on the nx x ny grid)
  double inv_np;     // 1 / (px py)
};

__device__ __forceinline__ double2 cmul_r(double a, double2 e) { return make_double2(a * e.x, a * e.y); }
__device__ __forceinline__ double2 cdiv_r(double2 e, double d) { return make_double2(e.x / d, e.y / d); }
__device__ __forceinline__ double2 times_i(double2 e) { return make_double2(-e.y, e.x); }

// complex(w, 0) of a pitched real nx x ny block (hybrid.jl:24).
__global__ void to_complex_kernel(const double* __restrict__ w, long ldw, double2* __restrict__ out,
                                  int nx, int ny) {
  const size_t n = (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    out[t] = make_double2(w[(size_t)j * ldw + i], 0.0);
  }
}

// hybrid.jl:103,115: X0 = w_f (for w), X1 = w_f / k2 (for psi).
__global__ void hybrid_prep_kernel(const double2* __restrict__ wf, const double* __restrict__ kx,
                                   double2* __restrict__ X, int nx, int ny) {
  const size_t n = (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    const double k2 = kx[i] * kx[i] + kx[j] * kx[j];
    const double2 v = wf[t];
    X[t] = v;
    X[n + t] = cdiv_r(v, k2);
  }
}

// hybrid.jl:129-150 on the periodic grid: data = complex(-(j1 + j2 + j3) * hh, 0) with
// w = Re(X0) / N, s = Re(X1) / N (real(ifft)).
__global__ void hybrid_jac_kernel(const double2* __restrict__ X, double2* __restrict__ J, int nx,
                                  int ny, double inv_n, double gg, double hh) {
  const size_t n = (size_t)nx * ny;
  const double2* S = X + n;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    const int ie = i + 1 == nx ? 0 : i + 1, iw = i == 0 ? nx - 1 : i - 1;
    const int jn = j + 1 == ny ? 0 : j + 1, js = j == 0 ? ny - 1 : j - 1;
    auto W = [&](int a, int b) { return X[(size_t)b * nx + a].x * inv_n; };
    auto P = [&](int a, int b) { return S[(size_t)b * nx + a].x * inv_n; };
    const double wE = W(ie, j), wW = W(iw, j), wN = W(i, jn), wS = W(i, js);
    const double wNE = W(ie, jn), wSW = W(iw, js), wNW = W(iw, jn), wSE = W(ie, js);
    const double sE = P(ie, j), sW = P(iw, j), sN = P(i, jn), sS = P(i, js);
    const double sNE = P(ie, jn), sSW = P(iw, js), sNW = P(iw, jn), sSE = P(ie, js);
    const double j1 = gg * ((wE - wW) * (sN - sS) - (wN - wS) * (sE - sW));
    const double j2 =
        gg * (wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW));
    const double j3 =
        gg * (wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS));
    J[t] = make_double2(-(j1 + j2 + j3) * hh, 0.0);
  }
}

// The same on real fields (w = Rw / N, s = Rs / N), real result: the hand-written
// transforms hand over real(ifft(.)) as real arrays and take the product as one.
__global__ void hybrid_jac_real_kernel(const double* __restrict__ Rw,
                                       const double* __restrict__ Rs, double* __restrict__ Rj,
                                       int nx, int ny, double inv_n, double gg, double hh) {
  const size_t n = (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    const int ie = i + 1 == nx ? 0 : i + 1, iw = i == 0 ? nx - 1 : i - 1;
    const int jn = j + 1 == ny ? 0 : j + 1, js = j == 0 ? ny - 1 : j - 1;
    auto W = [&](int a, int b) { return Rw[(size_t)b * nx + a] * inv_n; };
    auto P = [&](int a, int b) { return Rs[(size_t)b * nx + a] * inv_n; };
    const double wE = W(ie, j), wW = W(iw, j), wN = W(i, jn), wS = W(i, js);
    const double wNE = W(ie, jn), wSW = W(iw, js), wNW = W(iw, jn), wSE = W(ie, js);
    const double sE = P(ie, j), sW = P(iw, j), sN = P(i, jn), sS = P(i, js);
    const double sNE = P(ie, jn), sSW = P(iw, js), sNW = P(iw, jn), sSE = P(ie, js);
    const double j1 = gg * ((wE - wW) * (sN - sS) - (wN - wS) * (sE - sW));
    const double j2 =
        gg * (wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW));
    const double j3 =
        gg * (wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS));
    Rj[t] = -(j1 + j2 + j3) * hh;
  }
}

// hybrid.jl:136-146 at one point (compass names: E = i+1, N = j+1), per-term gg.
__device__ __forceinline__ double hybrid_jac_point(double wE, double wW, double wN, double wS,
                                                   double wNE, double wSW, double wNW,
                                                   double wSE, double sE, double sW, double sN,
                                                   double sS, double sNE, double sSW,
                                                   double sNW, double sSE, double gg,
                                                   double hh) {
  const double j1 = gg * ((wE - wW) * (sN - sS) - (wN - wS) * (sE - sW));
  const double j2 =
      gg * (wE * (sNE - sSE) - wW * (sNW - sSW) - wN * (sNE - sNW) + wS * (sSE - sSW));
  const double j3 =
      gg * (wNE * (sN - sE) - wSW * (sW - sS) - wNW * (sN - sW) + wSE * (sE - sS));
  return -(j1 + j2 + j3) * hh;
}

// The same as hybrid_jac_real_kernel in the shape of the vortex-merger row-group stage kernel
// (vm_kernels.hip): a 256-thread workgroup owns 512 consecutive x of 2 consecutive rows, two
// x per lane, the 4 rows it needs loaded at once (16 B per lane); workgroups in row-major
// order, so the three streams advance through HBM sequentially.  x-neighbours by lane
// shuffles, across wavefronts through LDS, the workgroup's two periodic halo columns by one
// masked load.  nx a multiple of 512, ny even.
__global__ __launch_bounds__(256) void hybrid_jac_tile_kernel(const double* __restrict__ Rw,
                                                              const double* __restrict__ Rs,
                                                              double* __restrict__ Rj, int nx,
                                                              int ny, double inv_n, double gg,
                                                              double hh) {
  constexpr int G = 2, NR = G + 2, NW = 256 / kWave, TC = 512, XCDS = 8;
  __shared__ double left[NW][2 * NR], right[NW][2 * NR];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int strips = nx / TC;
  // workgroup b runs on XCD b % 8; the row groups above and below share halo rows and should
  // meet in one L2: automatic for 8 strips, else XCD (strip, band) walks a band of rows
  int strip = blockIdx.x % strips, grp = blockIdx.x / strips;
  if (strips < XCDS && XCDS % strips == 0) {
    const int bands = XCDS / strips, ngrp = ny / G;
    if (ngrp % bands == 0) {
      const int xcd = blockIdx.x % XCDS, i = blockIdx.x / XCDS;
      strip = xcd % strips;
      grp = (xcd / strips) * (ngrp / bands) + i;
    }
  }
  const int x0 = strip * TC, x = x0 + 2 * (int)threadIdx.x, y0 = grp * G;
  auto row = [&](const double* a, int y) {
    return a + (size_t)(y < 0 ? y + ny : (y >= ny ? y - ny : y)) * nx;
  };
  double2 wv[NR], sv[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    wv[j] = *reinterpret_cast<const double2*>(row(Rw, y0 - 1 + j) + x);
    sv[j] = *reinterpret_cast<const double2*>(row(Rs, y0 - 1 + j) + x);
  }
  static_assert(4 * NR <= kWave, "halo fetch needs one lane per value");
  double halo = 0.0;
  const int side = threadIdx.x / (2 * NR), rem = threadIdx.x % (2 * NR);
  if (threadIdx.x < 4 * NR) {
    const int xh = side == 0 ? (x0 == 0 ? nx - 1 : x0 - 1) : (x0 + TC >= nx ? x0 + TC - nx : x0 + TC);
    halo = row((rem & 1) ? Rs : Rw, y0 - 1 + rem / 2)[xh];
  }
  if ((lane == 0 && wave > 0) || (lane == kWave - 1 && wave < NW - 1)) {
    double* e = lane == 0 ? right[wave - 1] : left[wave + 1];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      e[2 * j] = lane == 0 ? wv[j].x : wv[j].y;
      e[2 * j + 1] = lane == 0 ? sv[j].x : sv[j].y;
    }
  }
  if (threadIdx.x < 4 * NR) (side == 0 ? left[0] : right[NW - 1])[rem] = halo;
  __syncthreads();
  Win ww[NR], sw[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    ww[j].l = __shfl_up(wv[j].y, 1, kWave);
    ww[j].r = __shfl_down(wv[j].x, 1, kWave);
    sw[j].l = __shfl_up(sv[j].y, 1, kWave);
    sw[j].r = __shfl_down(sv[j].x, 1, kWave);
    if (lane == 0) {
      ww[j].l = left[wave][2 * j];
      sw[j].l = left[wave][2 * j + 1];
    }
    if (lane == kWave - 1) {
      ww[j].r = right[wave][2 * j];
      sw[j].r = right[wave][2 * j + 1];
    }
    // w = real(ifft(.)): the transform's output times 1 / (nx ny)
    ww[j] = Win{ww[j].l * inv_n, wv[j].x * inv_n, wv[j].y * inv_n, ww[j].r * inv_n};
    sw[j] = Win{sw[j].l * inv_n, sv[j].x * inv_n, sv[j].y * inv_n, sw[j].r * inv_n};
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const Win &wm = ww[j], &wc = ww[j + 1], &wp = ww[j + 2];
    const Win &sm = sw[j], &sc = sw[j + 1], &sp = sw[j + 2];
    double2 o;
    o.x = hybrid_jac_point(wc.b, wc.l, wp.a, wm.a, wp.b, wm.l, wp.l, wm.b, sc.b, sc.l, sp.a,
                           sm.a, sp.b, sm.l, sp.l, sm.b, gg, hh);
    o.y = hybrid_jac_point(wc.r, wc.a, wp.b, wm.b, wp.r, wm.a, wp.a, wm.r, sc.r, sc.a, sp.b,
                           sm.b, sp.r, sm.a, sp.a, sm.r, gg, hh);
    *reinterpret_cast<double2*>(Rj + (size_t)(y0 + j) * nx + x) = o;
  }
}

// pseudospectral_*.jl:109-122 derivatives of w_f, placed on the px x py product grid:
//   2/3 rule (px = nx): modes i in [nxe/2, nx - nxe/2) or j in [nye/2, ny - nye/2) zeroed
//           (pseudospectral_23_rule.jl:124-133, 0-based);
//   3/2 rule (px = 3nx/2): quadrant copies (pseudospectral_32_rule.jl:124-154), everything
//           else zero, times (nxe nye) then divided by (nx ny).
// One thread per element of the px x py grid; batch b of D is j_{b+1} f.
__global__ void ps_derivs_kernel(const double2* __restrict__ wf, const double* __restrict__ kx,
                                 double2* __restrict__ D, int nx, int ny, int px, int py,
                                 int rule32, int tx0, int tx1, int ty0, int ty1, double sc,
                                 double sd) {
  const size_t np = (size_t)px * py;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < np;
       t += (size_t)gridDim.x * blockDim.x) {
    const int a = (int)(t % px), b = (int)(t / px);
    int i = a, j = b;
    bool keep;
    if (rule32) {
      const int hx = nx / 2, hy = ny / 2, qx = px - hx, qy = py - hy;
      keep = (a < hx || a >= qx) && (b < hy || b >= qy);
      i = a < hx ? a : a - qx + hx;
      j = b < hy ? b : b - qy + hy;
    } else {
      keep = !(a >= tx0 && a < tx1) && !(b >= ty0 && b < ty1);
    }
    double2 d1 = make_double2(0.0, 0.0), d2 = d1, d3 = d1, d4 = d1;
    if (keep) {
      const double kxi = kx[i], kyj = kx[j];
      const double k2 = kxi * kxi + kyj * kyj;
      const double2 iw = times_i(wf[(size_t)j * nx + i]);
      d1 = cdiv_r(cmul_r(kxi, iw), k2);  // 1im * wf * kx / k2
      d4 = cmul_r(kxi, iw);              // 1im * wf * kx
      d2 = cmul_r(kyj, iw);              // 1im * wf * ky
      d3 = cdiv_r(cmul_r(kyj, iw), k2);  // 1im * wf * ky / k2
      if (rule32) {
        d1 = make_double2(d1.x * sc / sd, d1.y * sc / sd);
        d2 = make_double2(d2.x * sc / sd, d2.y * sc / sd);
        d3 = make_double2(d3.x * sc / sd, d3.y * sc / sd);
        d4 = make_double2(d4.x * sc / sd, d4.y * sc / sd);
      }
    }
    D[t] = d1;
    D[np + t] = d2;
    D[2 * np + t] = d3;
    D[3 * np + t] = d4;
  }
}

// jacp = j1 j2 - j3 j4 with j_k = real(ifft(.)) = Re(D_k) / (px py).
__global__ void ps_product_kernel(const double2* __restrict__ D, double2* __restrict__ J, size_t np,
                                  double inv_np) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < np;
       t += (size_t)gridDim.x * blockDim.x) {
    const double j1 = D[t].x * inv_np, j2 = D[np + t].x * inv_np;
    const double j3 = D[2 * np + t].x * inv_np, j4 = D[3 * np + t].x * inv_np;
    J[t] = make_double2(j1 * j2 - j3 * j4, 0.0);
  }
}

// ... on real fields (the four real(ifft(.)) as real arrays), real product.
template <bool NT>
__global__ void ps_product_real_kernel(const double* __restrict__ D, double* __restrict__ Rj,
                                       size_t np, double inv_np) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < np;
       t += (size_t)gridDim.x * blockDim.x) {
    // the four fields are read once: streaming loads (the product stays cached for the
    // forward transform)
    const double j1 = load_stream<NT>(D + t) * inv_np, j2 = load_stream<NT>(D + np + t) * inv_np;
    const double j3 = load_stream<NT>(D + 2 * np + t) * inv_np;
    const double j4 = load_stream<NT>(D + 3 * np + t) * inv_np;
    Rj[t] = j1 * j2 - j3 * j4;
  }
}

// pseudospectral_32_rule.jl:171-178: quadrants of the padded product spectrum, * (nx ny)
// / (nxe nye).
__global__ void ps_unpad_kernel(const double2* __restrict__ Jp, double2* __restrict__ jf, int nx,
                                int ny, int px, int py, double sd, double sc) {
  const size_t n = (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    const int hx = nx / 2, hy = ny / 2;
    const int a = i < hx ? i : i - hx + (px - hx), b = j < hy ? j : j - hy + (py - hy);
    const double2 v = Jp[(size_t)b * px + a];
    jf[t] = make_double2(v.x * sd / sc, v.y * sd / sc);
  }
}

// The 3/2 rule on the half spectrum of its padded grid (library real transforms): element
// (a, b), a <= px/2, of the four padded derivative spectra, as the Hermitian part
// (P(a, b) + conj P(-a, -b)) / 2 that real(ifft(.)) keeps of the reference's padded array P
// (pseudospectral_32_rule.jl:109-154: corner blocks of i k w_f (/ k2), times (nxe nye) /
// (nx ny); the -nx/2 modes sit on the negative side only, kx[1] = eps is not odd -- P is not
// Hermitian).  D: 4 arrays of (px/2 + 1) x py, x contiguous.
template <bool NT>  // the four spectra (1.2 GB at 4096^2) by streaming stores
__global__ void ps32_derivs_half_kernel(const double2* __restrict__ wf,
                                        const double* __restrict__ kx, double2* __restrict__ D,
                                        int nx, int ny, int px, int py, double sc, double sd) {
  const int pxh = px / 2 + 1;
  const size_t nh = (size_t)pxh * py;
  const int hx = nx / 2, hy = ny / 2, qx = px - hx, qy = py - hy;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < nh;
       t += (size_t)gridDim.x * blockDim.x) {
    const int a0 = (int)(t % pxh), b0 = (int)(t / pxh);
    double2 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = make_double2(0.0, 0.0);
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int a = side ? (a0 == 0 ? 0 : px - a0) : a0, b = side ? (b0 == 0 ? 0 : py - b0) : b0;
      if (!((a < hx || a >= qx) && (b < hy || b >= qy))) continue;
      const int i = a < hx ? a : a - qx + hx, j = b < hy ? b : b - qy + hy;
      const double kxi = kx[i], kyj = kx[j];
      const double k2 = kxi * kxi + kyj * kyj;
      const double2 iw = times_i(wf[(size_t)j * nx + i]);
      double2 d[4];
      d[0] = cdiv_r(cmul_r(kxi, iw), k2);  // 1im * wf * kx / k2
      d[1] = cmul_r(kyj, iw);              // 1im * wf * ky
      d[2] = cdiv_r(cmul_r(kyj, iw), k2);  // 1im * wf * ky / k2
      d[3] = cmul_r(kxi, iw);              // 1im * wf * kx
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double2 p = make_double2(d[q].x * sc / sd, d[q].y * sc / sd);
        acc[q].x += 0.5 * p.x;
        acc[q].y += side ? -0.5 * p.y : 0.5 * p.y;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) store_stream<NT>(D + q * nh + t, acc[q]);
  }
}

// The same four spectra in the column layout of the hand-written 3 * 2^k transforms
// (fft2d_r2c3.hip): columns a = 0..nx/2 only (beyond, the padded spectrum is zero), element
// (a, b) of array q at (q (nx/2 + 1) + a) py + b, ky contiguous.  w_f is read along kx and the
// result written along ky, through a 16 x 16 tile in LDS; one 256-thread workgroup per tile,
// grid = (ceil((nx/2 + 1) / 16), py / 16).
__global__ __launch_bounds__(256) void ps32_derivs_cols_kernel(
    const double2* __restrict__ wf, const double* __restrict__ kx, double2* __restrict__ D,
    int nx, int ny, int px, int py, double sc, double sd) {
  __shared__ double2 tile[4][16][17];
  const int hx = nx / 2, hy = ny / 2, qx = px - hx, qy = py - hy, ncol = hx + 1;
  const int ta = threadIdx.x & 15, tb = threadIdx.x >> 4;
  const int a0 = blockIdx.x * 16 + ta, b0 = blockIdx.y * 16 + tb;
  double2 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = make_double2(0.0, 0.0);
  if (a0 < ncol) {
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int a = side ? (a0 == 0 ? 0 : px - a0) : a0, b = side ? (b0 == 0 ? 0 : py - b0) : b0;
      if (!((a < hx || a >= qx) && (b < hy || b >= qy))) continue;
      const int i = a < hx ? a : a - qx + hx, j = b < hy ? b : b - qy + hy;
      const double kxi = kx[i], kyj = kx[j];
      const double k2 = kxi * kxi + kyj * kyj;
      const double2 iw = times_i(wf[(size_t)j * nx + i]);
      double2 d[4];
      d[0] = cdiv_r(cmul_r(kxi, iw), k2);  // 1im * wf * kx / k2
      d[1] = cmul_r(kyj, iw);              // 1im * wf * ky
      d[2] = cdiv_r(cmul_r(kyj, iw), k2);  // 1im * wf * ky / k2
      d[3] = cmul_r(kxi, iw);              // 1im * wf * kx
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double2 p = make_double2(d[q].x * sc / sd, d[q].y * sc / sd);
        acc[q].x += 0.5 * p.x;
        acc[q].y += side ? -0.5 * p.y : 0.5 * p.y;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) tile[q][ta][tb] = acc[q];
  __syncthreads();
  const int wa = blockIdx.x * 16 + tb, wb = blockIdx.y * 16 + ta;  // ky fastest on the way out
  if (wa < ncol) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      D[((size_t)q * ncol + wa) * py + wb] = tile[q][tb][ta];
  }
}

// pseudospectral_32_rule.jl:171-178 from the columns 0..nx/2 of the product's spectrum in that
// layout (Jc, element (a, b) at a py + b): jf(i, j) = fft(product)(a, b) (nx ny) / (nxe nye);
// kx indices i >= nx/2 are the conjugates of (-a, -b).  Read along ky, written along kx
// through a 16 x 16 tile; grid = (nx / 16, ny / 16).
__global__ __launch_bounds__(256) void ps32_unpad_cols_kernel(const double2* __restrict__ Jc,
                                                              double2* __restrict__ jf, int nx,
                                                              int ny, int px, int py, double sd,
                                                              double sc) {
  __shared__ double2 tile[16][17];
  const int hx = nx / 2, hy = ny / 2;
  const int tj = threadIdx.x & 15, ti = threadIdx.x >> 4;  // ky fastest on the way in
  {
    const int i = blockIdx.x * 16 + ti, j = blockIdx.y * 16 + tj;
    const int a = i < hx ? i : i - hx + (px - hx), b = j < hy ? j : j - hy + (py - hy);
    double2 v;
    if (i < hx) {
      v = Jc[(size_t)a * py + b];
    } else {
      v = Jc[(size_t)(px - a) * py + (b == 0 ? 0 : py - b)];
      v.y = -v.y;
    }
    tile[ti][tj] = make_double2(v.x * sd / sc, v.y * sd / sc);
  }
  __syncthreads();
  const int wi = blockIdx.x * 16 + tj, wj = blockIdx.y * 16 + ti;
  jf[(size_t)wj * nx + wi] = tile[tj][ti];
}

// pseudospectral_32_rule.jl:171-178 from the half spectrum Jh ((px/2 + 1) x py) of the real
// product: jf(i, j) = fft(product)(a, b) * (nx ny) / (nxe nye), (a, b) the padded index of
// mode (i, j); a > px/2 is the conjugate of (-a, -b).
__global__ void ps32_unpad_half_kernel(const double2* __restrict__ Jh, double2* __restrict__ jf,
                                       int nx, int ny, int px, int py, double sd, double sc) {
  const size_t n = (size_t)nx * ny;
  const int pxh = px / 2 + 1;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    const int hx = nx / 2, hy = ny / 2;
    const int a = i < hx ? i : i - hx + (px - hx), b = j < hy ? j : j - hy + (py - hy);
    double2 v;
    if (a < pxh) {
      v = Jh[(size_t)b * pxh + a];
    } else {
      v = Jh[(size_t)(b == 0 ? 0 : py - b) * pxh + (px - a)];
      v.y = -v.y;
    }
    jf[t] = make_double2(v.x * sd / sc, v.y * sd / sc);
  }
}

// hybrid.jl:44-67, one RK3 / Crank-Nicolson substep.  z = .5dt k2 / re, d = alpha z;
// out = ((1 - d)/(1 + d)) * w + (cA * jA + cB * jB) / (1 + d)   (stage 1: cB = 0, no jB);
// out[1,1] = 0 after stages 1 and 2.
// HALF: the arrays are half spectra ((nx/2 + 1) columns of ny, ky contiguous), followed by
// `extra` elements of the modes (-m, ny/2), m = 0..extra-1 (the 3/2 rule's state; k2 is even).
template <int STAGE, bool HALF, bool NT>
__global__ void cn_update_kernel(const double2* __restrict__ w, const double2* __restrict__ jA,
                                 const double2* __restrict__ jB, double2* __restrict__ out,
                                 const double* __restrict__ kx, int nx, int ny, double hdt,
                                 double re, double alpha, double cA, double cB, int extra) {
  const size_t nh = (size_t)(nx / 2 + 1) * ny;
  const size_t n = HALF ? nh + extra : (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    int i = HALF ? (int)(t / ny) : (int)(t % nx), j = HALF ? (int)(t % ny) : (int)(t / nx);
    if (HALF && t >= nh) {
      i = (int)(t - nh);
      j = ny / 2;
    }
    const double k2 = kx[i] * kx[i] + kx[j] * kx[j];
    const double z = hdt * k2 / re;
    const double d = alpha * z;
    const double g = (1.0 - d) / (1.0 + d);
    const double e = 1.0 + d;
    // each read once and not again before the next transforms: streaming loads
    const double2 wv = load_stream<NT>(w + t);
    double2 f = cmul_r(cA, load_stream<NT>(jA + t));
    if constexpr (STAGE >= 2) {
      const double2 fb = cmul_r(cB, load_stream<NT>(jB + t));
      f = make_double2(f.x + fb.x, f.y + fb.y);
    }
    double2 o = make_double2(g * wv.x + f.x / e, g * wv.y + f.y / e);
    if (STAGE <= 2 && t == 0) o = make_double2(0.0, 0.0);
    out[t] = o;
  }
}

// hybrid.jl:71-76: ut[1:nx,1:ny] = real(ifft(w_f)), ut[nx+1,:] = ut[1,:], ut[:,ny+1] = ut[:,1];
// written into a pitched (nx+1) x (ny+1) block.
__global__ void to_field_kernel(const double2* __restrict__ X, double* __restrict__ ut, long ldu,
                                int nx, int ny, double inv_n) {
  const size_t n = (size_t)(nx + 1) * (ny + 1);
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % (nx + 1)), j = (int)(t / (nx + 1));
    const int a = i == nx ? 0 : i, b = j == ny ? 0 : j;
    ut[(size_t)j * ldu + i] = X[(size_t)b * nx + a].x * inv_n;
  }
}

// ... from a real nx x ny array R = real(ifft(.)) * (nx ny).
__global__ void to_field_real_kernel(const double* __restrict__ R, double* __restrict__ ut,
                                     long ldu, int nx, int ny, double inv_n) {
  const size_t n = (size_t)(nx + 1) * (ny + 1);
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % (nx + 1)), j = (int)(t / (nx + 1));
    const int a = i == nx ? 0 : i, b = j == ny ? 0 : j;
    ut[(size_t)j * ldu + i] = R[(size_t)b * nx + a] * inv_n;
  }
}

// Full spectrum (nx x ny, kx contiguous) <-> half spectrum ((nx/2 + 1) columns of ny, ky
// contiguous) of a real field: the other half is conj(w_f(-kx, -ky)).  HERM: the import keeps
// the Hermitian part (w_f(k) + conj(w_f(-k))) / 2 of whatever it is given -- all that
// hybrid.jl's jacobian() sees of w_f through real(ifft(w_f)) and real(ifft(w_f / k2))
// (hybrid.jl:103,115; k2 is even) -- so a spectrum that is not that of a real field gives the
// reference's Jacobian.  The pseudospectral rules multiply by i k and a band filter that are
// not Hermitian at index 1 (kx[1] = eps) and on the filter's edge, where the other part
// matters too: their import takes the columns as they are (exact for real fields' spectra).
// `extra` (the 3/2 rule's state): the half spectrum is followed by the row w_f(-m, ny/2),
// m = 0..nx/2, which that solver's spectra do not share with their other half.
template <bool HERM>
__global__ void full_to_half_kernel(const double2* __restrict__ full, double2* __restrict__ hs,
                                    int nx, int ny, int extra) {
  const size_t n = (size_t)(nx / 2 + 1) * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n + extra;
       t += (size_t)gridDim.x * blockDim.x) {
    if (t >= n) {
      const int m = (int)(t - n);
      hs[t] = full[(size_t)(ny / 2) * nx + (m == 0 ? 0 : nx - m)];
      continue;
    }
    const int m = (int)(t / ny), k = (int)(t % ny);
    const double2 a = full[(size_t)k * nx + m];
    if constexpr (HERM) {
      const double2 b = full[(size_t)(k == 0 ? 0 : ny - k) * nx + (m == 0 ? 0 : nx - m)];
      hs[t] = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
    } else {
      hs[t] = a;
    }
  }
}
// The same projection on the full layout: out(k) = (full(k) + conj(full(-k))) / 2.
__global__ void hermitian_part_kernel(const double2* __restrict__ full,
                                      double2* __restrict__ out, int nx, int ny) {
  const size_t n = (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    const double2 a = full[t];
    const double2 b = full[(size_t)(j == 0 ? 0 : ny - j) * nx + (i == 0 ? 0 : nx - i)];
    out[t] = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
  }
}
__global__ void half_to_full_kernel(const double2* __restrict__ hs, double2* __restrict__ full,
                                    int nx, int ny, int extra) {
  const size_t n = (size_t)nx * ny;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n;
       t += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % nx), j = (int)(t / nx);
    if (i <= nx / 2) {
      full[t] = hs[(size_t)i * ny + j];
    } else if (extra && j == ny / 2) {
      full[t] = hs[(size_t)(nx / 2 + 1) * ny + (nx - i)];
    } else {
      const double2 v = hs[(size_t)(nx - i) * ny + (j == 0 ? 0 : ny - j)];
      full[t] = make_double2(v.x, -v.y);
    }
  }
}

// The 3/2 rule's extra row of a REAL field's half spectrum: ex[m] = w_f(-m, ny/2) =
// conj(w_f(m, ny/2)).
__global__ void ps32_fill_extra_kernel(double2* __restrict__ hs, int nx, int ny) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m > nx / 2) return;
  const double2 v = hs[(size_t)m * ny + ny / 2];
  hs[(size_t)(nx / 2 + 1) * ny + m] = make_double2(v.x, -v.y);
}
// ... and what real(ifft(.)) keeps of a state whose row ky index ny/2 is not Hermitian:
// (w_f(m, ny/2) + conj(w_f(-m, ny/2))) / 2 in place of w_f(m, ny/2), 0 < m < nx/2 (the columns
// 0 and nx/2 are projected by the transform itself).
__global__ void ps32_project_row_kernel(double2* __restrict__ hs, int nx, int ny) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m <= 0 || m >= nx / 2) return;
  const double2 a = hs[(size_t)m * ny + ny / 2], b = hs[(size_t)(nx / 2 + 1) * ny + m];
  hs[(size_t)m * ny + ny / 2] = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
}

unsigned grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 65536) b = 65536;
  return (unsigned)(b ? b : 1);
}

}  // namespace

}  // namespace cfdj

using namespace cfdj;

struct cfdj_spec {
  int kind = CFDJ_SPEC_HYBRID;
  int nx = 0, ny = 0, px = 0, py = 0;
  double dx = 0, dy = 0, re = 0, eps = 0;
  int device = -1;
  hipStream_t stream = nullptr;
  double* kx = nullptr;
  double2 *wn = nullptr, *w1 = nullptr, *w2 = nullptr;   // spectra of the RK3 loop
  double2 *jn = nullptr, *j1 = nullptr, *j2 = nullptr;   // Jacobians
  double2* X = nullptr;   // hybrid: [w_f, w_f/k2]; PS: 4 derivative spectra (px x py)
  double2* J = nullptr;   // product grid (px x py): physical product -> its spectrum
  double* field = nullptr;  // (nx+1) x (ny+1) download staging
  Plans plans;
  rocfft_plan fwd = nullptr, inv = nullptr;      // nx x ny, batch 1 (in place)
  rocfft_plan inv_b = nullptr, fwd_p = nullptr;  // product grid: batch 2 / 4 inverse, forward
  // hand-written two-pass transform (fft2d_c2c.hip) on power-of-two grids; the library
  // plans above stay for the other sizes and for CFDJ_SPEC_FFT=rocfft
  bool hand_n = false, hand_p = false;           // nx x ny / px x py
  double2 *tw_n = nullptr, *tw_p = nullptr;      // twiddle tables (nx == ny, px == py)
  int nb = 2;                                    // arrays in X
  // physical-space fields of the hand-written path: nb real(ifft(.)) arrays and the
  // real product (real_fields: CFDJ_SPEC_REAL=0 keeps them complex)
  double *R = nullptr, *Rj = nullptr;
  bool real_fields = false;
  // half-spectrum state (fft2d_r2c.hip; square power-of-two grids of 1024..8192: hybrid and
  // 2/3 rule, and the 3/2 rule where hand32 below holds): every spectrum above holds the modes
  // kx index 0..nx/2 only, ky contiguous; the C interface converts (CFDJ_SPEC_HALF=0 keeps the
  // full spectra)
  bool half = false;
  bool stream_loads = false;  // fields beyond the last-level cache: load_stream
  // 3/2 rule: library REAL transforms on the padded grid (half the work of the complex
  // ones; any even grid); CFDJ_SPEC_REAL=0 or CFDJ_SPEC_FFT=rocfft keep the complex plans
  bool real32 = false;
  rocfft_plan inv_r = nullptr, fwd_r = nullptr;  // Z2D batch 4, D2Z on px x py
  // ... or, on product grids of 1536 / 3072 / 6144 points a side, the hand-written
  // 3 * 2^k transforms on the columns 0..nx/2 of that half spectrum (fft2d_r2c3.hip;
  // CFDJ_SPEC_PS32_HAND=0 keeps the library)
  bool hand32 = false;
  bool fuse32 = true;  // CFDJ_SPEC_PS32_FUSE=0: the product as a kernel of its own
  bool fuse23 = false;  // the same for the 2/3 rule on the half spectrum (CFDJ_SPEC_PS23_FUSE=0)
  Real2d3Args a3{};
  Ps32HalfArgs s3{};
  double2 *tw3_l3 = nullptr, *tw3_l = nullptr, *tw3_n = nullptr, *tw3_m3 = nullptr;
  Fused fz;
  HalfSpecArgs ha{};
  size_t nh() const { return (size_t)(nx / 2 + 1) * ny; }
  // the 3/2 rule's half-spectrum state carries the row w_f(-m, ny/2) behind the columns
  int extra() const { return half && kind == CFDJ_SPEC_PS32 ? nx / 2 + 1 : 0; }

  // In-place 2-D transform of `batch` arrays: the library plan `pl` or the hand-written one.
  void fft2(rocfft_plan pl, double2* buf, bool product_grid, int batch, int dir) {
    const bool hand = product_grid ? hand_p : hand_n;
    if (hand) {
      const int gx = product_grid ? px : nx, gy = product_grid ? py : ny;
      const double2* tw = product_grid ? tw_p : tw_n;
      launch_c2c2d(buf, gx, gy, batch, dir, tw, tw, stream);
    } else {
      plans.exec(pl, buf, nullptr);
    }
  }

  size_t n() const { return (size_t)nx * ny; }
  size_t np() const { return (size_t)px * py; }

  // Rj = j1 j2 - j3 j4 of the four real fields in R.
  void product_real(unsigned gb, double inv_np) {
    if (stream_loads)
      hipLaunchKernelGGL(ps_product_real_kernel<true>, dim3(gb), dim3(256), 0, stream, R, Rj,
                         np(), inv_np);
    else
      hipLaunchKernelGGL(ps_product_real_kernel<false>, dim3(gb), dim3(256), 0, stream, R, Rj,
                         np(), inv_np);
  }

  // jf = fft(-J(w, psi)) of the spectrum wf (hybrid.jl:92-152 / pseudospectral_*.jl).
  void jacobian(const double2* wf, double2* jf) {
    const unsigned gb = grid_for(np());
    if (half) {
      // both inverse transforms' inputs are formed inside their column pass; X is the
      // column-pass scratch of both directions
      if (kind == CFDJ_SPEC_HYBRID) {
        launch_half_c2r2d(ha, kHalfHybrid, wf, X, R, stream);
        // half2d_supported: nx a multiple of 512, ny even
        hipLaunchKernelGGL(hybrid_jac_tile_kernel, dim3((nx / 512) * (ny / 2)), dim3(256), 0,
                           stream, R, R + n(), Rj, nx, ny, 1.0 / ((double)nx * ny),
                           1.0 / (4.0 * dx * dy), 1.0 / 3.0);
      } else if (kind == CFDJ_SPEC_PS32) {
        // padding, derivative factors and unpadding inside the column passes of the padded grid
        const double inv_np = 1.0 / ((double)px * py);
        if (fuse32) {  // the fourth field's rows, the product and its row transform in one kernel
          launch_ps32_c2r2d3(a3, s3, wf, X, R, 3, stream);
          launch_ps32_product_r2c2d3(a3, s3, X + 3 * (size_t)(nx / 2 + 1) * py, R, J, jf, inv_np,
                                     stream);
          return;
        }
        launch_ps32_c2r2d3(a3, s3, wf, X, R, 4, stream);
        product_real(gb, inv_np);
        CFDJ_HIP(hipGetLastError());
        launch_ps32_r2c2d3(a3, s3, Rj, J, jf, stream);
        return;
      } else if (fuse23) {
        launch_half_ps23_jacobian(ha, wf, X, R, jf, stream);
        return;
      } else {
        launch_half_c2r2d(ha, kHalfPs23, wf, X, R, stream);
        product_real(gb, 1.0 / ((double)px * py));
      }
      CFDJ_HIP(hipGetLastError());
      launch_half_r2c2d(ha, Rj, X, jf, stream);
      return;
    }
    if (kind == CFDJ_SPEC_HYBRID) {
      const double gg = 1.0 / (4.0 * dx * dy), hh = 1.0 / 3.0;
      if (real_fields) {  // w_f and w_f / k2 are formed inside the inverse column pass
        launch_hybrid_c2r2d(wf, kx, X, R, nx, ny, tw_n, tw_n, stream);
        hipLaunchKernelGGL(hybrid_jac_real_kernel, dim3(grid_for(n())), dim3(256), 0, stream, R,
                           R + n(), Rj, nx, ny, 1.0 / ((double)nx * ny), gg, hh);
        CFDJ_HIP(hipGetLastError());
        launch_r2c2d(Rj, jf, nx, ny, 1, tw_n, tw_n, stream);
        return;
      }
      hipLaunchKernelGGL(hybrid_prep_kernel, dim3(grid_for(n())), dim3(256), 0, stream, wf, kx,
                         X, nx, ny);
      CFDJ_HIP(hipGetLastError());
      fft2(inv_b, X, true, nb, 1);
      hipLaunchKernelGGL(hybrid_jac_kernel, dim3(grid_for(n())), dim3(256), 0, stream, X, jf,
                         nx, ny, 1.0 / ((double)nx * ny), gg, hh);
      CFDJ_HIP(hipGetLastError());
      fft2(fwd, jf, false, 1, -1);
      return;
    }
    const bool r32 = kind == CFDJ_SPEC_PS32;
    if (hand32) {
      const double sc = (double)px * py, sd = (double)nx * ny;
      hipLaunchKernelGGL(ps32_derivs_cols_kernel, dim3((nx / 2 + 1 + 15) / 16, py / 16), dim3(256),
                         0, stream, wf, kx, X, nx, ny, px, py, sc, sd);
      CFDJ_HIP(hipGetLastError());
      launch_c2r2d3(a3, X, R, 4, stream);
      product_real(gb, 1.0 / sc);
      CFDJ_HIP(hipGetLastError());
      launch_r2c2d3(a3, Rj, J, stream);
      hipLaunchKernelGGL(ps32_unpad_cols_kernel, dim3(nx / 16, ny / 16), dim3(256), 0, stream, J,
                         jf, nx, ny, px, py, sd, sc);
      CFDJ_HIP(hipGetLastError());
      return;
    }
    if (real32) {
      const double sc = (double)px * py, sd = (double)nx * ny;
      const size_t nhp = (size_t)(px / 2 + 1) * py;
      if (stream_loads)
        hipLaunchKernelGGL(ps32_derivs_half_kernel<true>, dim3(grid_for(nhp)), dim3(256), 0,
                           stream, wf, kx, X, nx, ny, px, py, sc, sd);
      else
        hipLaunchKernelGGL(ps32_derivs_half_kernel<false>, dim3(grid_for(nhp)), dim3(256), 0,
                           stream, wf, kx, X, nx, ny, px, py, sc, sd);
      CFDJ_HIP(hipGetLastError());
      plans.exec(inv_r, X, R);
      product_real(gb, 1.0 / sc);
      CFDJ_HIP(hipGetLastError());
      plans.exec(fwd_r, Rj, J);
      hipLaunchKernelGGL(ps32_unpad_half_kernel, dim3(grid_for(n())), dim3(256), 0, stream, J, jf,
                         nx, ny, px, py, sd, sc);
      CFDJ_HIP(hipGetLastError());
      return;
    }
    const int nxe = (2 * nx) / 3, nye = (2 * ny) / 3;
    const int tx0 = nxe / 2, tx1 = nx - nxe / 2, ty0 = nye / 2, ty1 = ny - nye / 2;
    const double sc = (double)px * py, sd = (double)nx * ny;
    hipLaunchKernelGGL(ps_derivs_kernel, dim3(gb), dim3(256), 0, stream, wf, kx, X, nx, ny, px,
                       py, r32 ? 1 : 0, tx0, tx1, ty0, ty1, sc, sd);
    CFDJ_HIP(hipGetLastError());
    if (real_fields && !r32) {  // 2/3 rule on a power-of-two grid: product grid = grid
      launch_c2r2d(X, R, nx, ny, nb, tw_n, tw_n, stream);
      product_real(gb, 1.0 / sc);
      CFDJ_HIP(hipGetLastError());
      launch_r2c2d(Rj, jf, nx, ny, 1, tw_n, tw_n, stream);
      return;
    }
    fft2(inv_b, X, true, nb, 1);
    double2* P = r32 ? J : jf;
    hipLaunchKernelGGL(ps_product_kernel, dim3(gb), dim3(256), 0, stream, X, P, np(),
                       1.0 / sc);
    CFDJ_HIP(hipGetLastError());
    fft2(r32 ? fwd_p : fwd, P, r32, 1, -1);
    if (r32) {
      hipLaunchKernelGGL(ps_unpad_kernel, dim3(grid_for(n())), dim3(256), 0, stream, J, jf, nx,
                         ny, px, py, sd, sc);
      CFDJ_HIP(hipGetLastError());
    }
  }

  template <int STAGE>
  void update(const double2* w, const double2* jA, const double2* jB, double2* out, double dt,
              double alpha, double cA, double cB) {
    const dim3 g(grid_for(half ? nh() + extra() : n())), b(256);
    const double hdt = 0.5 * dt;
#define CFDJ_CN(H, N)                                                                       \
  hipLaunchKernelGGL((cn_update_kernel<STAGE, H, N>), g, b, 0, stream, w, jA, jB, out, kx, nx, \
                     ny, hdt, re, alpha, cA, cB, extra())
    if (half && stream_loads) CFDJ_CN(true, true);
    else if (half) CFDJ_CN(true, false);
    else if (stream_loads) CFDJ_CN(false, true);
    else CFDJ_CN(false, false);
#undef CFDJ_CN
    CFDJ_HIP(hipGetLastError());
  }

  // Full spectrum in `full` (device) -> the state layout in `dst`, and back.
  void import_spectrum(const double2* full, double2* dst) {
    if (half) {
      if (kind == CFDJ_SPEC_HYBRID)
        hipLaunchKernelGGL(full_to_half_kernel<true>, dim3(grid_for(nh())), dim3(256), 0, stream,
                           full, dst, nx, ny, 0);
      else
        hipLaunchKernelGGL(full_to_half_kernel<false>, dim3(grid_for(nh())), dim3(256), 0, stream,
                           full, dst, nx, ny, extra());
      CFDJ_HIP(hipGetLastError());
    } else if (kind == CFDJ_SPEC_HYBRID) {
      // hybrid.jl:103,115 sees w_f through real(ifft(.)) of w_f and w_f / k2 (k2 even), i.e.
      // its Hermitian part only; the real-field transforms here assume that symmetry
      hipLaunchKernelGGL(hermitian_part_kernel, dim3(grid_for(n())), dim3(256), 0, stream, full,
                         dst, nx, ny);
      CFDJ_HIP(hipGetLastError());
    } else {
      // pseudospectral rules: kept as given (see full_to_half_kernel)
      CFDJ_HIP(hipMemcpyAsync(dst, full, n() * sizeof(double2), hipMemcpyDeviceToDevice, stream));
    }
  }
  void export_spectrum(const double2* src, double2* full) {
    if (half) {
      hipLaunchKernelGGL(half_to_full_kernel, dim3(grid_for(n())), dim3(256), 0, stream, src,
                         full, nx, ny, extra());
      CFDJ_HIP(hipGetLastError());
    } else {
      CFDJ_HIP(hipMemcpyAsync(full, src, n() * sizeof(double2), hipMemcpyDeviceToDevice, stream));
    }
  }

  // hybrid.jl:41-67 (alpha, gamma, rho of hybrid.jl:30-32)
  void step(double dt) {
    const double a1 = 8.0 / 15.0, a2 = 2.0 / 15.0, a3 = 1.0 / 3.0;
    const double g1 = 8.0 / 15.0, g2 = 5.0 / 12.0, g3 = 3.0 / 4.0;
    const double r2 = -17.0 / 60.0, r3 = -5.0 / 12.0;
    jacobian(wn, jn);
    update<1>(wn, jn, nullptr, w1, dt, a1, g1 * dt, 0.0);
    jacobian(w1, j1);
    update<2>(w1, jn, j1, w2, dt, a2, r2 * dt, g2 * dt);
    jacobian(w2, j2);
    update<3>(w2, j1, j2, wn, dt, a3, r3 * dt, g3 * dt);
  }

  ~cfdj_spec() {
    if (stream) (void)hipStreamSynchronize(stream);
    plans.destroy();
    if (tw_p != tw_n) dfree(tw_p);
    dfree(tw_n);
    for (double2** p : {&tw3_l3, &tw3_l, &tw3_n, &tw3_m3}) dfree(*p);
    for (double2** p : {&wn, &w1, &w2, &jn, &j1, &j2, &X, &J}) dfree(*p);
    dfree(R);
    dfree(Rj);
    fz.destroy();
    dfree(kx);
    dfree(field);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

extern "C" {

int cfdj_spec_create(int nx, int ny, double dx, double dy, double re, double eps, int kind,
                     int device, cfdj_spec** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr, "out is NULL");
    *out = nullptr;
    CFDJ_REQUIRE(kind == CFDJ_SPEC_HYBRID || kind == CFDJ_SPEC_PS23 || kind == CFDJ_SPEC_PS32,
                 "bad solver kind");
    CFDJ_REQUIRE(nx == ny, "the spectral solvers alias ky = kx (Common.jl:198): nx == ny");
    CFDJ_REQUIRE(nx >= 8 && nx % 2 == 0, "nx must be even and >= 8 (kx loops to nx/2)");
    CFDJ_REQUIRE(dx > 0 && dy > 0 && std::isfinite(re) && re != 0.0, "bad dx, dy or re");
    fft_setup();
    select_device(device);
    std::unique_ptr<cfdj_spec> h(new cfdj_spec);
    CFDJ_HIP(hipGetDevice(&h->device));
    CFDJ_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->kind = kind;
    h->nx = nx;
    h->ny = ny;
    h->dx = dx;
    h->dy = dy;
    h->re = re;
    h->eps = eps;
    h->px = kind == CFDJ_SPEC_PS32 ? (3 * nx) / 2 : nx;
    h->py = kind == CFDJ_SPEC_PS32 ? (3 * ny) / 2 : ny;
    // Common.jl:190-196: hx = 2pi / (nx dx); kx[i] = hx (i-1), kx[i+nx/2] = hx (i-nx/2-1)
    std::vector<double> k(nx);
    const double hx = (2.0 * M_PI) / ((double)nx * dx);
    for (int i = 1; i <= nx / 2; ++i) {
      k[i - 1] = hx * (i - 1.0);
      k[i + nx / 2 - 1] = hx * (double)(i - nx / 2 - 1);
    }
    k[0] = eps;
    h->kx = dalloc<double>(nx);
    CFDJ_HIP(hipMemcpy(h->kx, k.data(), nx * sizeof(double), hipMemcpyHostToDevice));
    const size_t n = h->n(), np = h->np();
    for (double2** p : {&h->wn, &h->w1, &h->w2, &h->jn, &h->j1, &h->j2}) {
      *p = dalloc<double2>(n);
      CFDJ_HIP(hipMemset(*p, 0, n * sizeof(double2)));
    }
    const int nb = kind == CFDJ_SPEC_HYBRID ? 2 : 4;
    h->nb = nb;
    const char* fe = std::getenv("CFDJ_SPEC_FFT");
    const bool want_hand = !(fe && std::strcmp(fe, "rocfft") == 0);
    h->hand_n = want_hand && c2c2d_supported(nx, ny);
    h->hand_p = want_hand && c2c2d_supported(h->px, h->py);
    if (h->hand_n) h->tw_n = twiddle_table(nx);
    if (h->hand_p) h->tw_p = (h->px == nx && h->tw_n) ? h->tw_n : twiddle_table(h->px);
    h->stream_loads = stream_loads_pay(np * sizeof(double));
    const char* re_ = std::getenv("CFDJ_SPEC_REAL");
    const bool want_real = !(re_ && re_[0] == '0');
    h->real_fields = h->hand_n && h->px == nx && want_real;
    h->real32 = kind == CFDJ_SPEC_PS32 && want_hand && want_real;
    const char* h32 = std::getenv("CFDJ_SPEC_PS32_HAND");
    h->hand32 = h->real32 && real2d3_supported(h->px) && nx % 16 == 0 &&
                !(h32 && h32[0] == '0');
    if (h->hand32) {
      h->tw3_l3 = twiddle_table(h->px / 6);
      h->tw3_l = twiddle_table(h->px / 2);
      h->tw3_n = twiddle_table(h->px);
      h->tw3_m3 = twiddle_table(h->px / 3);
      h->a3 = Real2d3Args{h->px, nx / 2, h->tw3_l3, h->tw3_l, h->tw3_n, h->tw3_m3,
                          h->stream_loads};
      const double sc = (double)h->px * h->py, sd = (double)nx * ny;
      h->s3 = Ps32HalfArgs{h->kx, sc / sd, sd / sc};
      const char* f32 = std::getenv("CFDJ_SPEC_PS32_FUSE");
      h->fuse32 = !(f32 && f32[0] == '0');
    }
    // half-spectrum state: the solvers whose product grid is the grid itself, and the 3/2 rule
    // where its padded grid has the hand-written 3 * 2^k transforms
    const char* he = std::getenv("CFDJ_SPEC_HALF");
    h->half = want_hand && want_real && (h->px == nx || h->hand32) && half2d_supported(nx, ny) &&
              !(he && he[0] == '0');
    if (h->half) {
      const char* f23 = std::getenv("CFDJ_SPEC_PS23_FUSE");
      h->fuse23 = kind == CFDJ_SPEC_PS23 && half_ps23_jacobian_supported(nx) &&
                  !(f23 && f23[0] == '0');
      h->fz.init(nx, ny);
      const int nxe = (2 * nx) / 3, nye = (2 * ny) / 3;
      h->ha = HalfSpecArgs{nx, h->fz.twL, h->fz.twN, h->fz.ncu, h->kx, nxe / 2, nye / 2,
                           ny - nye / 2, h->stream_loads};
    }
    if (h->real_fields || h->half || h->real32) {
      h->R = dalloc<double>((size_t)nb * np);
      h->Rj = dalloc<double>(np);
    }
    const size_t nhp = (size_t)(h->px / 2 + 1) * h->py;  // half spectrum of the product grid
    h->X = dalloc<double2>((size_t)nb * (h->real32 ? nhp : np));
    if (kind == CFDJ_SPEC_PS32) h->J = dalloc<double2>(h->real32 ? nhp : np);
    h->field = dalloc<double>((size_t)(nx + 1) * (ny + 1));
    size_t lens[2] = {(size_t)nx, (size_t)ny};
    size_t lp[2] = {(size_t)h->px, (size_t)h->py};
    // library plans only where a path uses them (the half-spectrum path uses none)
    if (!h->half) {
      h->fwd = h->plans.add(rocfft_transform_type_complex_forward, rocfft_placement_inplace, 2,
                            lens, 1, nullptr);
      h->inv = h->plans.add(rocfft_transform_type_complex_inverse, rocfft_placement_inplace, 2,
                            lens, 1, nullptr);
    }
    if (!h->real32 && !h->half)
      h->inv_b = h->plans.add(rocfft_transform_type_complex_inverse, rocfft_placement_inplace, 2,
                              lp, nb, nullptr);
    if (kind == CFDJ_SPEC_PS32 && !h->real32)
      h->fwd_p = h->plans.add(rocfft_transform_type_complex_forward, rocfft_placement_inplace,
                              2, lp, 1, nullptr);
    if (h->real32 && !h->hand32) {
      h->inv_r = h->plans.add(rocfft_transform_type_real_inverse, rocfft_placement_notinplace,
                              2, lp, nb, nullptr);
      h->fwd_r = h->plans.add(rocfft_transform_type_real_forward, rocfft_placement_notinplace,
                              2, lp, 1, nullptr);
    }
    h->plans.finalize(h->stream);
    *out = h.release();
  });
}

// hybrid.jl:24-28: w_f = fft(complex(wn[2:nx+1, 2:ny+1])); w_f[1,1] = 0.
int cfdj_spec_upload(cfdj_spec* h, const double* wn, long ldw) {
  return guard([&] {
    CFDJ_REQUIRE(h && wn, "NULL argument");
    CFDJ_REQUIRE(ldw >= (long)h->nx + 2, "ldw: leading dimension too small");
    select_device(h->device);
    const int nx = h->nx, ny = h->ny;
    CFDJ_HIP(hipMemcpy2DAsync(h->field, (nx + 1) * sizeof(double), wn + 1 + ldw,
                              ldw * sizeof(double), nx * sizeof(double), ny,
                              hipMemcpyHostToDevice, h->stream));
    if (h->half) {
      CFDJ_HIP(hipMemcpy2DAsync(h->Rj, nx * sizeof(double), h->field, (nx + 1) * sizeof(double),
                                nx * sizeof(double), ny, hipMemcpyDeviceToDevice, h->stream));
      launch_half_r2c2d(h->ha, h->Rj, h->X, h->wn, h->stream);
      if (h->extra())
        hipLaunchKernelGGL(ps32_fill_extra_kernel, dim3((nx / 2 + 256) / 256), dim3(256), 0,
                           h->stream, h->wn, nx, ny);
    } else {
      hipLaunchKernelGGL(to_complex_kernel, dim3(grid_for(h->n())), dim3(256), 0, h->stream,
                         h->field, (long)(nx + 1), h->wn, nx, ny);
      CFDJ_HIP(hipGetLastError());
      h->fft2(h->fwd, h->wn, false, 1, -1);
    }
    CFDJ_HIP(hipMemsetAsync(h->wn, 0, sizeof(double2), h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_spec_step(cfdj_spec* h, double dt, int nsteps) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(nsteps >= 0 && std::isfinite(dt), "bad dt or nsteps");
    select_device(h->device);
    for (int k = 0; k < nsteps; ++k) h->step(dt);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

// hybrid.jl:71-76: ut = real(ifft(w_f)) with the periodic row / column, (nx+1) x (ny+1).
int cfdj_spec_download(cfdj_spec* h, double* ut, long ldu) {
  return guard([&] {
    CFDJ_REQUIRE(h && ut, "NULL argument");
    CFDJ_REQUIRE(ldu >= (long)h->nx + 1, "ldu: leading dimension too small");
    select_device(h->device);
    const int nx = h->nx, ny = h->ny;
    const unsigned gf = grid_for((size_t)(nx + 1) * (ny + 1));
    if (h->half) {
      const double2* src = h->wn;
      if (h->extra()) {  // j2 is scratch between steps
        CFDJ_HIP(hipMemcpyAsync(h->j2, h->wn, (h->nh() + h->extra()) * sizeof(double2),
                                hipMemcpyDeviceToDevice, h->stream));
        hipLaunchKernelGGL(ps32_project_row_kernel, dim3((nx / 2 + 256) / 256), dim3(256), 0,
                           h->stream, h->j2, nx, ny);
        src = h->j2;
      }
      launch_half_c2r2d(h->ha, kHalfPlain, src, h->X, h->R, h->stream);
      hipLaunchKernelGGL(to_field_real_kernel, dim3(gf), dim3(256), 0, h->stream, h->R,
                         h->field, (long)(nx + 1), nx, ny, 1.0 / ((double)nx * ny));
    } else {
      CFDJ_HIP(hipMemcpyAsync(h->j2, h->wn, h->n() * sizeof(double2), hipMemcpyDeviceToDevice,
                              h->stream));  // j2 is scratch between steps
      h->fft2(h->inv, h->j2, false, 1, 1);
      hipLaunchKernelGGL(to_field_kernel, dim3(gf), dim3(256), 0, h->stream, h->j2, h->field,
                         (long)(nx + 1), nx, ny, 1.0 / ((double)nx * ny));
    }
    CFDJ_HIP(hipGetLastError());
    CFDJ_HIP(hipMemcpy2DAsync(ut, ldu * sizeof(double), h->field, (nx + 1) * sizeof(double),
                              (nx + 1) * sizeof(double), ny + 1, hipMemcpyDeviceToHost,
                              h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

// The spectrum itself (complex nx x ny, column-major, interleaved re/im), in and out.
int cfdj_spec_get_spectrum(cfdj_spec* h, double* wf) {
  return guard([&] {
    CFDJ_REQUIRE(h && wf, "NULL argument");
    select_device(h->device);
    h->export_spectrum(h->wn, h->j2);  // j2 is scratch between steps
    CFDJ_HIP(hipMemcpyAsync(wf, h->j2, h->n() * sizeof(double2), hipMemcpyDeviceToHost,
                            h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_spec_set_spectrum(cfdj_spec* h, const double* wf) {
  return guard([&] {
    CFDJ_REQUIRE(h && wf, "NULL argument");
    select_device(h->device);
    CFDJ_HIP(hipMemcpyAsync(h->j2, wf, h->n() * sizeof(double2), hipMemcpyHostToDevice,
                            h->stream));
    h->import_spectrum(h->j2, h->wn);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

// One Jacobian evaluation jf = fft(-J(w, psi)) of the spectrum wf (both complex nx x ny).
int cfdj_spec_jacobian(cfdj_spec* h, const double* wf, double* jf) {
  return guard([&] {
    CFDJ_REQUIRE(h && wf && jf, "NULL argument");
    select_device(h->device);
    const size_t b = h->n() * sizeof(double2);
    CFDJ_HIP(hipMemcpyAsync(h->j2, wf, b, hipMemcpyHostToDevice, h->stream));
    h->import_spectrum(h->j2, h->w2);
    h->jacobian(h->w2, h->j1);
    h->export_spectrum(h->j1, h->j2);
    CFDJ_HIP(hipMemcpyAsync(jf, h->j2, b, hipMemcpyDeviceToHost, h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

void cfdj_spec_destroy(cfdj_spec* h) {
  if (!h) return;
  (void)guard([&] {
    select_device(h->device);
    delete h;
  });
}

}  // extern "C"
