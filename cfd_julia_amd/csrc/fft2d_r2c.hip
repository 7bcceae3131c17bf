// 2-D real <-> half-spectrum transforms of the spectral solvers (gfx950) for square
// power-of-two grids of 1024..8192: 20_NS2D_Hybrid_Solver/hybrid.jl and
// 22_NS2D_PseudoSpectral_23_Rule transform REAL fields (fft(complex(w, 0)), real(ifft(.))),
// so the spectrum of every field they hold is Hermitian and half of it is enough: the modes
// kx index m = 0..L (L = n/2), all ky.
//
// Layout of a half spectrum: (L + 1) columns of n elements, ky contiguous: element (m, k) at
// m n + k.  Column L is the kx = -L (Nyquist) column.
//
// Forward  (r -> hs): the FD-FFT Poisson solver's row pass (poisson_fft.hip, real rows ->
//          column-major packed half spectrum: column 0 holds X[0] + i X[L] of every row),
//          then ONE contiguous column per workgroup: forward FFT along y, written to hs; the
//          packed column's transform Z is split with its partner Z[-k] into the DC and the
//          Nyquist column.
// Inverse  (hs -> r): one column per workgroup and array: the column is read from hs,
//          multiplied by the array's spectral factor (half_factor, modes kHalf*), inverse FFT along y,
//          written to the scratch spectrum x; columns 0 and L are packed into column 0 as
//          A + i B after projecting each onto its Hermitian part (A[k] + conj A[-k]) / 2 --
//          what real(ifft(.)) keeps of them.  Then the Poisson solver's inverse row pass.
//
// real(ifft(.)) of a derivative spectrum that is not Hermitian (the reference's kx[1] = eps,
// Common.jl:199, and the 2/3 rule's unsymmetric zero band) keeps its Hermitian part; the
// column pass forms exactly that part from the half spectrum (half_factor).
//
// Both directions are unnormalised, like the library transforms they stand in for.
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

namespace cfdj {

namespace {

// Spectral factor of array `arr` at mode (m, k), applied to w = w_f(m, k).  kxm, kyk: the
// wavenumbers as the reference's elementwise expressions use them (kx[1] = eps).
template <int MODE>
__device__ __forceinline__ double2 half_factor(double2 w, int arr, int m, int k,
                                               const HalfSpecArgs& a) {
#pragma clang fp contract(off)
  if constexpr (MODE == kHalfPlain) {
    return w;
  } else {
    const double kxm = a.kx[m], kyk = a.kx[k];
    const double k2 = kxm * kxm + kyk * kyk;
    // x / k2 as x * (1 / k2), the reciprocal within an ulp (recip_nr): one rounding more than
    // the reference's division, far inside the transforms' own round-off
    const double ik2 = recip_nr(k2);
    if constexpr (MODE == kHalfHybrid) {  // hybrid.jl:103,115: w_f, w_f / k2
      return arr == 0 ? w : make_double2(w.x * ik2, w.y * ik2);
    } else {  // pseudospectral_23_rule.jl:109-133, arrays j1f..j4f
      // real(ifft(.)) keeps the Hermitian part of the filtered derivative spectrum
      // F g w_f, g = i kappa (/ k2): with w_f Hermitian that is i keff w_f (/ k2),
      // keff = (F(m, k) kappa(m, k) - F(-m, -k) kappa(-m, -k)) / 2.  For an odd kappa and a
      // symmetric filter keff = kappa; but the zeroed index band [tx0, n - tx0) is not
      // symmetric (+tx0 is zeroed, -tx0 kept: keff = kappa / 2 there), and kappa is not odd at
      // index 0 (kx[1] = eps, Common.jl:199: keff = 0 except on those filter edges).
      const int mq = (a.n - m) & (a.n - 1), kq = (a.n - k) & (a.n - 1);
      const bool fp = !(m >= a.tx0 && m < a.n - a.tx0) && !(k >= a.ty0 && k < a.ty1);
      const bool fm = !(mq >= a.tx0 && mq < a.n - a.tx0) && !(kq >= a.ty0 && kq < a.ty1);
      if (!fp && !fm) return make_double2(0.0, 0.0);
      const bool xder = arr == 0 || arr == 3;
      const double kap_p = fp ? (xder ? kxm : kyk) : 0.0;
      const double kap_m = fm ? (xder ? a.kx[mq] : a.kx[kq]) : 0.0;
      const double keff = 0.5 * (kap_p - kap_m);
      const double2 d = make_double2(keff * -w.y, keff * w.x);  // 1im * w_f * k
      return (arr == 0 || arr == 2) ? make_double2(d.x * ik2, d.y * ik2) : d;
    }
  }
}

// The scratch spectrum between the column and the row pass: column-major (m M + y), or in
// the row passes' 8-mode tiles (((m/8) M + y) 8 + m%8) where a row's modes are whole lines.
#ifndef CFDJ_HALF_TILE8
#define CFDJ_HALF_TILE8 0
#endif
constexpr bool kTile8 = CFDJ_HALF_TILE8 != 0;
// The inverse row pass skips the columns the 2/3 rule zeroes (its band limit) for rows of up
// to 4096 reals in the column-major layout; elsewhere the column pass writes them as zeros.
__host__ __device__ constexpr bool band_limited(int n) { return !kTile8 && n <= 4096; }
template <int M>
__device__ __forceinline__ size_t xidx(int m, int y) {
  if constexpr (kTile8) return ((((size_t)(m >> 3)) * M + y) << 3) + (m & 7);
  else return (size_t)m * M + y;
}

// (c[k] + conj c[-k]) / 2
__device__ __forceinline__ double2 herm_part(double2 ck, double2 cq) {
  return make_double2(0.5 * (ck.x + cq.x), 0.5 * (ck.y - cq.y));
}

// One column (MODE 0: forward, H -> hs; else inverse, hs -> x).  EDGE = the packed column 0:
// a separate instantiation of the whole body, so its extra loads do not set the register
// count of the other L - 1 columns' code.
template <int M, int MODE, bool EDGE, bool NT>
__device__ __forceinline__ void half_column(double* lds, const HalfSpecArgs& a,
                                            const double2* __restrict__ src,
                                            double2* __restrict__ dst, int m, int arr, int tid) {
  using P = Plan<M>;
  constexpr int DIR = MODE == 0 ? -1 : 1;
  constexpr int L = M / 2;
  const TwGlobal<M> tw{a.twN};
  const double2* col = src + (size_t)m * M;
  double2 v[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int k = in_pos<M, 0>(tid, b, r);
      if constexpr (MODE == 0) {
        v[b * R0 + r] = load_stream<NT>(src + xidx<M>(m, k));  // scratch, dead after
      } else if constexpr (!EDGE) {
        v[b * R0 + r] = half_factor<MODE>(col[k], arr, m, k, a);
      } else {
        const int kq = (M - k) & (M - 1);
        const double2* colL = src + (size_t)L * M;
        const double2 A = half_factor<MODE>(herm_part(col[k], col[kq]), arr, 0, k, a);
        const double2 B = half_factor<MODE>(herm_part(colL[k], colL[kq]), arr, L, k, a);
        v[b * R0 + r] = make_double2(A.x - B.y, A.y + B.x);
      }
    }
  stage_regs<M, 0, DIR>(v, tid, tw);
  run_stages_half<M, 1, DIR>(lds, v, tid, tw);
  // the last stage's outputs j + r*NS are in natural order
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  // forward, packed column: Z goes to column L first and is split in place there
  double2* ocol = dst + (size_t)((MODE == 0 && EDGE) ? L : m) * M;
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) {
      if constexpr (MODE == 0) ocol[out_pos<M, SL>(tid, b, r)] = v[b * RL + r];
      else store_stream<NT>(dst + xidx<M>(m, out_pos<M, SL>(tid, b, r)), v[b * RL + r]);
    }
  if constexpr (MODE == 0 && EDGE) {
    // Z = FFT_y(X0 + i XL), X0 and XL real: F0[k] = (Z[k] + conj Z[-k]) / 2,
    // FL[k] = (Z[k] - conj Z[-k]) / (2i); a thread owns the pair (k, M - k)
    __syncthreads();  // workgroup-scope release / acquire of the global stores
    double2* c0 = dst;
#pragma unroll 1
    for (int k = tid; k <= M / 2; k += P::T) {
      const int kq = (M - k) & (M - 1);
      const double2 Zk = ocol[k], Zq = ocol[kq];
      const double2 A = herm_part(Zk, Zq);
      const double2 Bk = make_double2(0.5 * (Zk.y + Zq.y), -0.5 * (Zk.x - Zq.x));
      c0[k] = A;
      ocol[k] = Bk;
      if (kq != k) {
        c0[kq] = cconj(A);
        ocol[kq] = cconj(Bk);
      }
    }
  }
}

#ifndef CFDJ_HALF_COLS_WAVES
#define CFDJ_HALF_COLS_WAVES 4
#endif
#ifndef CFDJ_HALF_COLS_WAVES_M3
// mode 3 (four derivative spectra per column): 33 spilled registers at 4 waves per SIMD, none
// at 3 -- and 139 us against 158 at 4096^2: occupancy wins
#define CFDJ_HALF_COLS_WAVES_M3 4
#endif
template <int MODE>
constexpr int half_cols_waves() {
  return MODE == 3 ? CFDJ_HALF_COLS_WAVES_M3 : CFDJ_HALF_COLS_WAVES;
}
template <int M, int MODE, bool NT>
__global__ __launch_bounds__(Plan<M>::T)
    __attribute__((amdgpu_waves_per_eu(half_cols_waves<MODE>(), half_cols_waves<MODE>()))) void half_cols_kernel(const HalfSpecArgs a,
                                                             const double2* __restrict__ src,
                                                             double2* __restrict__ dst, int arr0,
                                                             int nb) {
  using P = Plan<M>;
  static_assert(P::NSTAGES >= 2, "column length");
  constexpr int L = M / 2;
  __shared__ double lds[P::PAD];
  const int tid = threadIdx.x;
  // A workgroup forms `nb` arrays [arr0, arr0 + nb) of its column one after the other, the
  // gridDim.x / L workgroups of a column are neighbours on one XCD.  With four arrays at
  // 4096^2 one workgroup per column is fastest (186 against 203 us per launch: the column
  // comes from HBM once and from L2 after that); with two arrays, or on smaller grids that
  // need the workgroups to fill the chip, one workgroup per array.
  const int id = xcd_remap(blockIdx.x, gridDim.x), per_col = gridDim.x / L;
  const int m = __builtin_amdgcn_readfirstlane(id / per_col);
  arr0 += __builtin_amdgcn_readfirstlane(id % per_col) * nb;
#pragma unroll 1
  for (int arr = arr0; arr < arr0 + nb; ++arr) {
    double2* out = dst + (size_t)arr * L * M;
    if constexpr (MODE == kHalfPs23) {
      // columns the 2/3 rule zeroes on both sides (+m and -m): nothing to transform, and the
      // row pass does not read them (band limit tx0)
      if (m > a.tx0) {
        if constexpr (!band_limited(M))
          for (int k = tid; k < M; k += P::T) out[xidx<M>(m, k)] = make_double2(0.0, 0.0);
        continue;
      }
    }
    // an opaque copy of the thread index per array: what depends only on it (twiddles,
    // offsets) is formed again inside each pass instead of staying live across the loop
    int t = tid;
    asm volatile("" : "+v"(t));
    if (m == 0) half_column<M, MODE, true, NT>(lds, a, src, out, m, arr, t);
    else half_column<M, MODE, false, NT>(lds, a, src, out, m, arr, t);
  }
}

template <int M>
void launch_half_cols(int mode, const HalfSpecArgs& a, const double2* src, double2* dst, int arr0,
                      int nb, hipStream_t st) {
  const int per_wg = (M >= 4096 && nb > 2) ? nb : 1;  // arrays per workgroup
  const dim3 grid((unsigned)((M / 2) * (nb / per_wg))), block(Plan<M>::T);
  nb = per_wg;
  switch (mode) {
    case 0:  // NT = the input (the scratch spectrum, dead after this read) by streaming loads
      if (a.stream)
        hipLaunchKernelGGL((half_cols_kernel<M, 0, true>), grid, block, 0, st, a, src, dst, arr0,
                           nb);
      else
        hipLaunchKernelGGL((half_cols_kernel<M, 0, false>), grid, block, 0, st, a, src, dst, arr0,
                           nb);
      break;
    // inverse modes: NT = the scratch spectrum (134 MB per array at 4096^2, read back only
    // after the whole pass) by streaming stores
    case kHalfPlain:
      hipLaunchKernelGGL((half_cols_kernel<M, kHalfPlain, false>), grid, block, 0, st, a, src,
                         dst, arr0, nb);
      break;
    case kHalfHybrid:
      if (a.stream)
        hipLaunchKernelGGL((half_cols_kernel<M, kHalfHybrid, true>), grid, block, 0, st, a, src,
                           dst, arr0, nb);
      else
        hipLaunchKernelGGL((half_cols_kernel<M, kHalfHybrid, false>), grid, block, 0, st, a, src,
                           dst, arr0, nb);
      break;
    default:
      if (a.stream)
        hipLaunchKernelGGL((half_cols_kernel<M, kHalfPs23, true>), grid, block, 0, st, a, src,
                           dst, arr0, nb);
      else
        hipLaunchKernelGGL((half_cols_kernel<M, kHalfPs23, false>), grid, block, 0, st, a, src,
                           dst, arr0, nb);
      break;
  }
}

// Arrays [arr0, arr0 + nb) of the mode.
void half_cols(int mode, const HalfSpecArgs& a, const double2* src, double2* dst, int arr0,
               int nb, hipStream_t st) {
  switch (a.n) {
    case 1024: launch_half_cols<1024>(mode, a, src, dst, arr0, nb, st); break;
    case 2048: launch_half_cols<2048>(mode, a, src, dst, arr0, nb, st); break;
    case 4096: launch_half_cols<4096>(mode, a, src, dst, arr0, nb, st); break;
    default: launch_half_cols<8192>(mode, a, src, dst, arr0, nb, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

// The row passes of the FD-FFT Poisson solver on one array.
FusedPoissonArgs row_args(const HalfSpecArgs& a, const double* f, double* s, double2* H) {
  FusedPoissonArgs p{};
  p.nx = p.ny = p.rows = a.n;
  p.f = f;
  p.s = s;
  p.H = p.C = H;
  p.tile8 = kTile8 ? 1 : 0;
  p.stream = a.stream;
  p.twL = a.twL;
  p.twN = a.twN;
  p.ncu = a.ncu;
  return p;
}

void check(const HalfSpecArgs& a) {
  if (!half2d_supported(a.n, a.n)) throw Error{CFDJ_ERR_ARG, "half-spectrum transform: unsupported size"};
}

int arrays_of(int mode) { return mode == kHalfHybrid ? 2 : mode == kHalfPs23 ? 4 : 1; }

}  // namespace

bool half2d_supported(int nx, int ny) {
  return nx == ny && (nx == 1024 || nx == 2048 || nx == 4096 || nx == 8192) &&
         fused_rows_supported(nx, ny);
}

void launch_half_r2c2d(const HalfSpecArgs& a, const double* r, double2* scratch, double2* hs,
                       hipStream_t st) {
  check(a);
  launch_fused_poisson_pass(0, row_args(a, r, nullptr, scratch), st);
  half_cols(0, a, scratch, hs, 0, 1, st);
}

void launch_half_c2r2d(const HalfSpecArgs& a, int mode, const double2* hs, double2* x, double* r,
                       hipStream_t st) {
  check(a);
  if (mode != kHalfPlain && mode != kHalfHybrid && mode != kHalfPs23)
    throw Error{CFDJ_ERR_ARG, "half-spectrum transform: bad mode"};
  const int nb = arrays_of(mode);
  const size_t half = (size_t)(a.n / 2) * a.n, full = (size_t)a.n * a.n;
  half_cols(mode, a, hs, x, 0, nb, st);
  for (int b = 0; b < nb; ++b) {
    FusedPoissonArgs p = row_args(a, nullptr, r + b * full, x + b * half);
    if (mode == kHalfPs23 && band_limited(a.n)) p.mmax = a.tx0;
    launch_fused_poisson_pass(2, p, st);
  }
}

bool half_ps23_jacobian_supported(int n) {
  return half2d_supported(n, n) && band_limited(n) && rows_jac_supported(n, n);
}

void launch_half_ps23_jacobian(const HalfSpecArgs& a, const double2* hs, double2* x, double* r,
                               double2* hs_out, hipStream_t st) {
  check(a);
  if (!half_ps23_jacobian_supported(a.n))
    throw Error{CFDJ_ERR_ARG, "half-spectrum 2/3-rule product: unsupported size"};
  const size_t half = (size_t)(a.n / 2) * a.n, full = (size_t)a.n * a.n;
  half_cols(kHalfPs23, a, hs, x, 0, 4, st);
  for (int b = 0; b < 3; ++b) {
    FusedPoissonArgs p = row_args(a, nullptr, r + b * full, x + b * half);
    p.mmax = a.tx0;
    launch_fused_poisson_pass(2, p, st);
  }
  // the product's scratch spectrum goes where the first field's was (consumed above)
  FusedPoissonArgs p = row_args(a, r, nullptr, x + 3 * half);
  p.C = x;
  p.mmax = a.tx0;
  launch_rows_jac(p, 1.0 / ((double)a.n * a.n), st);
  half_cols(0, a, x, hs_out, 0, 1, st);
}

}  // namespace cfdj
