// In-place 2-D complex-to-complex FFT of power-of-two grids (gfx950), unnormalised in both
// directions like the library transform it stands in for: the spectral solvers of
// 20_NS2D_Hybrid_Solver/hybrid.jl and 22_NS2D_PseudoSpectral_23_Rule (fft / ifft of
// nx-by-ny complex arrays, x contiguous) in TWO passes over the array and no transposes,
// where the library runs four (row FFT, transpose, row FFT, transpose):
//
//   rows : one contiguous row of N complex per workgroup (N / 16 threads, Stockham radix-16
//          stages, component-wise LDS exchange), loaded, transformed and stored in place;
//   cols : FOUR neighbouring columns per workgroup, so every access to a row of the array
//          is a whole 64-B segment; 4 M / 16 threads, the four transforms interleaved
//          element by element in a component-wise LDS buffer (4 M doubles, 139 KB at
//          M = 4096: what makes four columns fit at all), in place.
//
// The physical-space side of these solvers is real (real(ifft(.)) in, complex(., 0) out):
// launch_c2r2d runs the column pass first and lets the row pass store real parts only, into
// a real array; launch_r2c2d lets the row pass read a real array and the column pass finish
// in place -- a quarter less traffic per transform and half-size fields for the kernels
// between them.
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

namespace cfdj {

namespace {

// MODE 0: complex row in place; 1: real row in (`rin`), complex row out; 2: complex row in,
// its real part out (`rout`).
template <int N, int DIR, int MODE>
__global__ __launch_bounds__(Plan<N>::T) void c2c_rows_kernel(double2* __restrict__ a,
                                                             const double* __restrict__ rin,
                                                             double* __restrict__ rout,
                                                             const double2* __restrict__ tw_) {
  using P = Plan<N>;
  static_assert(P::NSTAGES >= 2, "row length");
  __shared__ double lds[P::PAD];
  const TwGlobal<N> tw{tw_};
  const int tid = threadIdx.x;
  double2* row = a + (size_t)blockIdx.x * N;
  double2 v[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      if constexpr (MODE == 1)
        v[b * R0 + r] = make_double2(rin[(size_t)blockIdx.x * N + in_pos<N, 0>(tid, b, r)], 0.0);
      else
        v[b * R0 + r] = row[in_pos<N, 0>(tid, b, r)];
    }
  stage_regs<N, 0, DIR>(v, tid, tw);
  run_stages_half<N, 1, DIR>(lds, v, tid, tw);
  // the last stage's outputs j + r*NS are in natural order
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) {
      if constexpr (MODE == 2)
        rout[(size_t)blockIdx.x * N + out_pos<N, SL>(tid, b, r)] = v[b * RL + r].x;
      else
        row[out_pos<N, SL>(tid, b, r)] = v[b * RL + r];
    }
}

#ifndef CFDJ_C2C_XC
#define CFDJ_C2C_XC 4
#endif
constexpr int kColsPerGroup = CFDJ_C2C_XC;

// kx[i]^2 + kx[j]^2 as the spectral solvers' own kernels form it (no contraction).
__device__ __forceinline__ double k2_of(double kxi, double kyj) {
#pragma clang fp contract(off)
  return kxi * kxi + kyj * kyj;
}

// PREP (hybrid.jl:103,115 folded into the inverse column pass): the columns are read from
// ONE source spectrum `src` = w_f and written to the arrays of `a`: array 0 gets the
// transform of w_f, array 1 that of w_f / k2 (k2 = kx[i]^2 + kx[j]^2, a true division as in
// the separate kernel) -- neither input array is ever materialised.
template <int M, int DIR, bool PREP>
__global__ __launch_bounds__(kColsPerGroup* Plan<M>::T) void c2c_cols_kernel(
    double2* __restrict__ a, int nx, int groups_per_array, const double2* __restrict__ tw_,
    const double2* __restrict__ src, const double* __restrict__ kx) {
  using P = Plan<M>;
  static_assert(P::NSTAGES >= 2, "column length");
  constexpr int XC = kColsPerGroup;
  __shared__ double lds[XC * P::PAD];
  const TwGlobal<M> tw{tw_};
  const int c = threadIdx.x % XC;   // column of the group: 4 lanes = one 64-B row segment
  const int tid = threadIdx.x / XC;  // thread of that column's transform
  // neighbouring groups share 128-B lines (two 64-B halves): keep them on one XCD's L2
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int arr = wg / groups_per_array, grp = wg % groups_per_array;
  // wave-uniform base and 32-bit element offsets (y * nx + c): one offset register per access
  double2* base = a + (size_t)__builtin_amdgcn_readfirstlane(arr) * nx * M +
                  (size_t)__builtin_amdgcn_readfirstlane(grp) * XC;
  const double2* in = PREP ? src + (size_t)__builtin_amdgcn_readfirstlane(grp) * XC : base;
  double* buf = lds + c;
  double2 v[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r)
      v[b * R0 + r] = in[(unsigned)(in_pos<M, 0>(tid, b, r) * nx + c)];
  if constexpr (PREP) {
    if (arr == 1) {
      const double kxi = kx[grp * XC + c];
#pragma unroll
      for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
        for (int r = 0; r < R0; ++r) {
          const double k2 = k2_of(kxi, kx[in_pos<M, 0>(tid, b, r)]);
          v[b * R0 + r] = make_double2(v[b * R0 + r].x / k2, v[b * R0 + r].y / k2);
        }
    }
  }
  stage_regs<M, 0, DIR>(v, tid, tw);
  run_stages_half<M, 1, DIR, XC>(buf, v, tid, tw);
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r)
      base[(unsigned)(out_pos<M, SL>(tid, b, r) * nx + c)] = v[b * RL + r];
}

// mode 0: in place (dir either way); 1: real in, forward; 2: real out, inverse
template <int N>
void launch_rows(double2* a, const double* rin, double* rout, int rows, int dir, int mode,
                 const double2* tw, hipStream_t st) {
  const dim3 g(rows), b(Plan<N>::T);
  if (mode == 1)
    hipLaunchKernelGGL((c2c_rows_kernel<N, -1, 1>), g, b, 0, st, a, rin, rout, tw);
  else if (mode == 2)
    hipLaunchKernelGGL((c2c_rows_kernel<N, 1, 2>), g, b, 0, st, a, rin, rout, tw);
  else if (dir < 0)
    hipLaunchKernelGGL((c2c_rows_kernel<N, -1, 0>), g, b, 0, st, a, rin, rout, tw);
  else
    hipLaunchKernelGGL((c2c_rows_kernel<N, 1, 0>), g, b, 0, st, a, rin, rout, tw);
}

// src != nullptr: the hybrid solver's inverse pass with its preparation folded in (2 arrays)
template <int M>
void launch_cols(double2* a, int nx, int batch, int dir, const double2* tw, hipStream_t st,
                 const double2* src = nullptr, const double* kx = nullptr) {
  const int groups = nx / kColsPerGroup;
  const dim3 grid((unsigned)(groups * batch)), block(kColsPerGroup * Plan<M>::T);
  if (src != nullptr)
    hipLaunchKernelGGL((c2c_cols_kernel<M, 1, true>), grid, block, 0, st, a, nx, groups, tw, src,
                       kx);
  else if (dir < 0)
    hipLaunchKernelGGL((c2c_cols_kernel<M, -1, false>), grid, block, 0, st, a, nx, groups, tw,
                       src, kx);
  else
    hipLaunchKernelGGL((c2c_cols_kernel<M, 1, false>), grid, block, 0, st, a, nx, groups, tw,
                       src, kx);
}

constexpr bool pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

}  // namespace

// Row lengths 256..4096 (one row's component-wise buffer is 34 KB at most), column lengths
// 256..4096 (four columns: 139 KB at most).
bool c2c2d_supported(int nx, int ny) {
  return pow2(nx) && pow2(ny) && nx >= 256 && nx <= 4096 && ny >= 256 && ny <= 4096;
}

namespace {

void rows_pass(double2* a, const double* rin, double* rout, int nx, int rows, int dir, int mode,
               const double2* tw, hipStream_t st) {
  switch (nx) {
    case 256: launch_rows<256>(a, rin, rout, rows, dir, mode, tw, st); break;
    case 512: launch_rows<512>(a, rin, rout, rows, dir, mode, tw, st); break;
    case 1024: launch_rows<1024>(a, rin, rout, rows, dir, mode, tw, st); break;
    case 2048: launch_rows<2048>(a, rin, rout, rows, dir, mode, tw, st); break;
    default: launch_rows<4096>(a, rin, rout, rows, dir, mode, tw, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void cols_pass(double2* a, int nx, int ny, int batch, int dir, const double2* tw,
               hipStream_t st, const double2* src = nullptr, const double* kx = nullptr) {
  switch (ny) {
    case 256: launch_cols<256>(a, nx, batch, dir, tw, st, src, kx); break;
    case 512: launch_cols<512>(a, nx, batch, dir, tw, st, src, kx); break;
    case 1024: launch_cols<1024>(a, nx, batch, dir, tw, st, src, kx); break;
    case 2048: launch_cols<2048>(a, nx, batch, dir, tw, st, src, kx); break;
    default: launch_cols<4096>(a, nx, batch, dir, tw, st, src, kx); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void check_size(int nx, int ny, int batch) {
  if (!c2c2d_supported(nx, ny) || batch < 1)
    throw Error{CFDJ_ERR_ARG, "2-D complex FFT: unsupported size"};
}

}  // namespace

// dir < 0: forward (exp(-i ...)), dir > 0: inverse, both unnormalised.  `batch` arrays of
// nx * ny elements back to back.  twX / twY: exp(-2 pi i k / nx), k < nx, and the same for
// ny (device tables).
void launch_c2c2d(double2* a, int nx, int ny, int batch, int dir, const double2* twX,
                  const double2* twY, hipStream_t st) {
  check_size(nx, ny, batch);
  rows_pass(a, nullptr, nullptr, nx, ny * batch, dir, 0, twX, st);
  cols_pass(a, nx, ny, batch, dir, twY, st);
}

// real(ifft2(a)) * (nx ny) -> r (batch real arrays of nx * ny); `a` is overwritten.
void launch_c2r2d(double2* a, double* r, int nx, int ny, int batch, const double2* twX,
                  const double2* twY, hipStream_t st) {
  check_size(nx, ny, batch);
  cols_pass(a, nx, ny, batch, 1, twY, st);
  rows_pass(a, nullptr, r, nx, ny * batch, 1, 2, twX, st);
}

// The hybrid solver's two inverse transforms from one spectrum (hybrid.jl:103-127):
// r[0] = real(ifft2(wf)), r[1] = real(ifft2(wf / k2)) (unnormalised), k2 = kx[i]^2 + kx[j]^2;
// `x` (2 complex arrays) is scratch, wf is left intact.  nx == ny (one kx table).
void launch_hybrid_c2r2d(const double2* wf, const double* kx, double2* x, double* r, int nx,
                         int ny, const double2* twX, const double2* twY, hipStream_t st) {
  check_size(nx, ny, 2);
  if (nx != ny) throw Error{CFDJ_ERR_ARG, "hybrid transform: square grids only"};
  cols_pass(x, nx, ny, 2, 1, twY, st, wf, kx);
  rows_pass(x, nullptr, r, nx, ny * 2, 1, 2, twX, st);
}

// fft2(complex(r, 0)) -> a.
void launch_r2c2d(const double* r, double2* a, int nx, int ny, int batch, const double2* twX,
                  const double2* twY, hipStream_t st) {
  check_size(nx, ny, batch);
  rows_pass(a, r, nullptr, nx, ny * batch, -1, 1, twX, st);
  cols_pass(a, nx, ny, batch, -1, twY, st);
}

}  // namespace cfdj
