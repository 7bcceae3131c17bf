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
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

namespace cfdj {

namespace {

template <int N, int DIR>
__global__ __launch_bounds__(Plan<N>::T) void c2c_rows_kernel(double2* __restrict__ a,
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
    for (int r = 0; r < R0; ++r) v[b * R0 + r] = row[in_pos<N, 0>(tid, b, r)];
  stage_regs<N, 0, DIR>(v, tid, tw);
  run_stages_half<N, 1, DIR>(lds, v, tid, tw);
  // the last stage's outputs j + r*NS are in natural order
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) row[out_pos<N, SL>(tid, b, r)] = v[b * RL + r];
}

#ifndef CFDJ_C2C_XC
#define CFDJ_C2C_XC 4
#endif
constexpr int kColsPerGroup = CFDJ_C2C_XC;

template <int M, int DIR>
__global__ __launch_bounds__(kColsPerGroup* Plan<M>::T) void c2c_cols_kernel(
    double2* __restrict__ a, int nx, int groups_per_array, const double2* __restrict__ tw_) {
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
  double* buf = lds + c;
  double2 v[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r)
      v[b * R0 + r] = base[(unsigned)(in_pos<M, 0>(tid, b, r) * nx + c)];
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

template <int N>
void launch_rows(double2* a, int rows, int dir, const double2* tw, hipStream_t st) {
  if (dir < 0)
    hipLaunchKernelGGL((c2c_rows_kernel<N, -1>), dim3(rows), dim3(Plan<N>::T), 0, st, a, tw);
  else
    hipLaunchKernelGGL((c2c_rows_kernel<N, 1>), dim3(rows), dim3(Plan<N>::T), 0, st, a, tw);
}

template <int M>
void launch_cols(double2* a, int nx, int batch, int dir, const double2* tw, hipStream_t st) {
  const int groups = nx / kColsPerGroup;
  const dim3 grid((unsigned)(groups * batch)), block(kColsPerGroup * Plan<M>::T);
  if (dir < 0)
    hipLaunchKernelGGL((c2c_cols_kernel<M, -1>), grid, block, 0, st, a, nx, groups, tw);
  else
    hipLaunchKernelGGL((c2c_cols_kernel<M, 1>), grid, block, 0, st, a, nx, groups, tw);
}

constexpr bool pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

}  // namespace

// Row lengths 256..4096 (one row's component-wise buffer is 34 KB at most), column lengths
// 256..4096 (four columns: 139 KB at most).
bool c2c2d_supported(int nx, int ny) {
  return pow2(nx) && pow2(ny) && nx >= 256 && nx <= 4096 && ny >= 256 && ny <= 4096;
}

// dir < 0: forward (exp(-i ...)), dir > 0: inverse, both unnormalised.  `batch` arrays of
// nx * ny elements back to back.  twX / twY: exp(-2 pi i k / nx), k < nx, and the same for
// ny (device tables).
void launch_c2c2d(double2* a, int nx, int ny, int batch, int dir, const double2* twX,
                  const double2* twY, hipStream_t st) {
  if (!c2c2d_supported(nx, ny) || batch < 1)
    throw Error{CFDJ_ERR_ARG, "2-D complex FFT: unsupported size"};
  const int rows = ny * batch;
  switch (nx) {
    case 256: launch_rows<256>(a, rows, dir, twX, st); break;
    case 512: launch_rows<512>(a, rows, dir, twX, st); break;
    case 1024: launch_rows<1024>(a, rows, dir, twX, st); break;
    case 2048: launch_rows<2048>(a, rows, dir, twX, st); break;
    default: launch_rows<4096>(a, rows, dir, twX, st); break;
  }
  CFDJ_HIP(hipGetLastError());
  switch (ny) {
    case 256: launch_cols<256>(a, nx, batch, dir, twY, st); break;
    case 512: launch_cols<512>(a, nx, batch, dir, twY, st); break;
    case 1024: launch_cols<1024>(a, nx, batch, dir, twY, st); break;
    case 2048: launch_cols<2048>(a, nx, batch, dir, twY, st); break;
    default: launch_cols<4096>(a, nx, batch, dir, twY, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
