// Sum of a field's column-sum partial rows (one per block of rows, written by the stage
// kernels or colpart_kernel) to one row: the body shared by colsum_row_kernel and the extra
// workgroups of the y-slab forward row pass.
#pragma once
#include "cfdj_internal.hpp"

namespace cfdj {

namespace {

// 64 columns x0 .. x0 + 63 by the first four waves of a workgroup (of 256 threads or more,
// all of which must call): wave w sums every 4th block from w on (eight loads in flight per
// lane, added in the order of the plain loop), then lane x of wave 0 adds the four sums in a
// fixed order.  Returns the total in wave 0 (other waves: garbage); `part` is 4 x 64 doubles
// of LDS.
__device__ __forceinline__ double colsum_block(const double* __restrict__ colpart, int nb,
                                               int nx, int x0, double (*part)[64]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = x0 + lane;
  double s = 0.0;
  if (x < nx && w < 4) {
    int b = w;
    for (; b + 28 < nb; b += 32) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = colpart[(size_t)(b + 4 * u) * nx + x];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nb; b += 4) s += colpart[(size_t)b * nx + x];
  }
  if (w < 4) part[w][lane] = s;
  __syncthreads();
  return (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

}  // namespace

}  // namespace cfdj
