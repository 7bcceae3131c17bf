// Streaming ceilings on MI355X for the access shapes of the vortex-merger stage kernels:
// R read streams + 1 write stream of 4096^2 doubles each, 16 B per lane, one pass per launch.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/streambench.hip -o tools/micro/streambench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int R, int U>
__global__ __launch_bounds__(256) void stream_kernel(const double2* __restrict__ a,
                                                     const double2* __restrict__ b,
                                                     const double2* __restrict__ c,
                                                     double2* __restrict__ o, size_t n) {
  // each thread handles U elements, strided by the grid (coalesced)
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  double2 va[U], vb[U], vc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t j = i + u * stride;
    if (j < n) {
      va[u] = a[j];
      if (R >= 2) vb[u] = b[j];
      if (R >= 3) vc[u] = c[j];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t j = i + u * stride;
    if (j < n) {
      double2 r = va[u];
      if (R >= 2) { r.x += vb[u].x; r.y += vb[u].y; }
      if (R >= 3) { r.x += vc[u].x; r.y += vc[u].y; }
      o[j] = r;
    }
  }
}

// row-marching variant: a wave owns 128 columns and marches `rows` rows (like the stage kernel)
template <int R>
__global__ __launch_bounds__(256) void march_kernel(const double* __restrict__ a,
                                                    const double* __restrict__ b,
                                                    const double* __restrict__ c,
                                                    double* __restrict__ o, int nx, int ny, int rpw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int strips = nx / 128;
  const int tile = blockIdx.x;
  const int strip = tile % strips, chunk = tile / strips;
  const int x = strip * 128 + 2 * lane;
  const int y0 = (chunk * 4 + wave) * rpw;
  double2 pa, pb, pc;
  pa = *reinterpret_cast<const double2*>(a + (size_t)y0 * nx + x);
  if (R >= 2) pb = *reinterpret_cast<const double2*>(b + (size_t)y0 * nx + x);
  if (R >= 3) pc = *reinterpret_cast<const double2*>(c + (size_t)y0 * nx + x);
  for (int y = y0; y < y0 + rpw; ++y) {
    const int yn = y + 1 < y0 + rpw ? y + 1 : y;
    double2 na, nb, nc;
    na = *reinterpret_cast<const double2*>(a + (size_t)yn * nx + x);
    if (R >= 2) nb = *reinterpret_cast<const double2*>(b + (size_t)yn * nx + x);
    if (R >= 3) nc = *reinterpret_cast<const double2*>(c + (size_t)yn * nx + x);
    double2 r = pa;
    if (R >= 2) { r.x += pb.x; r.y += pb.y; }
    if (R >= 3) { r.x += pc.x; r.y += pc.y; }
    *reinterpret_cast<double2*>(o + (size_t)y * nx + x) = r;
    pa = na; pb = nb; pc = nc;
  }
}

// march with a D-row-deep register prefetch ring
template <int R, int D>
__global__ __launch_bounds__(256) void march_deep_kernel(const double* __restrict__ a,
                                                         const double* __restrict__ b,
                                                         const double* __restrict__ c,
                                                         double* __restrict__ o, int nx, int ny, int rpw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int strips = nx / 128;
  const int tile = blockIdx.x;
  const int strip = tile % strips, chunk = tile / strips;
  const int x = strip * 128 + 2 * lane;
  const int y0 = (chunk * 4 + wave) * rpw;
  double2 pa[D], pb[D], pc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    pa[d] = *reinterpret_cast<const double2*>(a + (size_t)(y0 + d) * nx + x);
    if (R >= 2) pb[d] = *reinterpret_cast<const double2*>(b + (size_t)(y0 + d) * nx + x);
    if (R >= 3) pc[d] = *reinterpret_cast<const double2*>(c + (size_t)(y0 + d) * nx + x);
  }
  for (int yb = y0; yb < y0 + rpw; yb += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int y = yb + d;
      const int yn = y + D < y0 + rpw ? y + D : y;
      double2 r = pa[d];
      if (R >= 2) { r.x += pb[d].x; r.y += pb[d].y; }
      if (R >= 3) { r.x += pc[d].x; r.y += pc[d].y; }
      pa[d] = *reinterpret_cast<const double2*>(a + (size_t)yn * nx + x);
      if (R >= 2) pb[d] = *reinterpret_cast<const double2*>(b + (size_t)yn * nx + x);
      if (R >= 3) pc[d] = *reinterpret_cast<const double2*>(c + (size_t)yn * nx + x);
      *reinterpret_cast<double2*>(o + (size_t)y * nx + x) = r;
    }
  }
}

// row-group tile: a 256-thread workgroup covers 512 columns x G rows; every thread loads its
// column pair of rows y0-1 .. y0+G of a and b (halo rows re-read through L1 / L2) and of rows
// y0 .. y0+G-1 of c, writes G rows: the traffic shape of a stencil stage without marching.
template <int R, int G>
__global__ __launch_bounds__(256) void tile_kernel(const double* __restrict__ a,
                                                   const double* __restrict__ b,
                                                   const double* __restrict__ c,
                                                   double* __restrict__ o, int nx, int ny) {
  const int strips = nx / 512;
  const int strip = blockIdx.x % strips, grp = blockIdx.x / strips;
  const int x = strip * 512 + 2 * threadIdx.x;
  const int y0 = grp * G;
  double2 va[G + 2], vb[G + 2], vc[G];
#pragma unroll
  for (int j = 0; j < G + 2; ++j) {
    const int y = (y0 - 1 + j + ny) % ny;
    va[j] = *reinterpret_cast<const double2*>(a + (size_t)y * nx + x);
    if (R >= 2) vb[j] = *reinterpret_cast<const double2*>(b + (size_t)y * nx + x);
  }
  if (R >= 3) {
#pragma unroll
    for (int j = 0; j < G; ++j) vc[j] = *reinterpret_cast<const double2*>(c + (size_t)(y0 + j) * nx + x);
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    double2 r;
    r.x = va[j].x + va[j + 1].x + va[j + 2].x;
    r.y = va[j].y + va[j + 1].y + va[j + 2].y;
    if (R >= 2) { r.x += vb[j].x + vb[j + 1].x + vb[j + 2].x; r.y += vb[j].y + vb[j + 1].y + vb[j + 2].y; }
    if (R >= 3) { r.x += vc[j].x; r.y += vc[j].y; }
    *reinterpret_cast<double2*>(o + (size_t)(y0 + j) * nx + x) = r;
  }
}

int main(int argc, char** argv) {
  const int nx = argc > 1 ? atoi(argv[1]) : 4096, ny = argc > 2 ? atoi(argv[2]) : nx;
  printf("arrays of %d x %d doubles (%.0f MB each)\n", nx, ny, (double)nx * ny * 8 / 1e6);
  const size_t n = (size_t)nx * ny, n2 = n / 2;
  double *a, *b, *c, *o;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&c, n * 8)); CK(hipMalloc(&o, n * 8));
  CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8)); CK(hipMemset(c, 0, n * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int reps = 20;
  auto report = [&](const char* name, int R, float ms) {
    const double bytes = (double)(R + 1) * n * 8;
    printf("%-34s R=%d  %7.2f us  %7.1f GB/s\n", name, R, ms * 1e3 / reps, bytes * reps / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
#define RUN_STREAM(R, U)                                                                      \
  {                                                                                           \
    const unsigned grid = (unsigned)((n2 + 256ull * U - 1) / (256ull * U));                   \
    hipLaunchKernelGGL((stream_kernel<R, U>), dim3(grid), dim3(256), 0, 0, (const double2*)a, \
                       (const double2*)b, (const double2*)c, (double2*)o, n2);                \
    CK(hipEventRecord(e0));                                                                   \
    for (int i = 0; i < reps; ++i)                                                            \
      hipLaunchKernelGGL((stream_kernel<R, U>), dim3(grid), dim3(256), 0, 0,                  \
                         (const double2*)a, (const double2*)b, (const double2*)c,             \
                         (double2*)o, n2);                                                    \
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                                      \
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));                                           \
    char nm[64]; snprintf(nm, 64, "stream U=%d", U); report(nm, R, ms);                       \
  }
  RUN_STREAM(1, 1) RUN_STREAM(1, 4) RUN_STREAM(1, 8)
  RUN_STREAM(2, 1) RUN_STREAM(2, 4) RUN_STREAM(2, 8)
  RUN_STREAM(3, 1) RUN_STREAM(3, 4) RUN_STREAM(3, 8)
#define RUN_MARCH(R, RPW)                                                                     \
  {                                                                                           \
    const unsigned grid = (unsigned)((nx / 128) * (ny / (4 * RPW)));                          \
    hipLaunchKernelGGL((march_kernel<R>), dim3(grid), dim3(256), 0, 0, a, b, c, o, nx, ny, RPW); \
    CK(hipEventRecord(e0));                                                                   \
    for (int i = 0; i < reps; ++i)                                                            \
      hipLaunchKernelGGL((march_kernel<R>), dim3(grid), dim3(256), 0, 0, a, b, c, o, nx, ny, RPW); \
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                                      \
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));                                           \
    char nm[64]; snprintf(nm, 64, "march rows/wave=%d", RPW); report(nm, R, ms);              \
  }
  RUN_MARCH(1, 32) RUN_MARCH(2, 32) RUN_MARCH(3, 32) RUN_MARCH(2, 8) RUN_MARCH(3, 8) RUN_MARCH(2, 64) RUN_MARCH(3, 64)
#define RUN_DEEP(R, D, RPW)                                                                   \
  {                                                                                           \
    const unsigned grid = (unsigned)((nx / 128) * (ny / (4 * RPW)));                          \
    hipLaunchKernelGGL((march_deep_kernel<R, D>), dim3(grid), dim3(256), 0, 0, a, b, c, o, nx, ny, RPW); \
    CK(hipEventRecord(e0));                                                                   \
    for (int i = 0; i < reps; ++i)                                                            \
      hipLaunchKernelGGL((march_deep_kernel<R, D>), dim3(grid), dim3(256), 0, 0, a, b, c, o, nx, ny, RPW); \
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                                      \
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));                                           \
    char nm[64]; snprintf(nm, 64, "march deep D=%d rows/wave=%d", D, RPW); report(nm, R, ms); \
  }
#define RUN_TILE(R, G)                                                                        \
  {                                                                                           \
    const unsigned grid = (unsigned)((nx / 512) * (ny / G));                                  \
    hipLaunchKernelGGL((tile_kernel<R, G>), dim3(grid), dim3(256), 0, 0, a, b, c, o, nx, ny); \
    CK(hipEventRecord(e0));                                                                   \
    for (int i = 0; i < reps; ++i)                                                            \
      hipLaunchKernelGGL((tile_kernel<R, G>), dim3(grid), dim3(256), 0, 0, a, b, c, o, nx, ny); \
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                                      \
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));                                           \
    char nm[64]; snprintf(nm, 64, "tile 512 x %d rows", G); report(nm, R, ms);                \
  }
  RUN_TILE(2, 2) RUN_TILE(2, 4) RUN_TILE(2, 8) RUN_TILE(3, 2) RUN_TILE(3, 4) RUN_TILE(3, 8) RUN_TILE(2, 1) RUN_TILE(3, 1)
  RUN_DEEP(2, 2, 32) RUN_DEEP(2, 4, 32) RUN_DEEP(2, 8, 32) RUN_DEEP(3, 2, 32) RUN_DEEP(3, 4, 32) RUN_DEEP(3, 8, 32)
  RUN_DEEP(2, 4, 16) RUN_DEEP(3, 4, 16) RUN_DEEP(2, 8, 64) RUN_DEEP(3, 8, 64)
  return 0;
}
