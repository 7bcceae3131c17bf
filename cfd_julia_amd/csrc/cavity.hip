// Lid-driven cavity (18_NS2D_Lid_Driven_Cavity/lid_driven_cavity.jl) and n-level V-cycle
// multigrid (17_Poisson_Solver_Multigrid/mg_N.jl + Common.jl:21-92,229-246) on gfx950.
//
// Fields are (nx+1) x (ny+1) node arrays, x contiguous, pitch nx+2 (even: 16-B rows).
// Stencil / boundary / multigrid kernels keep the reference's expression order and are
// compiled without FMA contraction (Makefile), so given the same inputs they reproduce the
// CPU oracle bit for bit.  The DST-I Poisson (fps_sine) is a real DST-I on the (nx-1) x
// (ny-1) interior in three passes (dst_poisson.hip) with the reference's iden multiplier;
// CFDJ_CAVITY_EXT=1 (and grids the DST kernels do not cover) run it as the periodic FFT
// Poisson of the odd-odd extension onto a (2nx) x (2ny) grid instead (host_common.hpp,
// kSymbolDirichletExt).
#include "host_common.hpp"

namespace cfdj {

namespace {

constexpr int kBX = 64, kBY = 4;

struct CavCoef {
  double aa, bb, gg, hh, dt, c25dt, c13, c23, c23dt;
};

// lid_driven_cavity.jl:124-159 at an interior node from its nine omega and eight psi
// values (c = centre, E/W = i +- 1, N/S = j +- 1); gg inside each term.
struct Nine {
  double c, E, W, N, S, NE, SW, NW, SE;
};
__device__ __forceinline__ double cavity_rhs_vals(const Nine& w, const Nine& s,
                                                  const CavCoef& k) {
  const double j1 = k.gg * ((w.E - w.W) * (s.N - s.S) - (w.N - w.S) * (s.E - s.W));
  const double j2 = k.gg * (w.E * (s.NE - s.SE) - w.W * (s.NW - s.SW) - w.N * (s.NE - s.NW) +
                            w.S * (s.SE - s.SW));
  const double j3 = k.gg * (w.NE * (s.N - s.E) - w.SW * (s.W - s.S) - w.NW * (s.N - s.W) +
                            w.SE * (s.E - s.S));
  const double jac = (j1 + j2 + j3) * k.hh;
  return -jac + (k.aa * (w.E - 2.0 * w.c + w.W) + k.bb * (w.N - 2.0 * w.c + w.S));
}
__device__ __forceinline__ Nine nine_at(const double* __restrict__ a, size_t c, int P) {
  Nine n;
  n.c = a[c];
  n.E = a[c + 1];
  n.W = a[c - 1];
  n.N = a[c + P];
  n.S = a[c - P];
  n.NE = a[c + P + 1];
  n.SW = a[c - P - 1];
  n.NW = a[c + P - 1];
  n.SE = a[c - P + 1];
  return n;
}
__device__ __forceinline__ double cavity_rhs_at(const double* __restrict__ w,
                                                const double* __restrict__ s, size_t c,
                                                int P, const CavCoef& k) {
  return cavity_rhs_vals(nine_at(w, c, P), nine_at(s, c, P), k);
}

template <int STAGE>
__device__ __forceinline__ double cavity_update(double r, double w, double wn,
                                                const CavCoef& k) {
  if constexpr (STAGE == 0) return r;
  else if constexpr (STAGE == 1) return w + k.dt * r;
  else if constexpr (STAGE == 2) return (0.75 * wn + 0.25 * w) + k.c25dt * r;
  else return (k.c13 * wn + k.c23 * w) + k.c23dt * r;
}

// Stage updates of lid_driven_cavity.jl:80, 89-93, 102-106 (interior only).
template <int STAGE>
__global__ __launch_bounds__(kBX* kBY) void cavity_stage_kernel(
    const double* __restrict__ w, const double* __restrict__ s, const double* wn, double* out,
    int nx, int ny, int P, CavCoef k) {
  const int i = 1 + blockIdx.x * kBX + threadIdx.x;
  const int j = 1 + blockIdx.y * kBY + threadIdx.y;
  if (i >= nx || j >= ny) return;
  const size_t c = (size_t)j * P + i;
  const double r = cavity_rhs_at(w, s, c, P, k);
  out[c] = cavity_update<STAGE>(r, w[c], STAGE >= 2 ? wn[c] : 0.0, k);
}

// Row-group variant of the stage kernel with the wall vorticity (bc2, below) fused in: a
// 256-thread workgroup owns 512 consecutive i of 2 consecutive rows j0, j0 + 1 (j0 odd),
// two i per lane loaded as 16 B from the 4 rows j0 - 1 .. j0 + 2 of omega and psi at once;
// workgroups in row-major order, so the chip works on one narrow band of rows and each array
// is one sequential stream.  i-neighbours by lane shuffles, across wavefronts through LDS,
// the two halo columns of the workgroup by one load in the first wavefront.  Node i = 0 of
// the first pair, row ny of the last group and anything outside the interior are loaded
// (clamped) but not updated; instead the lanes and groups next to a wall write that wall's
// omega from psi (lid_driven_cavity.jl:39-51; corners take the bottom / top formula, which
// the reference applies last).  Needs nx a multiple of 512 and ny even.
constexpr int kCavTileCols = 512;
constexpr int kCavXcds = 8;

struct W4 {
  double l, a, b, r;
};

template <int STAGE>
__global__ __launch_bounds__(256) void cavity_stage_tile_kernel(
    const double* __restrict__ w, const double* __restrict__ s, const double* wn, double* out,
    int nx, int ny, int P, CavCoef k, double dx2, double dy2, double dy) {
  constexpr int G = 2, NR = G + 2, NW = 4, kWave = 64;
  __shared__ double left[NW][2 * NR], right[NW][2 * NR];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int strips = nx / kCavTileCols, ngrp = ny / 2;
  int strip = blockIdx.x % strips, grp = blockIdx.x / strips;
  if (strips < kCavXcds && kCavXcds % strips == 0) {  // halo rows stay in one XCD's L2
    const int bands = kCavXcds / strips;
    if (ngrp % bands == 0) {
      const int xcd = blockIdx.x % kCavXcds, i = blockIdx.x / kCavXcds;
      strip = xcd % strips;
      grp = (xcd / strips) * (ngrp / bands) + i;
    }
  }
  const int x0 = strip * kCavTileCols;
  const int x = x0 + 2 * (int)threadIdx.x;  // <= nx - 2
  const int j0 = 1 + grp * G;               // <= ny - 1

  double2 wv[NR], sv[NR], wnv[G];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const size_t row = (size_t)min(j0 - 1 + j, ny) * P;
    wv[j] = *reinterpret_cast<const double2*>(w + row + x);
    sv[j] = *reinterpret_cast<const double2*>(s + row + x);
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    wnv[j] = make_double2(0.0, 0.0);
    if constexpr (STAGE >= 2)
      wnv[j] = *reinterpret_cast<const double2*>(wn + (size_t)min(j0 + j, ny) * P + x);
  }
  static_assert(4 * NR <= kWave, "halo fetch needs one lane per value");
  double halo = 0.0;
  if (threadIdx.x < 4 * NR) {
    const int side = threadIdx.x / (2 * NR), rem = threadIdx.x % (2 * NR);
    const int xh = side == 0 ? max(x0 - 1, 0) : x0 + kCavTileCols;  // <= nx
    const size_t row = (size_t)min(j0 - 1 + rem / 2, ny) * P;
    halo = ((rem & 1) ? s : w)[row + xh];
  }
  if ((lane == 0 && wave > 0) || (lane == kWave - 1 && wave < NW - 1)) {
    double* e = lane == 0 ? right[wave - 1] : left[wave + 1];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      e[2 * j] = lane == 0 ? wv[j].x : wv[j].y;
      e[2 * j + 1] = lane == 0 ? sv[j].x : sv[j].y;
    }
  }
  if (threadIdx.x < 4 * NR) {
    const int side = threadIdx.x / (2 * NR), rem = threadIdx.x % (2 * NR);
    (side == 0 ? left[0] : right[NW - 1])[rem] = halo;
  }
  __syncthreads();
  W4 ww[NR], sw[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    ww[j].a = wv[j].x;
    ww[j].b = wv[j].y;
    sw[j].a = sv[j].x;
    sw[j].b = sv[j].y;
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
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int jr = j0 + j;
    if (jr >= ny) continue;  // row ny of the last group: a wall
    const W4 &wm = ww[j], &wc = ww[j + 1], &wp = ww[j + 2];
    const W4 &sm = sw[j], &sc = sw[j + 1], &sp = sw[j + 2];
    Nine n0, n1, m0, m1;  // cells i = x and i = x + 1
    n0.c = wc.a; n0.E = wc.b; n0.W = wc.l; n0.N = wp.a; n0.S = wm.a;
    n0.NE = wp.b; n0.SW = wm.l; n0.NW = wp.l; n0.SE = wm.b;
    n1.c = wc.b; n1.E = wc.r; n1.W = wc.a; n1.N = wp.b; n1.S = wm.b;
    n1.NE = wp.r; n1.SW = wm.a; n1.NW = wp.a; n1.SE = wm.r;
    m0.c = sc.a; m0.E = sc.b; m0.W = sc.l; m0.N = sp.a; m0.S = sm.a;
    m0.NE = sp.b; m0.SW = sm.l; m0.NW = sp.l; m0.SE = sm.b;
    m1.c = sc.b; m1.E = sc.r; m1.W = sc.a; m1.N = sp.b; m1.S = sm.b;
    m1.NE = sp.r; m1.SW = sm.a; m1.NW = sp.a; m1.SE = sm.r;
    double2 o;
    o.x = cavity_update<STAGE>(cavity_rhs_vals(n0, m0, k), wc.a, wnv[j].x, k);
    o.y = cavity_update<STAGE>(cavity_rhs_vals(n1, m1, k), wc.b, wnv[j].y, k);
    double* orow = out + (size_t)jr * P;
    if (x == 0) {  // node 0 is the left wall
      o.x = (-4.0 * sc.b + 0.5 * sc.r) / dx2;
    }
    *reinterpret_cast<double2*>(orow + x) = o;
    if (x == nx - 2) orow[nx] = (-4.0 * sc.b + 0.5 * sc.a) / dx2;  // right wall
  }
  if (j0 == 1) {  // bottom wall, row 0: psi rows 1 and 2 are sw[1], sw[2]
    double2 o;
    o.x = (-4.0 * sw[1].a + 0.5 * sw[2].a) / dy2;
    o.y = (-4.0 * sw[1].b + 0.5 * sw[2].b) / dy2;
    *reinterpret_cast<double2*>(out + x) = o;
    if (x == nx - 2) out[nx] = (-4.0 * sw[1].r + 0.5 * sw[2].r) / dy2;
  }
  if (j0 == ny - 1) {  // top wall, row ny: psi rows ny - 1 and ny - 2 are sw[1], sw[0]
    double* orow = out + (size_t)ny * P;
    double2 o;
    o.x = (-4.0 * sw[1].a + 0.5 * sw[0].a) / dy2 - 3.0 / dy;
    o.y = (-4.0 * sw[1].b + 0.5 * sw[0].b) / dy2 - 3.0 / dy;
    *reinterpret_cast<double2*>(orow + x) = o;
    if (x == nx - 2) orow[nx] = (-4.0 * sw[1].r + 0.5 * sw[0].r) / dy2 - 3.0 / dy;
  }
}

// lid_driven_cavity.jl:39-51: Jensen wall vorticity.  The reference's bottom/top loop runs
// second and overwrites the corners, so corners take the bottom/top formula.
__global__ __launch_bounds__(256) void bc2_kernel(double* __restrict__ w,
                                                  const double* __restrict__ s, int nx,
                                                  int ny, int P, double dx2, double dy2,
                                                  double dy) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t <= nx) {  // bottom (j = 0) and top (j = ny) rows, all i
    const int i = t;
    w[i] = (-4.0 * s[(size_t)P + i] + 0.5 * s[(size_t)2 * P + i]) / dy2;
    w[(size_t)ny * P + i] =
        (-4.0 * s[(size_t)(ny - 1) * P + i] + 0.5 * s[(size_t)(ny - 2) * P + i]) / dy2 -
        3.0 / dy;
  } else if (t <= nx + ny - 1) {  // left / right columns, j = 1..ny-1
    const int j = t - nx;
    const size_t r = (size_t)j * P;
    w[r] = (-4.0 * s[r + 1] + 0.5 * s[r + 2]) / dx2;
    w[r + nx] = (-4.0 * s[r + nx - 1] + 0.5 * s[r + nx - 2]) / dx2;
  }
}

// Odd-odd extension of the interior of w onto the (2nx) x (2ny) periodic grid (pitch 2nx):
// E(i', j') = sx sy w(|i|, |j|), zero on the lines i' in {0, nx}, j' in {0, ny}.
__global__ __launch_bounds__(256) void odd_extend_kernel(const double* __restrict__ w,
                                                         double* __restrict__ E, int nx,
                                                         int ny, int P) {
  const int ip = blockIdx.x * blockDim.x + threadIdx.x;
  const int jp = blockIdx.y;
  if (ip >= 2 * nx) return;
  const int i = ip <= nx ? ip : 2 * nx - ip;
  const int j = jp <= ny ? jp : 2 * ny - jp;
  double v = 0.0;
  if (i != 0 && i != nx && j != 0 && j != ny) {
    v = w[(size_t)j * P + i];
    if ((ip > nx) != (jp > ny)) v = -v;
  }
  E[(size_t)jp * (2 * nx) + ip] = v;
}

// s[i, j] = psi_ext[j][i] on the interior (the reference's sn boundary stays untouched).
__global__ __launch_bounds__(256) void extract_kernel(const double* __restrict__ X,
                                                      double* __restrict__ s, int nx, int ny,
                                                      int P) {
  const int i = 1 + blockIdx.x * blockDim.x + threadIdx.x;
  const int j = 1 + blockIdx.y;
  if (i >= nx) return;
  s[(size_t)j * P + i] = X[(size_t)j * (2 * nx) + i];
}

// Deterministic two-pass sum of squares over an n0 x n1 block (pitch P) of (a - b) or a.
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const double* __restrict__ a,
                                                            const double* __restrict__ b,
                                                            int i0, int n0, int j0, int n1,
                                                            int P, double* __restrict__ part) {
  __shared__ double red[256];
  double acc = 0.0;
  const long total = (long)n0 * n1;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int j = (int)(e / n0), i = (int)(e % n0);
    const size_t c = (size_t)(j0 + j) * P + (i0 + i);
    const double d = b ? a[c] - b[c] : a[c];
    acc += d * d;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// Workgroup b reduces the partials part[b stride ..] into out[b] (one workgroup per set).
__global__ __launch_bounds__(256) void sumsq_final_kernel(const double* __restrict__ part,
                                                          int nparts, double denom,
                                                          double* __restrict__ out,
                                                          int stride = 0) {
  __shared__ double red[256];
  part += (size_t)blockIdx.x * stride;
  out += blockIdx.x;
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sqrt(red[0] / denom);
}

// Common.jl:239-246
__global__ __launch_bounds__(kBX* kBY) void residual_kernel(const double* __restrict__ f,
                                                            const double* __restrict__ u,
                                                            double* __restrict__ r, int nx,
                                                            int ny, int P, double dx2,
                                                            double dy2) {
  const int i = 1 + blockIdx.x * kBX + threadIdx.x;
  const int j = 1 + blockIdx.y * kBY + threadIdx.y;
  if (i >= nx || j >= ny) return;
  const size_t c = (size_t)j * P + i;
  const double uc = u[c];
  r[c] = f[c] - ((u[c + 1] - 2.0 * uc + u[c - 1]) / dx2 + (u[c + P] - 2.0 * uc + u[c - P]) / dy2);
}

// 15_Poisson_Solver_Gauss_Seidel/gauss_seidel.jl:33-39 (a Jacobi sweep despite the name):
// r = f - lap(u_old) everywhere, then u += r / dd -- ping-pong buffers, same expressions.
__global__ __launch_bounds__(kBX* kBY) void jacobi_kernel(const double* __restrict__ f,
                                                          const double* __restrict__ u,
                                                          double* __restrict__ un,
                                                          double* __restrict__ r, int nx,
                                                          int ny, int P, double dx2, double dy2,
                                                          double dd) {
  const int i = 1 + blockIdx.x * kBX + threadIdx.x;
  const int j = 1 + blockIdx.y * kBY + threadIdx.y;
  if (i >= nx || j >= ny) return;
  const size_t c = (size_t)j * P + i;
  const double uc = u[c];
  const double rc = f[c] - ((u[c + 1] - 2.0 * uc + u[c - 1]) / dx2 +
                            (u[c + P] - 2.0 * uc + u[c - P]) / dy2);
  r[c] = rc;
  un[c] = uc + rc / dd;
}

__global__ __launch_bounds__(256) void negate_kernel(const double* __restrict__ a,
                                                     double* __restrict__ b, size_t n) {
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e < n) b[e] = -a[e];
}

dim3 interior_grid(int nx, int ny) {
  return dim3((nx - 1 + kBX - 1) / kBX, (ny - 1 + kBY - 1) / kBY);
}

// ---- multigrid V-cycle kernels (device-resident convergence control) -------------------
// ctl[0] = converged flag, ctl[1] = number of residual norms recorded so far (hist index).
// Every kernel of a cycle returns at once when the flag is set, so cycles enqueued past the
// converged one (the host enqueues whole cycles without reading the norm back) change
// nothing: the iterate stays the one mg_N.jl:70 breaks on.
__device__ __forceinline__ bool mg_done(const int* ctl) { return ctl != nullptr && ctl[0] != 0; }

// One red-black half sweep of the Common.jl:84-88 update on points with (i + j) % 2 ==
// parity (the reference's lexicographic order is inherently serial; converged solutions
// agree to the solver tolerance, tests/test_gpu_cavity.py).
__global__ __launch_bounds__(kBX* kBY) void mg_rbgs_kernel(const double* __restrict__ f,
                                                           double* __restrict__ u, int nx, int ny,
                                                           int P, double dx2, double dy2,
                                                           double dd, int parity,
                                                           const int* __restrict__ ctl) {
  if (mg_done(ctl)) return;
  const int j = 1 + blockIdx.y * kBY + threadIdx.y;
  const int i = 1 + 2 * (blockIdx.x * kBX + threadIdx.x) + ((j + 1 + parity) & 1);
  if (i >= nx || j >= ny) return;
  const size_t c = (size_t)j * P + i;
  const double uc = u[c];
  const double rt = f[c] - ((u[c + 1] - 2.0 * uc + u[c - 1]) / dx2 +
                            (u[c + P] - 2.0 * uc + u[c - P]) / dy2);
  u[c] = uc + rt / dd;
}

// S full red-black sweeps (2S half sweeps) of the same update in ONE pass over the level:
// a workgroup loads its (128 - 4S) x 24 tile of u and f plus a halo of 2S nodes into LDS, runs the
// half sweeps there (each one valid on a region one node smaller all round: an update needs
// its four neighbours' values of the previous half sweep), and writes the tile to `uout`.
// Every point of the tile sees exactly the neighbour values the separate half-sweep
// launches would give it, so the result is bit-identical to them; HBM traffic per call is
// f + u in + u out (24 B per node) instead of 2S x (f + u + u).  Out of place: neighbouring
// tiles read each other's old values (the caller ping-pongs the two buffers).
//
// RCP: dx^2, dy^2 and the diagonal -2/dx^2 - 2/dy^2 are exact powers of two (any 2^k-cell
// unit box), so the three divisions of the update are multiplications by the exact
// reciprocals passed in their place -- the same bits, a third of the instructions (with the
// data in LDS the kernel is bound by that arithmetic, not by memory).
constexpr int kFsW = 128, kFsTY = 24;  // LDS row of 128 nodes: tile = (128 - 4S) x 24 nodes
// wavefronts per tile on the small levels: the most (up to 16) that divide the tile's rows
constexpr int fs_wide_nw(int ht) {
  return ht % 16 == 0 ? 16 : ht % 14 == 0 ? 14 : ht % 12 == 0 ? 12 : ht % 10 == 0 ? 10 : 4;
}
template <bool RCP>
__device__ __forceinline__ double mg_div(double x, double d) {
  return RCP ? x * d : x / d;
}
//
// ucor != nullptr: the coarse-grid correction of the ascent (Common.jl:50-76 prolongation +
// mg_N.jl:99-101) is added to the interior nodes while the tile is loaded, instead of a
// separate pass over u before the smoothing.
//
// Thread layout: 64 lanes along x (one lane per pair of nodes of a 128-node LDS row: the
// lane's node of the half sweep's colour), NW wavefronts taking every NW-th row: 16 (12
// for the descent's 36-row tile at S = 2), or 4 with 8-9 rows per lane.
//
// DESC (the descent's smoothing call): the halo is two nodes wider, so after the sweeps the
// iterate is valid two nodes beyond the tile, the residual (Common.jl:239-246) one node
// beyond it, and the tile's share of the next steps of the descent comes from LDS instead
// of three more passes over the level: the sum of squares of the residual (the norm of
// Common.jl:229-232, level 0), the residual itself where the one-workgroup coarse kernel
// wants it in memory, and the full-weighting restriction to the next level (Common.jl:21-48;
// its boundary nodes inject the residual's boundary, which is zero) with that level's
// iterate zeroed (mg_N.jl:88) -- the same expressions in the same order as the separate
// kernels.
struct MgDescArgs {
  double* rout;  // residual of this level, or nullptr
  double* part;  // per-workgroup sums of r^2, or nullptr
  double* fc;    // next level's right-hand side, or nullptr
  double* ucz;   // next level's iterate (zeroed), with fc
  int nxc, nyc, Pc;
};

template <int S, bool RCP, bool DESC, int NW>
__global__ __launch_bounds__(64 * NW) void mg_smooth_fused_kernel(const double* __restrict__ f,
                                                              const double* __restrict__ uin,
                                                              double* __restrict__ uout, int nx,
                                                              int ny, int P, double dx2,
                                                              double dy2, double dd,
                                                              const double* __restrict__ ucor,
                                                              int Pc,
                                                              const int* __restrict__ ctl,
                                                              const MgDescArgs da) {
  if (mg_done(ctl)) return;
  constexpr int H = 2 * S + (DESC ? 2 : 0), W = kFsW, TX = W - 2 * H, HT = kFsTY + 2 * H;
  // Only u goes through LDS (neighbours belong to other lanes and wavefronts).  A lane
  // updates nothing but its own two nodes (2 tx, 2 tx + 1) of its rows, so their f, their
  // current u and, of the four neighbours, the lane's other node stay in registers.
  __shared__ double su[HT * W];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int x0 = blockIdx.x * TX - H, y0 = blockIdx.y * kFsTY - H;  // node of local (0, 0)
  // load: one 16-B access per lane covers a whole 128-node row (x0 and the pitch are even,
  // so the pair (gi, gi + 1) is aligned; gi + 1 = nx + 1 is the arrays' padding column);
  // all of a wavefront's rows are requested before the first one is used
  constexpr int ROWS = HT / NW, NT = 64 * NW;
  static_assert(HT % NW == 0, "rows per wavefront");
  const int gi = x0 + 2 * tx;
  const bool xin = gi >= 0 && gi <= nx;
  double2 ru[ROWS], rf[ROWS];
#pragma unroll
  for (int k = 0; k < ROWS; ++k) {
    const int gj = y0 + ty + NW * k;
    ru[k] = make_double2(0.0, 0.0);
    rf[k] = make_double2(0.0, 0.0);
    if (xin && gj >= 0 && gj <= ny) {
      const size_t c = (size_t)gj * P + gi;
      ru[k] = *reinterpret_cast<const double2*>(uin + c);
      rf[k] = *reinterpret_cast<const double2*>(f + c);
    }
  }
#pragma unroll
  for (int k = 0; k < ROWS; ++k) {
    const int lj = ty + NW * k, gj = y0 + lj;
    if (ucor != nullptr && gj >= 1 && gj < ny) {
      const size_t qr = (size_t)(gj >> 1) * Pc;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int g = gi + e;
        if (g >= 1 && g < nx) {
          const size_t q = qr + (g >> 1);
          double p;
          if (!(g & 1) && !(gj & 1)) p = ucor[q];
          else if (!(g & 1)) p = 0.5 * (ucor[q] + ucor[q + Pc]);
          else if (!(gj & 1)) p = 0.5 * (ucor[q] + ucor[q + 1]);
          else p = 0.25 * (ucor[q] + ucor[q + Pc] + ucor[q + 1] + ucor[q + Pc + 1]);
          if (e == 0) ru[k].x += p;
          else ru[k].y += p;
        }
      }
    }
    if (gi + 1 > nx) {  // the padding column is not a node
      ru[k].y = 0.0;
      rf[k].y = 0.0;
    }
    *reinterpret_cast<double2*>(su + lj * W + 2 * tx) = ru[k];
  }
  __syncthreads();
  // f - lap(u) at the lane's node `odd` (local index c) of a row, from the registers (uc,
  // the node's f, the lane's other node `own`: W if odd, else E) and three LDS reads
  auto defect = [dx2, dy2](int odd, int c, double uc, double own, double fo) {
    const double oth = su[odd ? c + 1 : c - 1];
    const double uE = odd ? oth : own, uW = odd ? own : oth;
    return fo - (mg_div<RCP>(uE - 2.0 * uc + uW, dx2) +
                 mg_div<RCP>(su[c + W] - 2.0 * uc + su[c - W], dy2));
  };
#pragma unroll 1
  for (int h = 1; h <= 2 * S; ++h) {
    const int parity = (h - 1) & 1;
    // valid region of this half sweep: local [h, W-1-h] x [h, HT-1-h].  The nodes of one
    // colour are independent of each other, so a lane's rows (every fourth) are unrolled
    // and all their LDS reads are in flight together; the writes follow.
    double res[ROWS];
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
      const int lj = ty + NW * k;
      const int odd = (x0 + y0 + lj + parity) & 1;  // (node x + node y) % 2 == parity
      const int li = 2 * tx + odd;
      const int c = (lj >= 1 && lj <= HT - 2 ? lj : 1) * W + (li >= 1 && li <= W - 2 ? li : 1);
      const double ux = ru[k].x, uy = ru[k].y, fx = rf[k].x, fy = rf[k].y;
      const double uc = odd ? uy : ux;
      const double own = odd ? ux : uy;
      const double fo = odd ? fy : fx;
      res[k] = uc + mg_div<RCP>(defect(odd, c, uc, own, fo), dd);
    }
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
      const int lj = ty + NW * k;
      const int gj = y0 + lj;
      const int odd = (x0 + gj + parity) & 1;
      const int li = 2 * tx + odd;
      const int gx = x0 + li;
      const bool act = lj >= h && lj <= HT - 1 - h && li >= h && li <= W - 1 - h && gx >= 1 &&
                       gx < nx && gj >= 1 && gj < ny;
      if (act) su[lj * W + li] = res[k];
      // value selects, not a store through a selected address: the arrays stay in registers
      ru[k].x = act && !odd ? res[k] : ru[k].x;
      ru[k].y = act && odd ? res[k] : ru[k].y;
    }
    __syncthreads();
  }
  if (2 * tx >= H && 2 * tx < H + TX && gi <= nx) {
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
      const int lj = ty + NW * k, gj = y0 + lj;
      if (lj >= H && lj < H + kFsTY && gj <= ny) {
        if (gi + 1 <= nx) *reinterpret_cast<double2*>(uout + (size_t)gj * P + gi) = ru[k];
        else uout[(size_t)gj * P + gi] = ru[k].x;
      }
    }
  }
  if constexpr (DESC) {
    // residual on the tile and one node around it (zero off the interior): into registers,
    // then -- every lane done with u -- into the LDS buffer in place of u
    constexpr int lo = 2 * S + 1;
    double2 rr[ROWS];
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
      const int lj = ty + NW * k, gj = y0 + lj;
      const int ljc = lj >= 1 && lj <= HT - 2 ? lj : 1;
      double rc[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int li = 2 * tx + e, gx = x0 + li;
        const int c = ljc * W + (li >= 1 && li <= W - 2 ? li : 1);
        const double d = defect(e, c, e ? ru[k].y : ru[k].x, e ? ru[k].x : ru[k].y,
                                e ? rf[k].y : rf[k].x);
        rc[e] = lj >= lo && lj <= HT - 1 - lo && li >= lo && li <= W - 1 - lo && gx >= 1 &&
                        gx < nx && gj >= 1 && gj < ny
                    ? d
                    : 0.0;
      }
      rr[k] = make_double2(rc[0], rc[1]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < ROWS; ++k)
      *reinterpret_cast<double2*>(su + (ty + NW * k) * W + 2 * tx) = rr[k];
    __syncthreads();
    double acc = 0.0;
    if (2 * tx >= H && 2 * tx < H + TX && gi <= nx && (da.rout != nullptr || da.part != nullptr)) {
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        const int lj = ty + NW * k, gj = y0 + lj;
        if (lj >= H && lj < H + kFsTY && gj <= ny) {
          acc += rr[k].x * rr[k].x + rr[k].y * rr[k].y;
          if (da.rout != nullptr) {
            if (gi + 1 <= nx) *reinterpret_cast<double2*>(da.rout + (size_t)gj * P + gi) = rr[k];
            else da.rout[(size_t)gj * P + gi] = rr[k].x;
          }
        }
      }
    }
    if (da.fc != nullptr) {
      const int I0 = (x0 + H) >> 1, J0 = (y0 + H) >> 1;  // x0 + H, y0 + H are even
      for (int e = threadIdx.x; e < (TX / 2) * (kFsTY / 2); e += NT) {
        const int ci = e % (TX / 2), cj = e / (TX / 2);
        const int I = I0 + ci, J = J0 + cj;
        if (I > da.nxc || J > da.nyc) continue;
        double v = 0.0;
        if (I > 0 && I < da.nxc && J > 0 && J < da.nyc) {
          const int c = (H + 2 * cj) * W + H + 2 * ci;
          const double center = 4.0 * su[c];
          const double grid = 2.0 * (su[c + W] + su[c - W] + su[c + 1] + su[c - 1]);
          const double corner = su[c + W + 1] + su[c - W + 1] + su[c + W - 1] + su[c - W - 1];
          v = (center + grid + corner) / 16.0;
        }
        da.fc[(size_t)J * da.Pc + I] = v;
        da.ucz[(size_t)J * da.Pc + I] = 0.0;
      }
    }
    if (da.part != nullptr) {
      __shared__ double red[1024];  // fixed summation tree, whatever NT
      for (int i = threadIdx.x; i < 1024; i += NT) red[i] = i < NT ? acc : 0.0;
      __syncthreads();
      for (int off = 512; off > 0; off >>= 1) {
        for (int i = threadIdx.x; i < off; i += NT) red[i] += red[i + off];
        __syncthreads();
      }
      if (threadIdx.x == 0) da.part[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
    }
  }
}

// Common.jl:239-246 residual; with part != nullptr also this block's sum of r^2 (fixed
// in-block order: the norm of Common.jl:229-232 without a second pass over r).
__global__ __launch_bounds__(kBX* kBY) void mg_residual_kernel(const double* __restrict__ f,
                                                               const double* __restrict__ u,
                                                               double* __restrict__ r, int nx,
                                                               int ny, int P, double dx2,
                                                               double dy2,
                                                               double* __restrict__ part,
                                                               const int* __restrict__ ctl) {
  if (mg_done(ctl)) return;
  __shared__ double red[kBX * kBY];
  const int i = 1 + blockIdx.x * kBX + threadIdx.x;
  const int j = 1 + blockIdx.y * kBY + threadIdx.y;
  double rc = 0.0;
  if (i < nx && j < ny) {
    const size_t c = (size_t)j * P + i;
    const double uc = u[c];
    rc = f[c] - ((u[c + 1] - 2.0 * uc + u[c - 1]) / dx2 + (u[c + P] - 2.0 * uc + u[c - P]) / dy2);
    r[c] = rc;
  }
  if (part == nullptr) return;
  const int t = threadIdx.y * kBX + threadIdx.x;
  red[t] = rc * rc;
  __syncthreads();
  for (int off = kBX * kBY / 2; off > 0; off >>= 1) {
    if (t < off) red[t] += red[t + off];
    __syncthreads();
  }
  if (t == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

// rms = sqrt(sum of the block partials / denom) -> hist[ctl[1]++]; first = 1: the initial
// residual (mg_N.jl:22, no test); else the convergence test of mg_N.jl:70 against hist[0].
__global__ __launch_bounds__(1024) void mg_norm_kernel(const double* __restrict__ part,
                                                       int nparts, double denom,
                                                       double* __restrict__ hist, int hist_cap,
                                                       int* __restrict__ ctl, double tol,
                                                       int first) {
  if (mg_done(ctl)) return;
  __shared__ double red[1024];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 512; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double rms = sqrt(red[0] / denom);
    const int idx = ctl[1];
    if (idx < hist_cap) hist[idx] = rms;
    ctl[1] = idx + 1;
    if (first) ctl[2] = 0;
    if (!first && !(rms / hist[0] > tol)) ctl[0] = 1;  // also stops on hist[0] == 0
  }
}

// Common.jl:21-48: full weighting on the coarse interior, injection on its boundary (the
// reference's bottom/top loops run first, then left/right overwrite the corners -- both
// inject the same node); mg_N.jl:88: the coarse iterate starts at zero.
__global__ __launch_bounds__(kBX* kBY) void mg_restrict_kernel(const double* __restrict__ r,
                                                               double* __restrict__ ec,
                                                               double* __restrict__ uc, int nxf,
                                                               int nyf, int Pf, int nxc, int nyc,
                                                               int Pc,
                                                               const int* __restrict__ ctl) {
  if (mg_done(ctl)) return;
  const int i = blockIdx.x * kBX + threadIdx.x;  // 0..nxc
  const int j = blockIdx.y * kBY + threadIdx.y;  // 0..nyc
  if (i > nxc || j > nyc) return;
  double v;
  if (i == 0 || i == nxc || j == 0 || j == nyc) {
    v = r[(size_t)(j == 0 ? 0 : (j == nyc ? nyf : 2 * j)) * Pf +
          (i == 0 ? 0 : (i == nxc ? nxf : 2 * i))];
  } else {
    const size_t c = (size_t)(2 * j) * Pf + 2 * i;
    const double center = 4.0 * r[c];
    const double grid = 2.0 * (r[c + Pf] + r[c - Pf] + r[c + 1] + r[c - 1]);
    const double corner = r[c + Pf + 1] + r[c - Pf + 1] + r[c + Pf - 1] + r[c - Pf - 1];
    v = (center + grid + corner) / 16.0;
  }
  ec[(size_t)j * Pc + i] = v;
  uc[(size_t)j * Pc + i] = 0.0;
}

// Common.jl:50-76 + mg_N.jl:99-101: u_f[interior] += bilinear prolongation of u_c
// (even/even: injection; one index odd: mean of 2; both odd: mean of 4).
__global__ __launch_bounds__(kBX* kBY) void mg_prolong_add_kernel(const double* __restrict__ uc,
                                                                  double* __restrict__ uf,
                                                                  int nxf, int nyf, int Pf,
                                                                  int Pc,
                                                                  const int* __restrict__ ctl) {
  if (mg_done(ctl)) return;
  const int I = 1 + blockIdx.x * kBX + threadIdx.x;
  const int J = 1 + blockIdx.y * kBY + threadIdx.y;
  if (I >= nxf || J >= nyf) return;
  const int ic = I >> 1, jc = J >> 1;
  const size_t c = (size_t)jc * Pc + ic;
  double p;
  if (!(I & 1) && !(J & 1)) {
    p = uc[c];
  } else if (!(I & 1)) {
    p = 0.5 * (uc[c] + uc[c + Pc]);
  } else if (!(J & 1)) {
    p = 0.5 * (uc[c] + uc[c + 1]);
  } else {
    p = 0.25 * (uc[c] + uc[c + Pc] + uc[c + 1] + uc[c + Pc + 1]);
  }
  uf[(size_t)J * Pf + I] += p;
}

// The coarse levels of a V-cycle (grids of at most 64 cells a side) in ONE workgroup with
// every level's u and f in LDS: descent from the residual of the finest LDS level's parent
// (global memory) to the coarsest grid and the ascent back, the same kernels' arithmetic
// point for point (red-black half sweeps separated by barriers), so the iterates are
// identical to the level-by-level launches -- which cost a dozen launches of a few hundred
// threads per level.
constexpr int kMgCoarseMaxLevels = 8;
constexpr int kMgCoarseCells = 64;
struct MgCoarseArgs {
  int n;                              // coarse levels held in LDS
  int lnx[kMgCoarseMaxLevels], lny[kMgCoarseMaxLevels], lP[kMgCoarseMaxLevels];
  double dx2[kMgCoarseMaxLevels], dy2[kMgCoarseMaxLevels], dd[kMgCoarseMaxLevels];
  int off_u[kMgCoarseMaxLevels], off_f[kMgCoarseMaxLevels], off_r;  // in doubles
  int sweeps_down[kMgCoarseMaxLevels];  // v1, or v2 on the coarsest level (mg_N.jl:91)
  int v3;
  const double* r_in;  // residual of the parent level (global)
  int nxf, nyf, Pf;    // parent level
  double* u_out;       // level 0 of the LDS levels, written back for the parent's correction
  const int* ctl;
};

// Loops over a w-wide index range run over the next power of two and skip the excess, so
// the (row, column) split is a shift and a mask instead of an integer division.
__device__ __forceinline__ int ceil_log2(int w) { return w <= 1 ? 0 : 32 - __clz(w - 1); }

template <bool RCP>
__device__ __forceinline__ void lds_smooth(const double* f, double* u, int nx, int ny, int P,
                                           double dx2, double dy2, double dd, int sweeps) {
  const int hw = (nx + 1) / 2;
  const int sh = ceil_log2(hw), mask = (1 << sh) - 1;
  const int total = (ny - 1) << sh;
  for (int s = 0; s < sweeps; ++s)
    for (int parity = 0; parity < 2; ++parity) {
      for (int e = threadIdx.x; e < total; e += blockDim.x) {
        const int j = 1 + (e >> sh);
        const int i = 1 + 2 * (e & mask) + ((j + 1 + parity) & 1);
        if ((e & mask) < hw && i < nx) {
          const int c = j * P + i;
          const double uc = u[c];
          const double rt = f[c] - (mg_div<RCP>(u[c + 1] - 2.0 * uc + u[c - 1], dx2) +
                                    mg_div<RCP>(u[c + P] - 2.0 * uc + u[c - P], dy2));
          u[c] = uc + mg_div<RCP>(rt, dd);
        }
      }
      __syncthreads();
    }
}

// restriction of a fine residual (any memory) into LDS f, u = 0
__device__ __forceinline__ void lds_restrict(const double* r, int nxf, int nyf, int Pf, double* ec,
                                             double* uc, int nxc, int nyc, int Pc) {
  const int sh = ceil_log2(nxc + 1), mask = (1 << sh) - 1;
  const int total = (nyc + 1) << sh;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int j = e >> sh, i = e & mask;
    if (i > nxc) continue;
    double v;
    if (i == 0 || i == nxc || j == 0 || j == nyc) {
      v = r[(size_t)(j == 0 ? 0 : (j == nyc ? nyf : 2 * j)) * Pf +
            (i == 0 ? 0 : (i == nxc ? nxf : 2 * i))];
    } else {
      const size_t c = (size_t)(2 * j) * Pf + 2 * i;
      const double center = 4.0 * r[c];
      const double grid = 2.0 * (r[c + Pf] + r[c - Pf] + r[c + 1] + r[c - 1]);
      const double corner = r[c + Pf + 1] + r[c - Pf + 1] + r[c + Pf - 1] + r[c - Pf - 1];
      v = (center + grid + corner) / 16.0;
    }
    ec[j * Pc + i] = v;
    uc[j * Pc + i] = 0.0;
  }
  __syncthreads();
}

// RCP: every level's dx^2, dy^2 and diagonal are powers of two and the arguments hold their
// reciprocals (exact): multiplications instead of divisions, the same bits.
template <bool RCP>
__global__ __launch_bounds__(1024) void mg_coarse_kernel(const MgCoarseArgs a) {
  if (mg_done(a.ctl)) return;
  extern __shared__ double sm[];
  double* rb = sm + a.off_r;
  // descent
  lds_restrict(a.r_in, a.nxf, a.nyf, a.Pf, sm + a.off_f[0], sm + a.off_u[0], a.lnx[0], a.lny[0],
               a.lP[0]);
  lds_smooth<RCP>(sm + a.off_f[0], sm + a.off_u[0], a.lnx[0], a.lny[0], a.lP[0], a.dx2[0],
                  a.dy2[0], a.dd[0], a.sweeps_down[0]);
  for (int c = 1; c < a.n; ++c) {
    // residual of level c-1 (Common.jl:239-246), boundary entries zero
    const int nx = a.lnx[c - 1], ny = a.lny[c - 1], P = a.lP[c - 1];
    const double* f = sm + a.off_f[c - 1];
    const double* u = sm + a.off_u[c - 1];
    const int sh = ceil_log2(nx + 1), mask = (1 << sh) - 1;
    for (int e = threadIdx.x; e < ((ny + 1) << sh); e += blockDim.x) {
      const int j = e >> sh, i = e & mask;
      if (i > nx) continue;
      double rc = 0.0;
      if (i >= 1 && i < nx && j >= 1 && j < ny) {
        const int q = j * P + i;
        const double uc = u[q];
        rc = f[q] - (mg_div<RCP>(u[q + 1] - 2.0 * uc + u[q - 1], a.dx2[c - 1]) +
                     mg_div<RCP>(u[q + P] - 2.0 * uc + u[q - P], a.dy2[c - 1]));
      }
      rb[j * P + i] = rc;
    }
    __syncthreads();
    lds_restrict(rb, nx, ny, P, sm + a.off_f[c], sm + a.off_u[c], a.lnx[c], a.lny[c], a.lP[c]);
    lds_smooth<RCP>(sm + a.off_f[c], sm + a.off_u[c], a.lnx[c], a.lny[c], a.lP[c], a.dx2[c],
                    a.dy2[c], a.dd[c], a.sweeps_down[c]);
  }
  // ascent
  for (int c = a.n - 1; c >= 1; --c) {
    const int nxf = a.lnx[c - 1], nyf = a.lny[c - 1], Pf = a.lP[c - 1], Pc = a.lP[c];
    const double* uc = sm + a.off_u[c];
    double* uf = sm + a.off_u[c - 1];
    const int sh = ceil_log2(nxf - 1), mask = (1 << sh) - 1;
    for (int e = threadIdx.x; e < ((nyf - 1) << sh); e += blockDim.x) {
      const int J = 1 + (e >> sh), I = 1 + (e & mask);
      if (I >= nxf) continue;
      const int q = (J >> 1) * Pc + (I >> 1);
      double p;
      if (!(I & 1) && !(J & 1)) p = uc[q];
      else if (!(I & 1)) p = 0.5 * (uc[q] + uc[q + Pc]);
      else if (!(J & 1)) p = 0.5 * (uc[q] + uc[q + 1]);
      else p = 0.25 * (uc[q] + uc[q + Pc] + uc[q + 1] + uc[q + Pc + 1]);
      uf[J * Pf + I] += p;
    }
    __syncthreads();
    lds_smooth<RCP>(sm + a.off_f[c - 1], uf, nxf, nyf, Pf, a.dx2[c - 1], a.dy2[c - 1],
                    a.dd[c - 1], a.v3);
  }
  const double* u0 = sm + a.off_u[0];
  for (int e = threadIdx.x; e < a.lP[0] * (a.lny[0] + 1); e += blockDim.x) a.u_out[e] = u0[e];
}

}  // namespace

// ---- host objects ----------------------------------------------------------------------
// Device-side reduction: rms written to *out (device pointer).
static void launch_rms(const double* a, const double* b, int i0, int n0, int j0, int n1, int P,
                       double denom, double* part, int nparts, double* out, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(nparts), dim3(256), 0, st, a, b, i0, n0, j0,
                     n1, P, part);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, st, part, nparts, denom, out, 0);
  CFDJ_HIP(hipGetLastError());
}

// n-level V-cycle (mg_N.jl:7-114) on device buffers.  The convergence test runs on the
// device (mg_norm_kernel); the host enqueues whole cycles -- one HIP graph replay each --
// and reads the control words back once per batch: as many cycles as the previous solve
// took (time loops re-solve nearly the same problem), then one at a time.
struct Multigrid {
  int nlev = 0, v1 = 2, v2 = 2, v3 = 2;
  std::vector<int> lnx, lny, lP;
  std::vector<double> ldx, ldy;
  std::vector<double*> u, f, r;  // level 0 u/f may alias caller buffers
  // fused multi-sweep smoother (mg_smooth_fused_kernel): second u buffer of the levels that
  // use it; flip[l] = 1 while level l's current iterate lives in alt[l].  Each such level is
  // smoothed twice per cycle (descent, ascent), so a whole cycle restores flip = 0.
  std::vector<double*> alt;
  std::vector<char> fused_lvl, flip;
  double* part = nullptr;        // block partials of the level-0 residual norm
  int nparts = 0;                // ... of mg_residual_kernel's grid (= the buffer's size)
  int nparts_cur = 0;            // ... written by the kernel that produced the current sums
  bool fuse_desc = true;         // descent residual / norm / restriction inside the smoother
  bool keep_r0 = false;          // level 0's residual is wanted in memory (cfdj_mg_residual)
  int* ctl = nullptr;            // device: [0] converged, [1] norms recorded, [2] spare
  double* hist = nullptr;        // device residual-norm history
  int hist_cap = 0;
  int kc = 0;                    // first level held in LDS by mg_coarse_kernel (nlev: none)
  MgCoarseArgs ca;
  bool ca_rcp = false;           // ca's dx2, dy2, dd hold exact reciprocals (powers of two)
  static bool exact_pow2(double d) {
    int e = 0;
    const double m = std::frexp(std::fabs(d), &e);
    return m == 0.5 && e > -500 && e < 500;
  }
  size_t coarse_lds = 0;
  bool use_graph = true;
  hipGraphExec_t gexec = nullptr;
  double *g_u0 = nullptr, *g_f0 = nullptr;
  double g_tol = -1.0;
  int last_count = 1;
  hipStream_t st = nullptr;

  void init(int nx, int ny, double dx, double dy, int n_level, int v1_, int v2_, int v3_,
            hipStream_t s) {
    CFDJ_REQUIRE(n_level >= 1, "n_level must be >= 1");
    CFDJ_REQUIRE((nx >> (n_level - 1)) >= 2 && (ny >> (n_level - 1)) >= 2,
                 "n_level exceeds the possible number of levels (mg_N.jl:26)");
    CFDJ_REQUIRE(nx % (1 << (n_level - 1)) == 0 && ny % (1 << (n_level - 1)) == 0,
                 "nx, ny must be divisible by 2^(n_level-1)");
    nlev = n_level;
    v1 = v1_;
    v2 = v2_;
    v3 = v3_;
    st = s;
    for (int l = 0; l < nlev; ++l) {
      lnx.push_back(l ? lnx[l - 1] / 2 : nx);
      lny.push_back(l ? lny[l - 1] / 2 : ny);
      lP.push_back(lnx[l] + 2);
      ldx.push_back(l ? 2.0 * ldx[l - 1] : dx);
      ldy.push_back(l ? 2.0 * ldy[l - 1] : dy);
      const size_t n = (size_t)lP[l] * (lny[l] + 1);
      u.push_back(l ? dalloc<double>(n) : nullptr);
      f.push_back(l ? dalloc<double>(n) : nullptr);
      r.push_back(dalloc<double>(n));
      CFDJ_HIP(hipMemset(r[l], 0, n * sizeof(double)));
      if (l) CFDJ_HIP(hipMemset(f[l], 0, n * sizeof(double)));
      if (l) CFDJ_HIP(hipMemset(u[l], 0, n * sizeof(double)));
    }
    const dim3 g0 = interior_grid(lnx[0], lny[0]);
    nparts = (int)(g0.x * g0.y);
    part = dalloc<double>(nparts);
    ctl = dalloc<int>(4);
    CFDJ_HIP(hipMemset(ctl, 0, 4 * sizeof(int)));
    const char* ge = std::getenv("CFDJ_MG_GRAPH");
    use_graph = !(ge && ge[0] == '0');
    plan_coarse();
    // levels smoothed by the fused kernel: both of a level's smoothing calls must use it
    // (1..3 sweeps each), the level must not be the coarsest (smoothed once per cycle)
    alt.assign(nlev, nullptr);
    fused_lvl.assign(nlev, 0);
    flip.assign(nlev, 0);
    const char* de = std::getenv("CFDJ_MG_FUSED_DESC");
    fuse_desc = !(de && de[0] == '0');
    const char* fe = std::getenv("CFDJ_MG_FUSED_SMOOTH");
    const bool want = !(fe && fe[0] == '0');
    auto ok = [](int v) { return v >= 1 && v <= 3; };
    for (int l = 0; l < nlev && want; ++l) {
      const bool twice = l < nlev - 1 && (l < kc);
      if (twice && lnx[l] >= 128 && lny[l] >= 128 && ok(v1) && ok(v3)) {
        fused_lvl[l] = 1;
        alt[l] = dalloc<double>((size_t)lP[l] * (lny[l] + 1));
        CFDJ_HIP(hipMemset(alt[l], 0, (size_t)lP[l] * (lny[l] + 1) * sizeof(double)));
      }
    }
  }
  double* ucur(int l) const { return flip[l] ? alt[l] : u[l]; }

  // Levels kc.. live in LDS when they all fit (every grid <= 64 cells a side).
  void plan_coarse() {
    kc = nlev;
    const char* ce = std::getenv("CFDJ_MG_COARSE");
    if (ce && ce[0] == '0') return;
    int first = nlev;
    for (int l = 1; l < nlev; ++l)
      if (lnx[l] <= kMgCoarseCells && lny[l] <= kMgCoarseCells) {
        first = l;
        break;
      }
    if (first >= nlev || nlev - first > kMgCoarseMaxLevels) return;
    size_t off = 0;
    ca = MgCoarseArgs();
    ca_rcp = true;
    ca.n = nlev - first;
    for (int c = 0; c < ca.n; ++c) {
      const int l = first + c;
      ca.lnx[c] = lnx[l];
      ca.lny[c] = lny[l];
      ca.lP[c] = lP[l];
      ca.dx2[c] = ldx[l] * ldx[l];
      ca.dy2[c] = ldy[l] * ldy[l];
      ca.dd[c] = -2.0 / ca.dx2[c] - 2.0 / ca.dy2[c];
      ca_rcp = ca_rcp && exact_pow2(ca.dx2[c]) && exact_pow2(ca.dy2[c]) && exact_pow2(ca.dd[c]);
      ca.sweeps_down[c] = l < nlev - 1 ? v1 : v2;
      const size_t n = (size_t)lP[l] * (lny[l] + 1);
      ca.off_u[c] = (int)off;
      off += n;
      ca.off_f[c] = (int)off;
      off += n;
    }
    ca.off_r = (int)off;
    off += (size_t)lP[first] * (lny[first] + 1);
    if (off * sizeof(double) > 150 * 1024) return;
    coarse_lds = off * sizeof(double);
    ca.v3 = v3;
    ca.r_in = r[first - 1];
    ca.nxf = lnx[first - 1];
    ca.nyf = lny[first - 1];
    ca.Pf = lP[first - 1];
    ca.u_out = u[first];
    ca.ctl = ctl;
    if (ca_rcp)  // exact reciprocals in place of the divisors
      for (int c = 0; c < ca.n; ++c) {
        ca.dx2[c] = 1.0 / ca.dx2[c];
        ca.dy2[c] = 1.0 / ca.dy2[c];
        ca.dd[c] = 1.0 / ca.dd[c];
      }
    CFDJ_HIP(hipFuncSetAttribute(
        ca_rcp ? reinterpret_cast<const void*>(mg_coarse_kernel<true>)
               : reinterpret_cast<const void*>(mg_coarse_kernel<false>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)coarse_lds));
    kc = first;
  }

  void destroy() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    gexec = nullptr;
    for (int l = 1; l < nlev; ++l) {
      dfree(u[l]);
      dfree(f[l]);
    }
    for (auto& p : r) dfree(p);
    for (auto& p : alt) dfree(p);
    dfree(part);
    dfree(ctl);
    dfree(hist);
  }
  // `sweeps` red-black sweeps on level l; cor >= 0: first add the prolongation of level
  // cor's iterate (the ascent's correction step).
  void smooth(int l, int sweeps, int cor = -1) { smooth(l, sweeps, cor, nullptr); }
  // desc != nullptr: the descent's call, with the residual / norm partials / restriction
  // of the level fused in (fused levels only: see fuses()).
  bool fuses(int l, int sweeps) const { return fused_lvl[l] && sweeps >= 1 && sweeps <= 3; }
  void smooth(int l, int sweeps, int cor, const MgDescArgs* desc) {
    const double dx2 = ldx[l] * ldx[l], dy2 = ldy[l] * ldy[l];
    const double dd = -2.0 / dx2 - 2.0 / dy2;
    const bool fuse = fuses(l, sweeps);
    if (desc && !fuse) throw Error{CFDJ_ERR_STATE, "multigrid: fused descent on an unfused level"};
    if (cor >= 0 && !fuse)
      hipLaunchKernelGGL(mg_prolong_add_kernel, interior_grid(lnx[l], lny[l]), dim3(kBX, kBY), 0,
                         st, ucur(cor), ucur(l), lnx[l], lny[l], lP[l], lP[cor], ctl);
    if (fuse) {
      const double* ucor = cor >= 0 ? ucur(cor) : nullptr;
      const int Pc = cor >= 0 ? lP[cor] : 0;
      // tile width of mg_smooth_fused_kernel<sweeps, ., desc>
      const int tx = kFsW - 4 * sweeps - (desc ? 4 : 0);
      const dim3 g((lnx[l] + 1 + tx - 1) / tx, (lny[l] + 1 + kFsTY - 1) / kFsTY);
      const double* in = ucur(l);
      flip[l] ^= 1;
      double* out = ucur(l);
      const bool rcp = exact_pow2(dx2) && exact_pow2(dy2) && exact_pow2(dd);
      const double a = rcp ? 1.0 / dx2 : dx2, b = rcp ? 1.0 / dy2 : dy2, c = rcp ? 1.0 / dd : dd;
      const MgDescArgs da = desc ? *desc : MgDescArgs{};
      if (desc && desc->part) {
        if ((int)(g.x * g.y) > nparts)
          throw Error{CFDJ_ERR_STATE, "multigrid: norm partial buffer too small"};
        nparts_cur = (int)(g.x * g.y);
      }
      // wavefronts per tile: as many as divide the tile's rows (fs_wide_nw) -- measured
      // faster on every level of the 2048^2 cavity (small levels: the kernel's cost is one
      // tile's latency; large ones: more rows in flight per CU) than 4 wavefronts taking
      // 8-9 rows each, which CFDJ_MG_WIDE_TILES=0 restores
      static const bool wide = [] {
        const char* e = std::getenv("CFDJ_MG_WIDE_TILES");
        return !(e && e[0] == '0');
      }();
#define CFDJ_FS(S, R, D, NW)                                                                \
  hipLaunchKernelGGL((mg_smooth_fused_kernel<S, R, D, NW>), g, dim3(64 * NW), 0, st, f[l], in, \
                     out, lnx[l], lny[l], lP[l], a, b, c, ucor, Pc, ctl, da)
#define CFDJ_FS_R(S, R)                                                       \
  do {                                                                        \
    if (desc) {                                                               \
      if (wide) CFDJ_FS(S, R, true, (fs_wide_nw(kFsTY + 4 * S + 4)));         \
      else CFDJ_FS(S, R, true, 4);                                            \
    } else {                                                                  \
      if (wide) CFDJ_FS(S, R, false, (fs_wide_nw(kFsTY + 4 * S)));            \
      else CFDJ_FS(S, R, false, 4);                                           \
    }                                                                         \
  } while (0)
#define CFDJ_FS_S(S)            \
  do {                          \
    if (rcp) CFDJ_FS_R(S, true); \
    else CFDJ_FS_R(S, false);   \
  } while (0)
      switch (sweeps) {
        case 1: CFDJ_FS_S(1); break;
        case 2: CFDJ_FS_S(2); break;
        default: CFDJ_FS_S(3); break;
      }
#undef CFDJ_FS_R
#undef CFDJ_FS_S
#undef CFDJ_FS
      return;
    }
    dim3 g((lnx[l] / 2 + kBX - 1) / kBX, (lny[l] - 1 + kBY - 1) / kBY);
    for (int s = 0; s < sweeps; ++s)
      for (int parity = 0; parity < 2; ++parity)
        hipLaunchKernelGGL(mg_rbgs_kernel, g, dim3(kBX, kBY), 0, st, f[l], ucur(l), lnx[l],
                           lny[l], lP[l], dx2, dy2, dd, parity, ctl);
  }
  void residual(int l, bool with_norm, bool always = false) {
    hipLaunchKernelGGL(mg_residual_kernel, interior_grid(lnx[l], lny[l]), dim3(kBX, kBY), 0, st,
                       f[l], ucur(l), r[l], lnx[l], lny[l], lP[l], ldx[l] * ldx[l],
                       ldy[l] * ldy[l], with_norm ? part : nullptr, always ? nullptr : ctl);
    if (with_norm) nparts_cur = nparts;
  }
  void norm0(double tol, bool first) {  // Common.jl:229-232 of level 0's residual
    hipLaunchKernelGGL(mg_norm_kernel, dim3(1), dim3(1024), 0, st, part, nparts_cur,
                       (double)(lnx[0] - 1) * (lny[0] - 1), hist, hist_cap, ctl, tol,
                       first ? 1 : 0);
  }
  void restrict_to(int k) {  // residual of level k - 1 -> f[k], u[k] = 0
    hipLaunchKernelGGL(mg_restrict_kernel,
                       dim3((lnx[k] + 1 + kBX - 1) / kBX, (lny[k] + 1 + kBY - 1) / kBY),
                       dim3(kBX, kBY), 0, st, r[k - 1], f[k], ucur(k), lnx[k - 1], lny[k - 1],
                       lP[k - 1], lnx[k], lny[k], lP[k], ctl);
  }

  // One iteration of the mg_N.jl:53-106 loop body.  Descent on the levels above the
  // one-workgroup coarse kernel: smoothing, residual (level 0: its norm and the convergence
  // test), restriction to the next level -- one kernel per level where the smoother is the
  // fused one, else one kernel per step.
  void cycle(double tol) {
    const int L = kc < nlev ? kc : nlev;  // levels 0..L-1 run as grid-wide kernels
    for (int l = 0; l < L; ++l) {
      const int sweeps = l < nlev - 1 ? v1 : v2;
      const bool next = l + 1 < L;                   // restriction to a grid-wide level
      const bool coarse = l == L - 1 && kc < nlev;   // residual read by the coarse kernel
      if (fuse_desc && fuses(l, sweeps) && (next || coarse)) {
        MgDescArgs da{};
        da.part = l == 0 ? part : nullptr;
        da.rout = coarse || (l == 0 && keep_r0) ? r[l] : nullptr;
        if (next) {
          da.fc = f[l + 1];
          da.ucz = ucur(l + 1);
          da.nxc = lnx[l + 1];
          da.nyc = lny[l + 1];
          da.Pc = lP[l + 1];
        }
        smooth(l, sweeps, -1, &da);
        if (l == 0) norm0(tol, false);
        continue;
      }
      smooth(l, sweeps);
      if (l == 0) {
        residual(0, true);
        norm0(tol, false);
      } else if (next || coarse) {
        residual(l, false);
      }
      if (next) restrict_to(l + 1);
    }
    if (kc < nlev) {
      if (ca_rcp) hipLaunchKernelGGL(mg_coarse_kernel<true>, dim3(1), dim3(1024), coarse_lds, st, ca);
      else hipLaunchKernelGGL(mg_coarse_kernel<false>, dim3(1), dim3(1024), coarse_lds, st, ca);
    }
    for (int k = (kc < nlev ? kc : nlev - 1); k >= 1; --k) smooth(k - 1, v3, k);
    CFDJ_HIP(hipGetLastError());
    for (int l = 0; l < nlev; ++l)
      if (flip[l]) throw Error{CFDJ_ERR_STATE, "multigrid: smoothing buffers out of phase"};
  }

  void launch_cycles(int n, double tol) {
    if (!use_graph) {
      for (int i = 0; i < n; ++i) cycle(tol);
      return;
    }
    if (!gexec || g_u0 != u[0] || g_f0 != f[0] || g_tol != tol) {
      if (gexec) (void)hipGraphExecDestroy(gexec);
      gexec = nullptr;
      hipGraph_t g = nullptr;
      CFDJ_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      try {
        cycle(tol);
      } catch (...) {
        (void)hipStreamEndCapture(st, &g);
        if (g) (void)hipGraphDestroy(g);
        throw;
      }
      CFDJ_HIP(hipStreamEndCapture(st, &g));
      const hipError_t e = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      CFDJ_HIP(e);
      g_u0 = u[0];
      g_f0 = f[0];
      g_tol = tol;
    }
    for (int i = 0; i < n; ++i) CFDJ_HIP(hipGraphLaunch(gexec, st));
  }

  // Solve on level-0 buffers u0 (in/out, boundary = Dirichlet data) and f0 (pitch nx+2).
  int solve(double* u0, double* f0, double tol, int max_iter, std::vector<double>* hist_out) {
    u[0] = u0;
    f[0] = f0;
    const int want = (hist_out ? max_iter : 0) + 2;
    if (want > hist_cap) {  // the history is kept only when the caller asks for it
      dfree(hist);
      hist = dalloc<double>(want);
      hist_cap = want;
      if (gexec) (void)hipGraphExecDestroy(gexec);  // the norm node holds the old pointer
      gexec = nullptr;
    }
    CFDJ_HIP(hipMemsetAsync(ctl, 0, 4 * sizeof(int), st));
    residual(0, true);
    norm0(tol, true);
    int host_ctl[4] = {0, 0, 0, 0};
    int launched = 0;
    int batch = last_count < 1 ? 1 : last_count;
    while (launched < max_iter) {
      if (batch > max_iter - launched) batch = max_iter - launched;
      launch_cycles(batch, tol);
      launched += batch;
      CFDJ_HIP(hipMemcpyAsync(host_ctl, ctl, sizeof(host_ctl), hipMemcpyDeviceToHost, st));
      CFDJ_HIP(hipStreamSynchronize(st));
      if (host_ctl[0]) break;
      batch = 1;
    }
    const int it = max_iter > 0 ? host_ctl[1] - 1 : 0;
    if (max_iter == 0) CFDJ_HIP(hipStreamSynchronize(st));
    last_count = it;
    // the converged iterate is the output of the cycle's first smoothing call (mg_N.jl:56,
    // 70): with the fused smoother on level 0 it sits in the second buffer
    if (host_ctl[0] && fused_lvl[0])
      CFDJ_HIP(hipMemcpyAsync(u0, alt[0], (size_t)lP[0] * (lny[0] + 1) * sizeof(double),
                              hipMemcpyDeviceToDevice, st));
    if (hist_out) {
      hist_out->resize((size_t)it + 1);
      CFDJ_HIP(hipMemcpyAsync(hist_out->data(), hist, ((size_t)it + 1) * sizeof(double),
                              hipMemcpyDeviceToHost, st));
      CFDJ_HIP(hipStreamSynchronize(st));
    }
    return it;
  }
};

}  // namespace cfdj

using namespace cfdj;

// =====================================================================================
// Multigrid handle (mg_N.jl:7-114)
// =====================================================================================
struct cfdj_mg {
  int device = -1, nx = 0, ny = 0;
  hipStream_t stream = nullptr;
  Multigrid mg;
  double *u = nullptr, *f = nullptr;
  ~cfdj_mg() {
    mg.destroy();
    dfree(u);
    dfree(f);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// =====================================================================================
// Lid-driven cavity handle (lid_driven_cavity.jl:58-118)
// =====================================================================================
struct cfdj_cavity {
  int device = -1, nx = 0, ny = 0, P = 0;
  double dx = 0, dy = 0, re = 0;
  hipStream_t stream = nullptr;
  double *wn = nullptr, *wa = nullptr, *wb = nullptr;  // omega^n and the two stage buffers
  double *sn = nullptr, *sp = nullptr;                 // psi and the previous step's psi
  // DST Poisson on the odd-odd (2nx) x (2ny) extension
  Symbol sym;
  Plans plans;
  rocfft_plan fwd = nullptr, inv = nullptr;
  Fused fused;
  bool use_fused = false;
  double* ext = nullptr;   // extension / psi_ext (2nx x 2ny real)
  double* ext2 = nullptr;  // rocFFT path output
  double2* spec = nullptr;
  // DST-I on the cavity's own interior (dst_poisson.hip; powers of two 512..4096)
  bool use_dst = false;
  int dst_half = 0;  // passes on the half-length DST kernels (dst_half_passes)
  double2* dstT = nullptr;
  double2 *twX = nullptr, *twY = nullptr;
  int ncu = 256;
  // multigrid alternative
  int poisson = CFDJ_CAVITY_DST;
  Multigrid mg;
  bool mg_ready = false;
  double mg_tol = 1e-9;
  int mg_max_iter = 100000;
  double* mg_f = nullptr;
  long mg_iters = 0;
  // rms
  double* part = nullptr;
  double* d_rms = nullptr;
  int rms_cap = 0;
  static constexpr int kParts = 2048;  // >= the workgroups of any partial-sum producer
  static constexpr int kRmsBatch = 32;  // steps whose partial sums share one reduction launch
  int rms_pending = 0, rms_first = 0;

  size_t field() const { return (size_t)P * (ny + 1); }

  DstPoissonArgs dst_args(const double* w, double* s) const {
    DstPoissonArgs a;
    a.nx = nx;
    a.ny = ny;
    a.P = P;
    a.JT = ny;
    a.w = w;
    a.s = s;
    a.T = dstT;
    a.tx = sym.cx;
    a.ty = sym.cy;
    a.scale = sym.scale;
    a.neg = true;
    a.twX = twX;
    a.twY = twY;
    a.ncu = ncu;
    a.sprev = nullptr;
    a.part = nullptr;
    a.half = dst_half;
    return a;
  }

  void dst_poisson(const double* w, double* s) {  // s_interior = fps_sine(-w)
    if (use_dst) {
      const DstPoissonArgs a = dst_args(w, s);
      for (int pass = 0; pass < 3; ++pass) launch_dst_poisson_pass(pass, a, stream);
      return;
    }
    const int NX = 2 * nx, NY = 2 * ny;
    hipLaunchKernelGGL(odd_extend_kernel, dim3((NX + 255) / 256, NY), dim3(256), 0, stream, w,
                       ext, nx, ny, P);
    CFDJ_HIP(hipGetLastError());
    double* psi = ext;
    if (use_fused) {
      const FusedPoissonArgs a = fused.args(sym, ext, ext, spec, true);
      for (int pass = 0; pass < 3; ++pass) launch_fused_poisson_pass(pass, a, stream);
    } else {
      plans.exec(fwd, ext, spec);
      launch_divide(sym.divide(spec, sym.nxh, NY, sym.nxh, 0, true), stream);
      plans.exec(inv, spec, ext2);
      psi = ext2;
    }
    hipLaunchKernelGGL(extract_kernel, dim3((nx - 1 + 255) / 256, ny - 1), dim3(256), 0, stream,
                       psi, s, nx, ny, P);
    CFDJ_HIP(hipGetLastError());
  }

  void mg_poisson(const double* w, double* s) {  // s (warm start, boundary 0) <- MG(-w)
    hipLaunchKernelGGL(negate_kernel, dim3((unsigned)((field() + 255) / 256)), dim3(256), 0,
                       stream, w, mg_f, field());
    CFDJ_HIP(hipGetLastError());
    mg_iters += mg.solve(s, mg_f, mg_tol, mg_max_iter, nullptr);
  }

  void poisson_solve(const double* w, double* s) {
    if (poisson == CFDJ_CAVITY_MG) mg_poisson(w, s);
    else dst_poisson(w, s);
  }

  CavCoef coef(double dt) const {
    CavCoef k;
    k.aa = 1.0 / (re * (dx * dx));
    k.bb = 1.0 / (re * (dy * dy));
    k.gg = 1.0 / ((4.0 * dx) * dy);
    k.hh = 1.0 / 3.0;
    k.dt = dt;
    k.c25dt = 0.25 * dt;
    k.c13 = 1.0 / 3.0;
    k.c23 = 2.0 / 3.0;
    k.c23dt = (2.0 / 3.0) * dt;
    return k;
  }

  void stage(int st_, const double* w, double* out, double dt) { stage(st_, w, out, dt, sn); }
  void stage(int st_, const double* w, double* out, double dt, const double* sn) {
    const CavCoef k = coef(dt);
    const dim3 g = interior_grid(nx, ny), b(kBX, kBY);
    switch (st_) {
      case 0: hipLaunchKernelGGL(cavity_stage_kernel<0>, g, b, 0, stream, w, sn, wn, out, nx, ny, P, k); break;
      case 1: hipLaunchKernelGGL(cavity_stage_kernel<1>, g, b, 0, stream, w, sn, wn, out, nx, ny, P, k); break;
      case 2: hipLaunchKernelGGL(cavity_stage_kernel<2>, g, b, 0, stream, w, sn, wn, out, nx, ny, P, k); break;
      default: hipLaunchKernelGGL(cavity_stage_kernel<3>, g, b, 0, stream, w, sn, wn, out, nx, ny, P, k); break;
    }
    CFDJ_HIP(hipGetLastError());
  }

  // One RK stage on the interior plus the wall vorticity of the result, both from the same
  // psi: one fused row-group kernel where the grid allows, else the two kernels.
  // CFDJ_CAVITY_TILE=0 at handle creation keeps the two separate kernels (A/B, tests)
  bool tile_ok = [] {
    const char* e = std::getenv("CFDJ_CAVITY_TILE");
    return !(e && e[0] == '0');
  }();
  void stage_bc(int st_, const double* w, double* out, double dt, const double* psi) {
    if (tile_ok && st_ >= 1 && nx % kCavTileCols == 0 && ny % 2 == 0) {
      const CavCoef k = coef(dt);
      const dim3 g((unsigned)((nx / kCavTileCols) * (ny / 2))), b(256);
      const double dx2 = dx * dx, dy2 = dy * dy;
      switch (st_) {
        case 1: hipLaunchKernelGGL(cavity_stage_tile_kernel<1>, g, b, 0, stream, w, psi, wn, out, nx, ny, P, k, dx2, dy2, dy); break;
        case 2: hipLaunchKernelGGL(cavity_stage_tile_kernel<2>, g, b, 0, stream, w, psi, wn, out, nx, ny, P, k, dx2, dy2, dy); break;
        default: hipLaunchKernelGGL(cavity_stage_tile_kernel<3>, g, b, 0, stream, w, psi, wn, out, nx, ny, P, k, dx2, dy2, dy); break;
      }
      CFDJ_HIP(hipGetLastError());
      return;
    }
    stage(st_, w, out, dt, psi);
    bc2(out, psi);
  }

  void bc2(double* w) { bc2(w, sn); }
  void bc2(double* w, const double* sn) {
    hipLaunchKernelGGL(bc2_kernel, dim3((nx + ny + 255) / 256), dim3(256), 0, stream, w, sn,
                       nx, ny, P, dx * dx, dy * dy, dy);
    CFDJ_HIP(hipGetLastError());
  }

  // rms of the steps whose partial sums are waiting -> d_rms[rms_first ..]
  void flush_rms() {
    if (rms_pending == 0) return;
    hipLaunchKernelGGL(sumsq_final_kernel, dim3(rms_pending), dim3(256), 0, stream, part,
                       dst_rows_grid(nx, ny, ncu, dst_half), (double)(nx + 1) * (ny + 1),
                       d_rms + rms_first, kParts);
    CFDJ_HIP(hipGetLastError());
    rms_pending = 0;
  }

  // lid_driven_cavity.jl:75-114; rms of step k into d_rms[k] (DST path: after flush_rms)
  void step(double dt, int k) {
    if (use_dst && poisson == CFDJ_CAVITY_DST) {
      // the three solves write the other psi buffer (its boundary equals sn's: upload),
      // so the previous step's psi survives for the RMS without a copy; the last row pass
      // leaves the per-workgroup sums of (psi_new - psi_old)^2
      double* A = sn;
      double* B = sp;
      stage_bc(1, wn, wa, dt, A);
      DstPoissonArgs a = dst_args(wa, B);
      for (int pass = 0; pass < 3; ++pass) launch_dst_poisson_pass(pass, a, stream);
      stage_bc(2, wa, wb, dt, B);
      a = dst_args(wb, B);
      for (int pass = 0; pass < 3; ++pass) launch_dst_poisson_pass(pass, a, stream);
      stage_bc(3, wb, wn, dt, B);
      a = dst_args(wn, B);
      a.sprev = A;
      // the partial sums of up to kRmsBatch steps wait in their own slots for one reduction
      // launch (a one-workgroup kernel per step cost 4.8 us of a 306 us step at 2048^2)
      a.part = part + (size_t)rms_pending * kParts;
      for (int pass = 0; pass < 3; ++pass) launch_dst_poisson_pass(pass, a, stream);
      if (rms_pending == 0) rms_first = k;
      if (++rms_pending == kRmsBatch) flush_rms();
      sn = B;
      sp = A;
      return;
    }
    CFDJ_HIP(hipMemcpyAsync(sp, sn, field() * sizeof(double), hipMemcpyDeviceToDevice, stream));
    stage_bc(1, wn, wa, dt, sn);  // wt = wn + dt r(wn, sn)
    poisson_solve(wa, sn);
    stage_bc(2, wa, wb, dt, sn);  // wt = (.75wn + .25wt) + .25dt r(wt, sn)
    poisson_solve(wb, sn);
    stage_bc(3, wb, wn, dt, sn);  // wn = ((1/3)wn + (2/3)wt) + (2/3)dt r(wt, sn)
    poisson_solve(wn, sn);
    launch_rms(sn, sp, 0, nx + 1, 0, ny + 1, P, (double)(nx + 1) * (ny + 1), part, kParts,
               d_rms + k, stream);
  }

  ~cfdj_cavity() {
    if (stream) (void)hipStreamSynchronize(stream);
    dfree(wn);
    dfree(wa);
    dfree(wb);
    dfree(sn);
    dfree(sp);
    sym.destroy();
    plans.destroy();
    fused.destroy();
    dfree(ext);
    dfree(ext2);
    dfree(spec);
    dfree(dstT);
    if (twY != twX) dfree(twY);
    dfree(twX);
    if (mg_ready) mg.destroy();
    dfree(mg_f);
    dfree(part);
    dfree(d_rms);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

void copy_in(double* d, int P, const double* h, long ld, int nx, int ny, hipStream_t st) {
  CFDJ_HIP(hipMemcpy2DAsync(d, P * sizeof(double), h, ld * sizeof(double),
                            (nx + 1) * sizeof(double), ny + 1, hipMemcpyHostToDevice, st));
}
void copy_out(double* h, long ld, const double* d, int P, int nx, int ny, hipStream_t st) {
  CFDJ_HIP(hipMemcpy2DAsync(h, ld * sizeof(double), d, P * sizeof(double),
                            (nx + 1) * sizeof(double), ny + 1, hipMemcpyDeviceToHost, st));
}

}  // namespace

extern "C" {

int cfdj_cavity_create(int nx, int ny, double dx, double dy, double re, int device,
                       cfdj_cavity** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr, "out is NULL");
    *out = nullptr;
    CFDJ_REQUIRE(nx >= 4 && ny >= 4, "nx, ny must be >= 4 (bc2 reads s[3, j])");
    CFDJ_REQUIRE(dx > 0 && dy > 0 && std::isfinite(re) && re != 0.0, "bad dx, dy or re");
    fft_setup();
    select_device(device);
    std::unique_ptr<cfdj_cavity> h(new cfdj_cavity);
    CFDJ_HIP(hipGetDevice(&h->device));
    CFDJ_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->nx = nx;
    h->ny = ny;
    h->dx = dx;
    h->dy = dy;
    h->re = re;
    h->P = nx + 2;
    const size_t n = h->field();
    for (double** p : {&h->wn, &h->wa, &h->wb, &h->sn, &h->sp}) {
      *p = dalloc<double>(n);
      CFDJ_HIP(hipMemset(*p, 0, n * sizeof(double)));
    }
    const int NX = 2 * nx, NY = 2 * ny;
    h->sym.init(NX, NY, dx, dy, 0.0, kSymbolDirichletExt);
    const char* ext_env = std::getenv("CFDJ_CAVITY_EXT");  // A/B: the extension-grid solver
    if (dst_poisson_supported(nx, ny) && !(ext_env && ext_env[0] == '1')) {
      h->use_dst = true;
      h->dst_half = dst_half_passes(nx, ny);
      h->dstT = dalloc<double2>((size_t)(nx / 2) * ny);
      h->twX = twiddle_table(NX);
      h->twY = NY == NX ? h->twX : twiddle_table(NY);
      CFDJ_HIP(hipDeviceGetAttribute(&h->ncu, hipDeviceAttributeMultiprocessorCount, h->device));
      h->part = dalloc<double>((size_t)cfdj_cavity::kParts * cfdj_cavity::kRmsBatch);
      *out = h.release();
      return;
    }
    h->ext = dalloc<double>((size_t)NX * NY);
    h->spec = dalloc<double2>((size_t)(NX / 2 + 1) * NY);
    if (fused_ok(NX, NY, 1)) {
      h->fused.init(NX, NY);
      h->use_fused = true;
    } else {
      size_t lens[2] = {(size_t)NX, (size_t)NY};
      h->fwd = h->plans.add(rocfft_transform_type_real_forward, rocfft_placement_notinplace, 2,
                            lens, 1, nullptr);
      h->inv = h->plans.add(rocfft_transform_type_real_inverse, rocfft_placement_notinplace, 2,
                            lens, 1, nullptr);
      h->plans.finalize(h->stream);
      h->ext2 = dalloc<double>((size_t)NX * NY);
    }
    h->part = dalloc<double>((size_t)cfdj_cavity::kParts * cfdj_cavity::kRmsBatch);
    *out = h.release();
  });
}

int cfdj_cavity_set_poisson(cfdj_cavity* h, int solver, int n_level, int v1, int v2, int v3,
                            double tol, int max_iter) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(solver == CFDJ_CAVITY_DST || solver == CFDJ_CAVITY_MG, "bad solver");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    if (solver == CFDJ_CAVITY_MG) {
      CFDJ_REQUIRE(tol > 0 && max_iter >= 1 && v1 >= 0 && v2 >= 0 && v3 >= 0, "bad MG args");
      if (h->mg_ready) h->mg.destroy();
      h->mg = Multigrid();
      h->mg.init(h->nx, h->ny, h->dx, h->dy, n_level, v1, v2, v3, h->stream);
      h->mg_ready = true;
      if (!h->mg_f) {
        h->mg_f = dalloc<double>(h->field());
        CFDJ_HIP(hipMemset(h->mg_f, 0, h->field() * sizeof(double)));
      }
      h->mg_tol = tol;
      h->mg_max_iter = max_iter;
    }
    h->poisson = solver;
  });
}

int cfdj_cavity_upload(cfdj_cavity* h, const double* wn, long ldw, const double* sn, long lds) {
  return guard([&] {
    CFDJ_REQUIRE(h && wn && sn, "NULL argument");
    CFDJ_REQUIRE(ldw >= h->nx + 1 && lds >= h->nx + 1, "leading dimension too small");
    select_device(h->device);
    copy_in(h->wn, h->P, wn, ldw, h->nx, h->ny, h->stream);
    copy_in(h->sn, h->P, sn, lds, h->nx, h->ny, h->stream);
    // both psi buffers carry the caller's boundary values (the solves write interiors only)
    CFDJ_HIP(hipMemcpyAsync(h->sp, h->sn, h->field() * sizeof(double), hipMemcpyDeviceToDevice,
                            h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_cavity_download(cfdj_cavity* h, double* wn, long ldw, double* sn, long lds) {
  return guard([&] {
    CFDJ_REQUIRE(h && wn && sn, "NULL argument");
    CFDJ_REQUIRE(ldw >= h->nx + 1 && lds >= h->nx + 1, "leading dimension too small");
    select_device(h->device);
    copy_out(wn, ldw, h->wn, h->P, h->nx, h->ny, h->stream);
    copy_out(sn, lds, h->sn, h->P, h->nx, h->ny, h->stream);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_cavity_step(cfdj_cavity* h, double dt, int nsteps, double* rms) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(nsteps >= 0 && std::isfinite(dt), "bad dt / nsteps");
    select_device(h->device);
    if (nsteps > h->rms_cap) {
      dfree(h->d_rms);
      h->d_rms = dalloc<double>(nsteps);
      h->rms_cap = nsteps;
    }
    h->rms_pending = 0;  // (a call that threw may have left partial sums waiting)
    for (int k = 0; k < nsteps; ++k) h->step(dt, k);
    h->flush_rms();
    if (rms && nsteps)
      CFDJ_HIP(hipMemcpyAsync(rms, h->d_rms, nsteps * sizeof(double), hipMemcpyDeviceToHost,
                              h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_cavity_rhs(cfdj_cavity* h, const double* w, long ldw, const double* s, long lds,
                    double* r, long ldr) {
  return guard([&] {
    CFDJ_REQUIRE(h && w && s && r, "NULL argument");
    CFDJ_REQUIRE(ldw >= h->nx + 1 && lds >= h->nx + 1 && ldr >= h->nx + 1, "bad ld");
    select_device(h->device);
    // the caller's psi goes to a buffer of its own: the handle's two psi buffers (and their
    // common boundary values, which cfdj_cavity_step relies on) stay as they are
    double* psi = dalloc<double>(h->field());
    try {
      copy_in(h->wa, h->P, w, ldw, h->nx, h->ny, h->stream);
      copy_in(psi, h->P, s, lds, h->nx, h->ny, h->stream);
      CFDJ_HIP(hipMemsetAsync(h->wb, 0, h->field() * sizeof(double), h->stream));
      h->stage(0, h->wa, h->wb, 0.0, psi);
      copy_out(r, ldr, h->wb, h->P, h->nx, h->ny, h->stream);
      CFDJ_HIP(hipStreamSynchronize(h->stream));
    } catch (...) {
      (void)hipStreamSynchronize(h->stream);
      dfree(psi);
      throw;
    }
    dfree(psi);
  });
}

long cfdj_cavity_mg_iterations(cfdj_cavity* h) { return h ? h->mg_iters : -1; }

void cfdj_cavity_destroy(cfdj_cavity* h) {
  if (!h) return;
  (void)guard([&] {
    select_device(h->device);
    delete h;
  });
}

int cfdj_fps_sine(int nx, int ny, double dx, double dy, const double* f, long ldf, double* s,
                  long lds) {
  cfdj_cavity* h = nullptr;
  int rc = cfdj_cavity_create(nx, ny, dx, dy, 1.0, -1, &h);
  if (rc != CFDJ_OK) return rc;
  rc = guard([&] {
    CFDJ_REQUIRE(f && s && ldf >= nx + 1 && lds >= nx + 1, "bad f / s");
    copy_in(h->wa, h->P, f, ldf, nx, ny, h->stream);
    copy_in(h->sn, h->P, s, lds, nx, ny, h->stream);
    // fps_sine(f) solves with +f: dst_poisson negates, so feed -f
    hipLaunchKernelGGL(negate_kernel, dim3((unsigned)((h->field() + 255) / 256)), dim3(256), 0,
                       h->stream, h->wa, h->wb, h->field());
    CFDJ_HIP(hipGetLastError());
    h->dst_poisson(h->wb, h->sn);
    copy_out(s, lds, h->sn, h->P, nx, ny, h->stream);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
  cfdj_cavity_destroy(h);
  return rc;
}

// ---- multigrid -----------------------------------------------------------------------
int cfdj_mg_create(int nx, int ny, double dx, double dy, int n_level, int v1, int v2, int v3,
                   int device, cfdj_mg** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr, "out is NULL");
    *out = nullptr;
    CFDJ_REQUIRE(nx >= 2 && ny >= 2 && dx > 0 && dy > 0, "bad grid");
    CFDJ_REQUIRE(v1 >= 0 && v2 >= 0 && v3 >= 0, "bad sweep counts");
    select_device(device);
    std::unique_ptr<cfdj_mg> h(new cfdj_mg);
    CFDJ_HIP(hipGetDevice(&h->device));
    CFDJ_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->nx = nx;
    h->ny = ny;
    h->mg.keep_r0 = true;  // cfdj_mg_residual returns the residual mg_N.jl leaves in r
    h->mg.init(nx, ny, dx, dy, n_level, v1, v2, v3, h->stream);
    const size_t n = (size_t)(nx + 2) * (ny + 1);
    h->u = dalloc<double>(n);
    h->f = dalloc<double>(n);
    *out = h.release();
  });
}

int cfdj_mg_solve(cfdj_mg* h, const double* f, long ldf, double* u, long ldu, double tol,
                  int max_iter, int* iterations, double* rms_hist) {
  return guard([&] {
    CFDJ_REQUIRE(h && f && u, "NULL argument");
    CFDJ_REQUIRE(ldf >= h->nx + 1 && ldu >= h->nx + 1, "leading dimension too small");
    CFDJ_REQUIRE(tol >= 0 && max_iter >= 0, "bad tol / max_iter");
    select_device(h->device);
    copy_in(h->f, h->nx + 2, f, ldf, h->nx, h->ny, h->stream);
    copy_in(h->u, h->nx + 2, u, ldu, h->nx, h->ny, h->stream);
    std::vector<double> hist;
    const int it = h->mg.solve(h->u, h->f, tol, max_iter, &hist);
    copy_out(u, ldu, h->u, h->nx + 2, h->nx, h->ny, h->stream);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    if (iterations) *iterations = it;
    if (rms_hist) std::memcpy(rms_hist, hist.data(), hist.size() * sizeof(double));
  });
}

int cfdj_mg_residual(cfdj_mg* h, double* r, long ldr) {
  return guard([&] {
    CFDJ_REQUIRE(h && r, "NULL argument");
    CFDJ_REQUIRE(ldr >= h->nx + 1, "leading dimension too small");
    select_device(h->device);
    copy_out(r, ldr, h->mg.r[0], h->nx + 2, h->nx, h->ny, h->stream);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_jacobi_solve(int nx, int ny, double dx, double dy, const double* f, long ldf,
                      double* u, long ldu, long max_iter, double tol, long freq,
                      long* iterations, double* rms_out) {
  return guard([&] {
    CFDJ_REQUIRE(f && u && ldf >= nx + 1 && ldu >= nx + 1, "bad f / u");
    CFDJ_REQUIRE(nx >= 2 && ny >= 2 && dx > 0 && dy > 0 && freq >= 1 && max_iter >= 0,
                 "bad arguments");
    hipStream_t st = nullptr;
    CFDJ_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int P = nx + 2;
    const size_t n = (size_t)P * (ny + 1);
    double *df = nullptr, *ua = nullptr, *ub = nullptr, *r = nullptr, *part = nullptr,
           *d_rms = nullptr;
    struct Free {
      std::vector<double**> ps;
      hipStream_t st;
      ~Free() {
        for (auto p : ps) dfree(*p);
        if (st) (void)hipStreamDestroy(st);
      }
    } fr{{&df, &ua, &ub, &r, &part, &d_rms}, st};
    df = dalloc<double>(n);
    ua = dalloc<double>(n);
    ub = dalloc<double>(n);
    r = dalloc<double>(n);
    part = dalloc<double>(512);
    d_rms = dalloc<double>(1);
    CFDJ_HIP(hipMemsetAsync(r, 0, n * sizeof(double), st));
    copy_in(df, P, f, ldf, nx, ny, st);
    copy_in(ua, P, u, ldu, nx, ny, st);
    CFDJ_HIP(hipMemcpyAsync(ub, ua, n * sizeof(double), hipMemcpyDeviceToDevice, st));
    const double dx2 = dx * dx, dy2 = dy * dy, dd = -2.0 / dx2 - 2.0 / dy2;
    auto rms_now = [&](const double* uu) {  // compute_residual + compute_l2norm
      hipLaunchKernelGGL(residual_kernel, interior_grid(nx, ny), dim3(kBX, kBY), 0, st, df, uu,
                         r, nx, ny, P, dx2, dy2);
      launch_rms(r, nullptr, 1, nx - 1, 1, ny - 1, P, (double)(nx - 1) * (ny - 1), part, 512,
                 d_rms, st);
      double h = 0.0;
      CFDJ_HIP(hipMemcpyAsync(&h, d_rms, sizeof(double), hipMemcpyDeviceToHost, st));
      CFDJ_HIP(hipStreamSynchronize(st));
      return h;
    };
    const double init_rms = rms_now(ua);
    double rms = init_rms;
    long it = 0;
    double* cur = ua;
    double* nxt = ub;
    while (it < 5 * max_iter) {  // gauss_seidel.jl:19
      ++it;
      hipLaunchKernelGGL(jacobi_kernel, interior_grid(nx, ny), dim3(kBX, kBY), 0, st, df, cur,
                         nxt, r, nx, ny, P, dx2, dy2, dd);
      std::swap(cur, nxt);
      if (it % freq == 0) {
        rms = rms_now(cur);
        if (rms / init_rms <= tol) break;
      }
    }
    CFDJ_HIP(hipGetLastError());
    copy_out(u, ldu, cur, P, nx, ny, st);
    CFDJ_HIP(hipStreamSynchronize(st));
    if (iterations) *iterations = it;
    if (rms_out) *rms_out = rms;
  });
}

void cfdj_mg_destroy(cfdj_mg* h) {
  if (!h) return;
  (void)guard([&] {
    select_device(h->device);
    delete h;
  });
}

}  // extern "C"
