// gfx950 kernels of the periodic vortex-merger step.
//
//  * vm_stage_kernel  -- fused Arakawa Jacobian + 5-point Laplacian (Common.jl:148-181)
//                        + SSP-RK3 stage update (vm.jl:28, 43-47, 62-66).
//  * divide_kernel    -- FD-symbol spectral divide of the FFT Poisson solve
//                        (Common.jl:115-121).
//  * pack / unpack    -- half-spectrum transposition blocks of the y-slab FFT.
//
// Built with -ffp-contract=off: every expression is evaluated in the order the reference
// writes it (no FMA contraction), so given the same streamfunction the stencil output is
// bit-identical to the CPU oracle (oracle/vm_oracle.py: arakawa_rhs, rk3_step).
#include <cstdlib>

#include "colsum.hpp"
#include "stencil.hpp"

namespace cfdj {

namespace {

#ifndef CFDJ_STAGE_WPB
#define CFDJ_STAGE_WPB 4  // wavefronts per stage-kernel workgroup
#endif
#ifndef CFDJ_STAGE_WAVES_X
#define CFDJ_STAGE_WAVES_X 0
#endif
constexpr int kWavesPerBlock = CFDJ_STAGE_WPB;
constexpr int kColsPerWave = 2 * kWave;  // two x-adjacent points per lane (16-B loads)

__device__ __forceinline__ const double* row_ptr(const double* a, const double* lo,
                                                 const double* hi, int y, int ny, int nx) {
  return y < 0 ? lo : (y >= ny ? hi : a + (size_t)y * nx);
}

// One wavefront owns 128 consecutive x (two per lane, 16-B loads) and marches
// `rows_per_wave` rows in y with a 3-row register window of omega and psi; x-neighbours
// come from lane shuffles, the two wave-edge values from one masked load each.  Four
// independent wavefronts per 256-thread workgroup take four consecutive row chunks.
template <int STAGE, bool NT>
__global__ __launch_bounds__(64 * CFDJ_STAGE_WPB) void vm_stage_kernel(const StageParams p) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nx = p.nx, ny = p.ny;
  // 1-D grid, XCD-aware: each XCD sweeps a contiguous band of (strip, chunk) tiles, strips
  // fastest, so x-neighbour strips and adjacent row chunks share one L2.
  const int strips = (nx + kColsPerWave - 1) / kColsPerWave;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
#if CFDJ_STAGE_WAVES_X
  // (variant: the workgroup's wavefronts side by side in x on the same rows)
  const int sg = strips / kWavesPerBlock;
  const int strip = (tile % sg) * kWavesPerBlock + wave, chunk = tile / sg;
#else
  const int strip = tile % strips, chunk = tile / strips;
#endif
  const int x = strip * kColsPerWave + 2 * lane;
  const bool valid = x < nx;
  const int xs = valid ? x : 0;
  const bool is_l = lane == 0;
  const bool is_r = (lane == kWave - 1) || (xs + 2 >= nx);
  const int xl = xs == 0 ? nx - 1 : xs - 1;
  const int xr = xs + 2 >= nx ? xs + 2 - nx : xs + 2;

  // A wavefront takes the part of ONE block of rows_per_wave rows (blocks are absolute: block
  // b = rows [b rpw, (b+1) rpw)) that lies in a window of the launch: the blocks the first
  // window touches, then those of the second.
#if CFDJ_STAGE_WAVES_X
  const int wi = chunk;
#else
  const int wi = chunk * kWavesPerBlock + wave;
#endif
  const int rpw = p.rows_per_wave;
  int blk, wy0, wy1;
  if (wi < p.nblk_a) {
    blk = p.y0 / rpw + wi;
    wy0 = p.y0;
    wy1 = p.y0 + p.ycount;
  } else if (wi < p.nblk_a + p.nblk_b) {
    blk = p.y0b / rpw + (wi - p.nblk_a);
    wy0 = p.y0b;
    wy1 = p.y0b + p.ycount_b;
  } else {
    return;
  }
  const int ybeg = max(wy0, blk * rpw);
  const int yend = min(wy1, (blk + 1) * rpw);

  const StageCoef k = p.k;
  Raw wr_p = fetch(row_ptr(p.w, p.w_lo, p.w_hi, ybeg + 1, ny, nx), xs, xl, xr, is_l, is_r);
  Raw sr_p = fetch(row_ptr(p.s, p.s_lo, p.s_hi, ybeg + 1, ny, nx), xs, xl, xr, is_l, is_r);
  Win wm = expand(fetch(row_ptr(p.w, p.w_lo, p.w_hi, ybeg - 1, ny, nx), xs, xl, xr, is_l, is_r), is_l, is_r);
  Win sm = expand(fetch(row_ptr(p.s, p.s_lo, p.s_hi, ybeg - 1, ny, nx), xs, xl, xr, is_l, is_r), is_l, is_r);
  Win wc = expand(fetch(row_ptr(p.w, p.w_lo, p.w_hi, ybeg, ny, nx), xs, xl, xr, is_l, is_r), is_l, is_r);
  Win sc = expand(fetch(row_ptr(p.s, p.s_lo, p.s_hi, ybeg, ny, nx), xs, xl, xr, is_l, is_r), is_l, is_r);

  // Column sums of `out` over the block (colpart).  Their order is fixed so that a slab
  // computed in one launch and one computed as interior rows + the first and the last row
  // (the rows that read the halo rows) agree to the bit: row 0 of the slab is added LAST to
  // its block's sum, every other row in increasing order.
  double2 csum = make_double2(0.0, 0.0), held = csum;
  const bool hold = p.colpart != nullptr && ybeg == 0 && yend > 1;
  for (int y = ybeg; y < yend; ++y) {
    // prefetch row y+2 (clamped: the last iteration re-reads row yend, harmlessly)
    const int yn = min(y + 2, yend);
    const Raw wr_n = fetch(row_ptr(p.w, p.w_lo, p.w_hi, yn, ny, nx), xs, xl, xr, is_l, is_r);
    const Raw sr_n = fetch(row_ptr(p.s, p.s_lo, p.s_hi, yn, ny, nx), xs, xl, xr, is_l, is_r);
    double2 wnv = make_double2(0.0, 0.0);
    if constexpr (STAGE >= 2)
      wnv = load_stream<NT>(reinterpret_cast<const double2*>(p.wn + (size_t)y * nx + xs));

    const Win wp = expand(wr_p, is_l, is_r);
    const Win sp = expand(sr_p, is_l, is_r);

    double r0, r1;
    pair_rhs(wm, wc, wp, sm, sc, sp, k, r0, r1);
    double2 o;
    o.x = stage_update<STAGE>(r0, wc.a, wnv.x, k);
    o.y = stage_update<STAGE>(r1, wc.b, wnv.y, k);
    // (streamed on large slabs: 1.3 % of the y-slab step; in the row-group kernel the same
    // brought nothing beyond what the streaming store of psi already gives)
    if (valid) store_stream<NT>(reinterpret_cast<double2*>(p.out + (size_t)y * nx + xs), o);
    if (hold && y == 0) {
      held = o;
    } else {
      csum.x += o.x;
      csum.y += o.y;
    }

    wm = wc;
    wc = wp;
    sm = sc;
    sc = sp;
    wr_p = wr_n;
    sr_p = sr_n;
  }
  if (p.colpart != nullptr && valid) {
    double2* cp = reinterpret_cast<double2*>(p.colpart + (size_t)blk * nx + xs);
    if (hold) {
      csum.x += held.x;
      csum.y += held.y;
    }
    if (p.cp_accumulate) {  // the rest of the block came from an earlier launch
      const double2 prev = *cp;
      csum.x = prev.x + csum.x;
      csum.y = prev.y + csum.y;
    }
    *cp = csum;
  }
}

// Row-group variant of the stage kernel: a 256-thread workgroup owns 512 consecutive x of
// kTileRows consecutive rows (two x per lane, every row of the group and its two halo rows
// loaded at once, 16 B per lane), instead of a wavefront marching down 32 rows.  Workgroups
// run in row-major order, so at any moment the chip works on one narrow band of rows: the
// three or four streams (omega_s, psi, omega^n, output) advance through HBM sequentially,
// which the memory system serves 14-18 % faster than the marching kernels' 128 scattered
// row fronts (6.1 against 5.0-5.3 TB/s for the bare access shapes, tools/micro/streambench).
// The halo rows a group shares with its neighbours are re-read through L2: the group above
// and below are workgroups b -/+ nx/512, which land on the same XCD for nx = 4096.
// x-neighbours: lane shuffles; across wavefronts of the workgroup through LDS; at the
// workgroup's two edges one masked load per row and field.  Same arithmetic (stencil.hpp).
#ifndef CFDJ_TILE_ROWS
#define CFDJ_TILE_ROWS 2
#endif
#ifndef CFDJ_TILE_WAVES
#define CFDJ_TILE_WAVES 0  // > 0: occupancy target in wavefronts per SIMD (register cap)
#endif
#if CFDJ_TILE_WAVES > 0
#define CFDJ_TILE_ATTR __attribute__((amdgpu_waves_per_eu(CFDJ_TILE_WAVES, CFDJ_TILE_WAVES)))
#else
#define CFDJ_TILE_ATTR
#endif
constexpr int kTileRows = CFDJ_TILE_ROWS;
constexpr int kTileCols = 512;
constexpr int kXcds = 8;  // MI355X: workgroup b is dispatched to XCD b % 8

template <int STAGE, bool NT>
__global__ __launch_bounds__(256) CFDJ_TILE_ATTR void vm_stage_tile_kernel(const StageParams p) {
  constexpr int G = kTileRows, NR = G + 2, NW = 256 / kWave;
  // left[w]: the value left of wavefront w's first x (w = 0: the workgroup's halo column);
  // right[w]: the value right of its last x (w = NW - 1: the halo column); per row and field
  __shared__ double left[NW][2 * NR], right[NW][2 * NR];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nx = p.nx, ny = p.ny;
  const int strips = nx / kTileCols;
  // Workgroup b runs on XCD b % 8.  A row group shares its halo rows with the groups above
  // and below, so those should sit on the same XCD (one L2): automatic when the strip count
  // is a multiple of 8; for 1, 2 or 4 strips the rows are split into 8 / strips bands and
  // XCD (strip, band) walks its band.
  int strip = blockIdx.x % strips, grp = blockIdx.x / strips;
  if (strips < kXcds && kXcds % strips == 0) {
    const int bands = kXcds / strips, ngrp = p.ycount / G;
    if (ngrp % bands == 0) {
      const int xcd = blockIdx.x % kXcds, i = blockIdx.x / kXcds;
      strip = xcd % strips;
      grp = (xcd / strips) * (ngrp / bands) + i;
    }
  }
  const int x0 = strip * kTileCols;
  const int x = x0 + 2 * (int)threadIdx.x;
  const int y0 = p.y0 + grp * G;

  double2 wv[NR], sv[NR], wnv[G];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const double* wr = row_ptr(p.w, p.w_lo, p.w_hi, y0 - 1 + j, ny, nx);
    const double* sr = row_ptr(p.s, p.s_lo, p.s_hi, y0 - 1 + j, ny, nx);
    wv[j] = *reinterpret_cast<const double2*>(wr + x);
    sv[j] = *reinterpret_cast<const double2*>(sr + x);
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    wnv[j] = make_double2(0.0, 0.0);
    if constexpr (STAGE >= 2)
      wnv[j] = load_stream<NT>(reinterpret_cast<const double2*>(p.wn + (size_t)(y0 + j) * nx + x));
  }
  // The two halo columns of the workgroup (periodic in x): one load in the first
  // wavefront, lane i < 4 NR fetching (side, row, field) = (i / 2NR, (i % 2NR) / 2, i % 2).
  static_assert(4 * NR <= kWave, "halo fetch needs one lane per value");
  double halo = 0.0;
  if (threadIdx.x < 4 * NR) {
    const int side = threadIdx.x / (2 * NR), rem = threadIdx.x % (2 * NR);
    const int xh = side == 0 ? (x0 == 0 ? nx - 1 : x0 - 1)
                             : (x0 + kTileCols >= nx ? x0 + kTileCols - nx : x0 + kTileCols);
    const double* r = (rem & 1) ? row_ptr(p.s, p.s_lo, p.s_hi, y0 - 1 + rem / 2, ny, nx)
                                : row_ptr(p.w, p.w_lo, p.w_hi, y0 - 1 + rem / 2, ny, nx);
    halo = r[xh];
  }
  // Edge lanes publish one value per row and field: lane 0 its first x as the right
  // neighbour of the wavefront before it, lane 63 its last x as the left neighbour of the
  // wavefront after it.
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
  const StageCoef k = p.k;
  Win ww[NR], sw[NR];
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
    double r0, r1;
    pair_rhs(ww[j], ww[j + 1], ww[j + 2], sw[j], sw[j + 1], sw[j + 2], k, r0, r1);
    double2 o;
    o.x = stage_update<STAGE>(r0, ww[j + 1].a, wnv[j].x, k);
    o.y = stage_update<STAGE>(r1, ww[j + 1].b, wnv[j].y, k);
    *reinterpret_cast<double2*>(p.out + (size_t)(y0 + j) * nx + x) = o;
  }
}

// Tall-tile variant, for the y-slabs of the substructured Poisson path: the row-group
// kernel's access shape (workgroups in row-major order, so the chip works on one narrow band
// of rows) that also delivers the slab's column sums.  A 256-thread workgroup owns 128
// consecutive x of 16 consecutive rows, wavefront w the rows 4w .. 4w + 3 (two x per lane;
// the wave's rows and their two halo rows loaded at once, the wave's two halo columns by one
// load of lane i < 24 = (side, row, field) and shuffles).  The sixteen output rows meet in
// LDS, where the first wavefront adds them up in the marching kernel's order (increasing, the
// slab's row 0 last): the same partial sums bit for bit, one per 16-row block.
#ifndef CFDJ_TALL_G
#define CFDJ_TALL_G 4
#endif
constexpr int kTallG = CFDJ_TALL_G;        // rows per wavefront
constexpr int kTallRows = 16;              // rows per workgroup = rows per column-sum block
constexpr int kTallW = kTallRows / kTallG;  // wavefronts per workgroup
#ifdef CFDJ_TALL_WAVES
#define CFDJ_TALL_ATTR __attribute__((amdgpu_waves_per_eu(CFDJ_TALL_WAVES, CFDJ_TALL_WAVES)))
#else
#define CFDJ_TALL_ATTR
#endif
template <int STAGE, bool NT>
__global__ __launch_bounds__(64 * kTallW) CFDJ_TALL_ATTR void vm_stage_tall_kernel(const StageParams p) {
  constexpr int G = kTallG, NR = G + 2;
  __shared__ double2 outs[kTallRows][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nx = p.nx, ny = p.ny;
  const int strips = nx / kColsPerWave;
  // workgroup b runs on XCD b % 8 = strip % 8: the blocks above and below share its L2
  const int strip = blockIdx.x % strips, grp = blockIdx.x / strips;
  const int x0 = strip * kColsPerWave;
  const int x = x0 + 2 * lane;
  const int yb = p.y0 + grp * kTallRows;
  const int y0 = yb + wave * G;

  double2 wv[NR], sv[NR], wnv[G];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const double* wr = row_ptr(p.w, p.w_lo, p.w_hi, y0 - 1 + j, ny, nx);
    const double* sr = row_ptr(p.s, p.s_lo, p.s_hi, y0 - 1 + j, ny, nx);
    wv[j] = *reinterpret_cast<const double2*>(wr + x);
    sv[j] = *reinterpret_cast<const double2*>(sr + x);
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    wnv[j] = make_double2(0.0, 0.0);
    if constexpr (STAGE >= 2)
      wnv[j] = load_stream<NT>(reinterpret_cast<const double2*>(p.wn + (size_t)(y0 + j) * nx + x));
  }
  static_assert(4 * NR <= kWave, "halo fetch needs one lane per value");
  double halo = 0.0;
  if (lane < 4 * NR) {
    const int side = lane / (2 * NR), rem = lane % (2 * NR);
    const int xh = side == 0 ? (x0 == 0 ? nx - 1 : x0 - 1)
                             : (x0 + kColsPerWave >= nx ? x0 + kColsPerWave - nx
                                                        : x0 + kColsPerWave);
    const double* r = (rem & 1) ? row_ptr(p.s, p.s_lo, p.s_hi, y0 - 1 + rem / 2, ny, nx)
                                : row_ptr(p.w, p.w_lo, p.w_hi, y0 - 1 + rem / 2, ny, nx);
    halo = r[xh];
  }
  const StageCoef k = p.k;
  // a row's window (its two x-neighbours from the neighbouring lanes, the wave's edge columns
  // from the halo load), formed when the row first enters a stencil: three windows per field
  // are live, not NR
  auto window = [&](const double2& c, int jh, int field) {
    Win w;
    w.a = c.x;
    w.b = c.y;
    w.l = __shfl_up(c.y, 1, kWave);
    w.r = __shfl_down(c.x, 1, kWave);
    const double hl = __shfl(halo, 2 * jh + field, kWave);
    const double hr = __shfl(halo, 2 * NR + 2 * jh + field, kWave);
    if (lane == 0) w.l = hl;
    if (lane == kWave - 1) w.r = hr;
    return w;
  };
  Win wm = window(wv[0], 0, 0), sm = window(sv[0], 0, 1);
  Win wc = window(wv[1], 1, 0), sc = window(sv[1], 1, 1);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const Win wp = window(wv[j + 2], j + 2, 0), sp = window(sv[j + 2], j + 2, 1);
    double r0, r1;
    pair_rhs(wm, wc, wp, sm, sc, sp, k, r0, r1);
    double2 o;
    o.x = stage_update<STAGE>(r0, wc.a, wnv[j].x, k);
    o.y = stage_update<STAGE>(r1, wc.b, wnv[j].y, k);
#ifdef CFDJ_TALL_PLAIN_STORE
    *reinterpret_cast<double2*>(p.out + (size_t)(y0 + j) * nx + x) = o;
#else
    store_stream<NT>(reinterpret_cast<double2*>(p.out + (size_t)(y0 + j) * nx + x), o);
#endif
    outs[wave * G + j][lane] = o;
    wm = wc;
    sm = sc;
    wc = wp;
    sc = sp;
  }
  __syncthreads();
  if (wave == 0) {
    const bool hold = yb == 0;  // the slab's row 0 is added last
    double2 c = make_double2(0.0, 0.0);
#pragma unroll
    for (int r = 0; r < kTallRows; ++r) {
      if (r == 0 && hold) continue;
      const double2 o = outs[r][lane];
      c.x += o.x;
      c.y += o.y;
    }
    if (hold) {
      const double2 o = outs[0][lane];
      c.x += o.x;
      c.y += o.y;
    }
    *reinterpret_cast<double2*>(p.colpart + (size_t)(yb / kTallRows) * nx + x) = c;
  }
}

// colpart[b][x] = sum over rows [b rpw, (b+1) rpw) of f[y][x], in the row order of the
// stage kernel's csum (increasing, row 0 last), so a field gets the same partials either way.
__global__ __launch_bounds__(256) void colpart_kernel(const double* __restrict__ f, int nx,
                                                      int rows, int rpw,
                                                      double* __restrict__ colpart) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (x >= nx) return;
  double s = 0.0;
  const int y1 = min((b + 1) * rpw, rows);
  for (int y = max(b * rpw, 1); y < y1; ++y) s += f[(size_t)y * nx + x];
  if (b == 0) s += f[x];  // row 0 last (the stage kernel's order)
  colpart[(size_t)b * nx + x] = s;
}

// out8[0][x] = sum of the nb partial rows; 64 columns per workgroup, the 4 waves sum every
// 4th block, then add up in a fixed order; rows 1..7 of out8 zeroed.
__global__ __launch_bounds__(256) void colsum_row_kernel(const double* __restrict__ colpart,
                                                         int nb, int nx,
                                                         double* __restrict__ out8) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = blockIdx.x * 64 + lane;
  const double t = colsum_block(colpart, nb, nx, blockIdx.x * 64, part);
  if (x >= nx) return;
  if (w == 0) out8[x] = t;
  else out8[(size_t)w * nx + x] = 0.0;
  out8[(size_t)(w + 4) * nx + x] = 0.0;
}

__global__ __launch_bounds__(256) void divide_kernel(const DivideParams p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (i >= p.width) return;
  const int kx = p.kx_off + i;
  double2* ptr = p.spec + (size_t)j * p.pitch + i;
  double2 o = make_double2(0.0, 0.0);
  if (kx < p.nxh && !(kx == 0 && j == 0)) {  // e[1,1] = 0 (Common.jl:118); padding -> 0
    double2 v = *ptr;
    if (p.neg) {
      v.x = -v.x;
      v.y = -v.y;
    }
    const double ax = p.aa + p.bb * p.cx[kx];
    const double d = ax + p.cc * p.cy[j];
    if (p.recip) {  // iden = 1/d precomputed by the reference, then e * iden
      const double id = 1.0 / d;
      o.x = (v.x * id) * p.scale;
      o.y = (v.y * id) * p.scale;
    } else if (p.cy_mirror == nullptr) {
      o.x = (v.x / d) * p.scale;  // Julia Complex/Real: componentwise division
      o.y = (v.y / d) * p.scale;
    } else {
      const double d2 = ax + p.cc * p.cy_mirror[j];
      o.x = (0.5 * (v.x / d + v.x / d2)) * p.scale;
      o.y = (0.5 * (v.y / d + v.y / d2)) * p.scale;
    }
  }
  *ptr = o;
}

__global__ __launch_bounds__(256) void pack_kernel(const double2* __restrict__ X,
                                                   double2* __restrict__ S, int nxh,
                                                   int rows, int kb) {
  const int kl = blockIdx.x * blockDim.x + threadIdx.x;
  const int jl = blockIdx.y;
  const int q = blockIdx.z;
  if (kl >= kb) return;
  const int kx = q * kb + kl;
  S[((size_t)q * rows + jl) * kb + kl] =
      kx < nxh ? X[(size_t)jl * nxh + kx] : make_double2(0.0, 0.0);
}

__global__ __launch_bounds__(256) void unpack_kernel(const double2* __restrict__ S,
                                                     double2* __restrict__ X, int nxh,
                                                     int rows, int kb) {
  const int kl = blockIdx.x * blockDim.x + threadIdx.x;
  const int jl = blockIdx.y;
  const int q = blockIdx.z;
  const int kx = q * kb + kl;
  if (kl >= kb || kx >= nxh) return;
  X[(size_t)jl * nxh + kx] = S[((size_t)q * rows + jl) * kb + kl];
}

__global__ __launch_bounds__(256) void finite_kernel(const double* __restrict__ a, size_t n,
                                                     int* flag) {
  bool bad = false;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    bad |= !isfinite(a[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

}  // namespace

// The row-group kernel where it applies: row length a multiple of 512, a row count that
// is a multiple of the group, no column partial sums, and the caller has not asked for the
// marching kernel.
static bool stage_tile_ok(const StageParams& p) {
  return !p.march && p.colpart == nullptr && p.nx % kTileCols == 0 &&
         p.ycount % kTileRows == 0 && p.ycount > 0 && p.ycount_b == 0;
}

bool stage_runs_row_group(const StageParams& p) { return stage_tile_ok(p); }

// The tall-tile kernel where it applies: column partial sums wanted for whole 16-row blocks
// in one launch (one window, nothing to add to), rows a multiple of 128.
// CFDJ_STAGE_TALL=0: the marching kernel instead.
static bool stage_tall_ok(const StageParams& p) {
  static const bool on = [] {
    const char* e = std::getenv("CFDJ_STAGE_TALL");
    return !(e && e[0] == '0');
  }();
  return on && !p.march && p.colpart != nullptr && !p.cp_accumulate &&
         p.rows_per_wave == kTallRows && p.nx % kColsPerWave == 0 && p.nx >= 8 * kColsPerWave &&
         p.y0 % kTallRows == 0 && p.ycount % kTallRows == 0 && p.ycount > 0 && p.ycount_b == 0;
}

void launch_stage(int stage, const StageParams& p, hipStream_t st) {
  if (p.ycount <= 0 || p.y0 < 0 || p.y0 + p.ycount > p.ny)
    throw Error{CFDJ_ERR_ARG, "stage kernel: bad row window"};
  if (p.ycount_b != 0 &&
      (p.ycount_b < 0 || p.y0b < p.y0 + p.ycount || p.y0b + p.ycount_b > p.ny))
    throw Error{CFDJ_ERR_ARG, "stage kernel: bad second row window"};
  if (stage_tile_ok(p)) {
    const long blocks = (long)(p.nx / kTileCols) * (p.ycount / kTileRows);
    if (blocks > 0x7fffffffL) throw Error{CFDJ_ERR_ARG, "grid too large"};
    const dim3 grid((unsigned)blocks), block(256);
    switch (stage) {
      // stages 0 and 1 read no omega^n: one instantiation
      case 0: hipLaunchKernelGGL((vm_stage_tile_kernel<0, false>), grid, block, 0, st, p); break;
      case 1: hipLaunchKernelGGL((vm_stage_tile_kernel<1, false>), grid, block, 0, st, p); break;
      case 2:
        if (p.stream) hipLaunchKernelGGL((vm_stage_tile_kernel<2, true>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((vm_stage_tile_kernel<2, false>), grid, block, 0, st, p);
        break;
      default:
        if (p.stream) hipLaunchKernelGGL((vm_stage_tile_kernel<3, true>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((vm_stage_tile_kernel<3, false>), grid, block, 0, st, p);
        break;
    }
    CFDJ_HIP(hipGetLastError());
    return;
  }
  if (stage_tall_ok(p)) {
    const long blocks = (long)(p.nx / kColsPerWave) * (p.ycount / kTallRows);
    if (blocks > 0x7fffffffL) throw Error{CFDJ_ERR_ARG, "grid too large"};
    const dim3 grid((unsigned)blocks), block(64 * kTallW);
    switch (stage) {
      case 0: hipLaunchKernelGGL((vm_stage_tall_kernel<0, false>), grid, block, 0, st, p); break;
      case 1:
        if (p.stream) hipLaunchKernelGGL((vm_stage_tall_kernel<1, true>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((vm_stage_tall_kernel<1, false>), grid, block, 0, st, p);
        break;
      case 2:
        if (p.stream) hipLaunchKernelGGL((vm_stage_tall_kernel<2, true>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((vm_stage_tall_kernel<2, false>), grid, block, 0, st, p);
        break;
      default:
        if (p.stream) hipLaunchKernelGGL((vm_stage_tall_kernel<3, true>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((vm_stage_tall_kernel<3, false>), grid, block, 0, st, p);
        break;
    }
    CFDJ_HIP(hipGetLastError());
    return;
  }
  const int rpw = p.rows_per_wave;
  if (rpw < 1) throw Error{CFDJ_ERR_ARG, "stage kernel: rows per wavefront must be >= 1"};
  const long strips = (p.nx + kColsPerWave - 1) / kColsPerWave;
  // blocks of rpw rows (absolute) that each window touches: one wavefront per block and strip
  StageParams q = p;
  q.nblk_a = (p.y0 + p.ycount - 1) / rpw - p.y0 / rpw + 1;
  q.nblk_b = p.ycount_b > 0 ? (p.y0b + p.ycount_b - 1) / rpw - p.y0b / rpw + 1 : 0;
#if CFDJ_STAGE_WAVES_X
  if (strips % kWavesPerBlock != 0) throw Error{CFDJ_ERR_ARG, "stage kernel: nx % 512 != 0"};
  const long chunks = q.nblk_a + q.nblk_b;
  dim3 grid((unsigned)(strips / kWavesPerBlock * chunks));
#else
  const long chunks = (q.nblk_a + q.nblk_b + kWavesPerBlock - 1) / kWavesPerBlock;
  if (strips * chunks > 0x7fffffffL) throw Error{CFDJ_ERR_ARG, "grid too large"};
  dim3 grid((unsigned)(strips * chunks));
#endif
  dim3 block(kWave * kWavesPerBlock);
  switch (stage) {
    case 0: hipLaunchKernelGGL((vm_stage_kernel<0, false>), grid, block, 0, st, q); break;
    case 1:
      if (p.stream) hipLaunchKernelGGL((vm_stage_kernel<1, true>), grid, block, 0, st, q);
      else hipLaunchKernelGGL((vm_stage_kernel<1, false>), grid, block, 0, st, q);
      break;
    case 2:
      if (p.stream) hipLaunchKernelGGL((vm_stage_kernel<2, true>), grid, block, 0, st, q);
      else hipLaunchKernelGGL((vm_stage_kernel<2, false>), grid, block, 0, st, q);
      break;
    default:
      if (p.stream) hipLaunchKernelGGL((vm_stage_kernel<3, true>), grid, block, 0, st, q);
      else hipLaunchKernelGGL((vm_stage_kernel<3, false>), grid, block, 0, st, q);
      break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_colpart(const double* f, int nx, int rows, int rpw, double* colpart,
                    hipStream_t st) {
  const dim3 grid((nx + 255) / 256, (rows + rpw - 1) / rpw);
  hipLaunchKernelGGL(colpart_kernel, grid, dim3(256), 0, st, f, nx, rows, rpw, colpart);
  CFDJ_HIP(hipGetLastError());
}

void launch_colsum_row(const double* colpart, int nb, int nx, double* out8, hipStream_t st) {
  hipLaunchKernelGGL(colsum_row_kernel, dim3((nx + 63) / 64), dim3(256), 0, st, colpart, nb,
                     nx, out8);
  CFDJ_HIP(hipGetLastError());
}

// dst[i ds] = src[i ss], i < n (complex elements): column 0 of a tiled spectrum <-> a
// contiguous column.
__global__ __launch_bounds__(256) void strided_copy_kernel(double2* __restrict__ dst, int ds,
                                                           const double2* __restrict__ src,
                                                           int ss, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[(size_t)i * ds] = src[(size_t)i * ss];
}

void launch_strided_copy(double2* dst, int ds, const double2* src, int ss, int n,
                         hipStream_t st) {
  hipLaunchKernelGGL(strided_copy_kernel, dim3((n + 255) / 256), dim3(256), 0, st, dst, ds, src,
                     ss, n);
  CFDJ_HIP(hipGetLastError());
}

void launch_divide(const DivideParams& p, hipStream_t st) {
  dim3 grid((p.width + 255) / 256, p.rows);
  hipLaunchKernelGGL(divide_kernel, grid, dim3(256), 0, st, p);
  CFDJ_HIP(hipGetLastError());
}

void launch_pack(const double2* X, double2* S, int nxh, int rows, int kb, int nranks,
                 hipStream_t st) {
  dim3 grid((kb + 255) / 256, rows, nranks);
  hipLaunchKernelGGL(pack_kernel, grid, dim3(256), 0, st, X, S, nxh, rows, kb);
  CFDJ_HIP(hipGetLastError());
}

void launch_unpack(const double2* S, double2* X, int nxh, int rows, int kb, int nranks,
                   hipStream_t st) {
  dim3 grid((kb + 255) / 256, rows, nranks);
  hipLaunchKernelGGL(unpack_kernel, grid, dim3(256), 0, st, S, X, nxh, rows, kb);
  CFDJ_HIP(hipGetLastError());
}

void launch_check_finite(const double* a, size_t n, int* flag, hipStream_t st) {
  size_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(finite_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, n, flag);
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
