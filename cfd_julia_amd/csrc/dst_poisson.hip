// DST-I Poisson solve of the lid-driven cavity (lid_driven_cavity.jl:11-21 `fps_sine`) on
// gfx950, on the cavity's own (nx-1) x (ny-1) interior -- three passes over 8 B per cell each
// way, no 2nx x 2ny extension grid in HBM:
//
//   rows_fwd : FFTW's RODFT00 of a row, S[k] = 2 sum_i x_i sin(pi i k / nx), is -Im of the
//              length-2nx DFT of the row's odd extension.  Two rows a, b ride one complex
//              transform z = ext(a) + i ext(b): Re Z[k] = S_b[k], -Im Z[k] = S_a[k].  The
//              extension is built in registers from the nx-1 loaded values; the 2nx-point
//              Stockham FFT runs in LDS; the coefficients go out as pairs of x-modes,
//              T[kappa][j] = (S_{2 kappa}[j], S_{2 kappa + 1}[j]), column-major (y
//              contiguous), so a workgroup's 4 (or more) rows make whole 64-B segments.
//   cols     : one workgroup per mode pair: its column is a contiguous double2 array whose
//              two components are two real columns -- again one packed odd-extension
//              transform (length 2ny), the multiplication by the reference's iden table
//              (lid_driven_cavity.jl:17,64-69; evaluated as tx[k] + ty[l], reciprocal, as
//              the periodic path's Dirichlet symbol), and the second DST-I (the same packed
//              transform: the spectrum of an odd sequence is odd, so the register contents
//              are already the extended input), 1 / ((2nx)(2ny)) folded in.  In place.
//   rows_inv : the second x-DST of each row pair from T, real rows out (interior only).
//
// The second half of this file holds the same three passes on a half-length transform (an
// n-point FFT per row pair, the odd coefficients as a running sum), which dst_half_passes()
// selects per pass where it is the faster one.
//
// Powers of two nx, ny in 512..4096 (FFT lengths 1024..8192); other sizes use the periodic
// solver on the odd-odd extension (cavity.hip).  FMA contraction is on, as in the periodic
// FFT passes: the transform is compared with scipy's DST-I at 1e-12 relative.
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

#include <cstdlib>

namespace cfdj {

namespace {

// Longest transform the small-item (non-persistent) row kernels take.
#ifndef CFDJ_DST_NP_MAXM2
#define CFDJ_DST_NP_MAXM2 8192
#endif

// Row passes: RP row pairs (2 RP rows) per work item, one packed FFT of length M2 each.
template <int M2>
struct DstRowCfg {
  static constexpr int T = Plan<M2>::T;
  static constexpr int RP = 8192 / M2 < 1 ? 1 : 8192 / M2;  // 139 KB of LDS
  static constexpr int ROWS = 2 * RP;
  static constexpr int THREADS = RP * T;
  static constexpr int ENTRIES = (M2 / 4) * ROWS / THREADS;  // (mode pair, row) per thread
  static_assert(ENTRIES == 8, "entry mapping");
};

// Entry e of a work item: row rr of the item, mode pair kappa.  16 consecutive lanes take
// 16 consecutive mode pairs of one row; ROWS consecutive 16-lane groups take the item's
// rows, so a wave's global accesses cover whole ROWS*16-B segments per mode pair.
template <int M2>
__device__ __forceinline__ void entry_index(int e, int& rr, int& kap) {
  using C = DstRowCfg<M2>;
  rr = (e >> 4) % C::ROWS;
  kap = ((e >> 4) / C::ROWS) * 16 + (e & 15);
}

// Stage-0 registers of the packed odd extension of rows ja (real part) and ja + 1
// (imaginary part) of the node array w (pitch P); rows beyond ny - 1 count as zero; sgn
// folds the reference's f = -w.
template <int M2>
__device__ __forceinline__ void load_row_pair(double2 (&v)[16], const double* __restrict__ w,
                                              int P, int ny, int ja, int tid, double sgn) {
  constexpr int nx = M2 / 2;
  constexpr int R0 = Plan<M2>::radix(0);
  const bool oka = ja <= ny - 1, okb = ja + 1 <= ny - 1;
  const double* ra = w + (size_t)(oka ? ja : 1) * P;
  const double* rb = w + (size_t)(okb ? ja + 1 : 1) * P;
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int p = in_pos<M2, 0>(tid, b, r);
      const int i = p < nx ? p : M2 - p;          // mirrored node, 1..nx-1 (or 0 / nx)
      const bool zero = (p & (nx - 1)) == 0;      // p == 0 or p == nx
      const double s = p < nx ? sgn : -sgn;
      const int ii = zero ? 1 : i;
      const double a = ra[ii], bq = rb[ii];
      v[b * R0 + r] = make_double2(zero || !oka ? 0.0 : s * a, zero || !okb ? 0.0 : s * bq);
    }
}

template <int M2>
__global__ __launch_bounds__(DstRowCfg<M2>::THREADS) void dst_rows_fwd_kernel(
    const double* __restrict__ w, int P, int ny, double2* __restrict__ T, int JT, double sgn,
    const double2* __restrict__ tw_) {
  using PL = Plan<M2>;
  using C = DstRowCfg<M2>;
  __shared__ double2 lds[C::RP * PL::PAD];
  __shared__ TwLds<M2> tw;
  const int q = threadIdx.x / PL::T;
  const int tid = threadIdx.x % PL::T;
  double2* buf = lds + q * PL::PAD;
  const Range rg = persistent_range(blockIdx.x, gridDim.x, ny / C::ROWS);
  tw.fill(tw_);
  if (rg.count <= 0) return;
  double2 nxt[16];
  load_row_pair<M2>(nxt, w, P, ny, 1 + rg.first * C::ROWS + 2 * q, tid, sgn);
  __syncthreads();
  for (int it = 0; it < rg.count; ++it) {
    const int slot0 = (rg.first + it * rg.stride) * C::ROWS;  // row j lives in slot j - 1
    stage_regs<M2, 0, -1>(nxt, tid, tw);
    lds_write<M2, 0>(buf, nxt, tid);
    if (it + 1 < rg.count)
      load_row_pair<M2>(nxt, w, P, ny, 1 + slot0 + rg.stride * C::ROWS + 2 * q, tid, sgn);
    __syncthreads();
    double2 v[16];
    run_stages<M2, 1, -1, true>(buf, v, tid, tw);
    double2* tb = T + __builtin_amdgcn_readfirstlane(slot0);
#pragma unroll
    for (int i = 0; i < C::ENTRIES; ++i) {
      int rr, kap;
      entry_index<M2>(threadIdx.x + i * C::THREADS, rr, kap);
      const double2* bq = lds + (rr >> 1) * PL::PAD;
      const double2 Z0 = bq[padx(2 * kap)];
      const double2 Z1 = bq[padx(2 * kap + 1)];
      // first row of the pair: -Im Z; second row: Re Z
      const double2 o = (rr & 1) ? make_double2(Z0.x, Z1.x) : make_double2(-Z0.y, -Z1.y);
      tb[(unsigned)(kap * JT + rr)] = o;
    }
    __syncthreads();  // LDS is rewritten by the next item
  }
}

// sprev / part (optional): this workgroup's sum of (s_new - sprev)^2 over the nodes it
// writes goes to part[blockIdx.x] (fixed order: per-thread running sums, then a tree), the
// first pass of the step's RMS of the streamfunction change (lid_driven_cavity.jl:112-114)
// without re-reading both fields.
template <int M2>
__global__ __launch_bounds__(DstRowCfg<M2>::THREADS) void dst_rows_inv_kernel(
    const double2* __restrict__ T, int JT, double* __restrict__ s, int P, int ny,
    const double2* __restrict__ tw_, const double* __restrict__ sprev,
    double* __restrict__ part) {
  using PL = Plan<M2>;
  using C = DstRowCfg<M2>;
  constexpr int nx = M2 / 2;
  __shared__ double2 lds[C::RP * PL::PAD];
  __shared__ TwLds<M2> tw;
  const int q = threadIdx.x / PL::T;
  const int tid = threadIdx.x % PL::T;
  double2* buf = lds + q * PL::PAD;
  const Range rg = persistent_range(blockIdx.x, gridDim.x, ny / C::ROWS);
  tw.fill(tw_);
  double acc = 0.0;
  auto load_entries = [&](double2 (&e)[C::ENTRIES], int slot0) {
    const double2* tb = T + __builtin_amdgcn_readfirstlane(slot0);
    int tx = threadIdx.x;
    asm volatile("" : "+v"(tx));  // keep the 8 offsets out of loop-invariant registers
#pragma unroll
    for (int i = 0; i < C::ENTRIES; ++i) {
      int rr, kap;
      entry_index<M2>(tx + i * C::THREADS, rr, kap);
      e[i] = tb[(unsigned)(kap * JT + rr)];
    }
  };
  double2 nxt[C::ENTRIES];
  if (rg.count > 0) load_entries(nxt, rg.first * C::ROWS);
  __syncthreads();
  for (int it = 0; it < rg.count; ++it) {
    const int slot0 = (rg.first + it * rg.stride) * C::ROWS;
    // entries -> packed odd extension in LDS: row parity picks the real / imaginary part,
    // mode k goes to p = k and, negated, to p = 2nx - k; p = 0 and p = nx are zero.
#pragma unroll
    for (int i = 0; i < C::ENTRIES; ++i) {
      int rr, kap;
      entry_index<M2>(threadIdx.x + i * C::THREADS, rr, kap);
      double* bq = reinterpret_cast<double*>(lds + (rr >> 1) * PL::PAD) + (rr & 1);
      const int k0 = 2 * kap, k1 = k0 + 1;
      const double v0 = k0 == 0 ? 0.0 : nxt[i].x;  // mode 0 of a sine series does not exist
      bq[2 * padx(k0)] = v0;
      bq[2 * padx(k1)] = nxt[i].y;
      if (k0 != 0) bq[2 * padx(M2 - k0)] = -v0;
      else bq[2 * padx(nx)] = 0.0;  // the kappa = 0 lanes also clear p = nx
      bq[2 * padx(M2 - k1)] = -nxt[i].y;
    }
    if (it + 1 < rg.count) load_entries(nxt, slot0 + rg.stride * C::ROWS);
    __syncthreads();
    double2 v[16];
    run_stages<M2, 0, -1, false>(buf, v, tid, tw);
    constexpr int SL = PL::NSTAGES - 1;
    constexpr int RL = PL::radix(SL);
    const int ja = 1 + slot0 + 2 * q;
    const bool oka = ja <= ny - 1, okb = ja + 1 <= ny - 1;
    double* sa = s + (size_t)ja * P;
    double* sb = sa + P;
#pragma unroll
    for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
      for (int r = 0; r < RL; ++r) {
        const int p = out_pos<M2, SL>(tid, b, r);
        if (p >= 1 && p < nx) {
          const double va = -v[b * RL + r].y, vb = v[b * RL + r].x;
          if (oka) sa[p] = va;
          if (okb) sb[p] = vb;
          if (sprev != nullptr) {
            if (oka) {
              const double d = va - sprev[(size_t)ja * P + p];
              acc += d * d;
            }
            if (okb) {
              const double d = vb - sprev[(size_t)(ja + 1) * P + p];
              acc += d * d;
            }
          }
        }
      }
    __syncthreads();  // LDS is rewritten by the next item
  }
  if (part != nullptr) {
    double* red = reinterpret_cast<double*>(lds);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = C::THREADS / 2; off > 0; off >>= 1) {
      if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
  }
}

// The inverse row pass for transforms of up to 4096 points: ONE small item (256 threads:
// one row pair at M2 = 4096) per workgroup, not persistent, component-wise LDS (34 KB), so
// four workgroups per CU overlap each other's loads, transforms and stores -- the shape of
// the periodic solver's rows_inv_np_kernel.  A thread's entries all belong to one row, so
// the real part of the packed extension (first row of a pair) is written by one half of the
// threads and the imaginary part by the other, one component at a time.
template <int M2>
struct DstNpCfg {
  static constexpr int T = Plan<M2>::T;
  static constexpr int RP = 256 / T < 1 ? 1 : 256 / T;
  static constexpr int ROWS = 2 * RP;
  static constexpr int THREADS = RP * T;
  static constexpr int ENTRIES = (M2 / 4) * ROWS / THREADS;
};

// Minimum wavefronts per SIMD the inverse kernel is compiled for: at M2 = 4096 (256-thread
// workgroups, 35 KB of LDS: four per CU) it wants 132 registers -- three workgroups per CU,
// and the 1024 workgroups of a 2048^2 solve take one round and a third; 128 registers make it
// one round.
#ifndef CFDJ_DST_INV_NP_WAVES_4096
#define CFDJ_DST_INV_NP_WAVES_4096 4
#endif
template <int M2>
constexpr int dst_inv_np_waves() {
  return M2 == 4096 ? CFDJ_DST_INV_NP_WAVES_4096 : 1;
}
template <int M2>
__global__ __launch_bounds__(DstNpCfg<M2>::THREADS)
    __attribute__((amdgpu_waves_per_eu(dst_inv_np_waves<M2>()))) void dst_rows_inv_np_kernel(
    const double2* __restrict__ T, int JT, double* __restrict__ s, int P, int ny,
    const double2* __restrict__ tw_, const double* __restrict__ sprev,
    double* __restrict__ part) {
  using PL = Plan<M2>;
  using C = DstNpCfg<M2>;
  constexpr int nx = M2 / 2;
  __shared__ double lds[C::RP * PL::PAD];
  const TwGlobal<M2> tw{tw_};
  const int q = threadIdx.x / PL::T, tid = threadIdx.x % PL::T;
  double* buf = lds + q * PL::PAD;
  const int slot0 = xcd_remap(blockIdx.x, gridDim.x) * C::ROWS;
  auto entry = [](int i, int& rr, int& kap) {
    const int e = threadIdx.x + i * C::THREADS;
    rr = (e >> 4) % C::ROWS;
    kap = ((e >> 4) / C::ROWS) * 16 + (e & 15);
  };
  double2 ent[C::ENTRIES];
  {
    const double2* tb = T + __builtin_amdgcn_readfirstlane(slot0);
#pragma unroll
    for (int i = 0; i < C::ENTRIES; ++i) {
      int rr, kap;
      entry(i, rr, kap);
      ent[i] = tb[(unsigned)(kap * JT + rr)];
    }
  }
  double2 v[16];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c) __syncthreads();
    // entries -> the odd extension of their row: mode k at p = k and, negated, at
    // p = 2nx - k; p = 0 and p = nx are zero (the kappa = 0 lanes write them)
#pragma unroll
    for (int i = 0; i < C::ENTRIES; ++i) {
      int rr, kap;
      entry(i, rr, kap);
      if ((rr & 1) == c) {
        double* bq = lds + (rr >> 1) * PL::PAD;
        const int k0 = 2 * kap, k1 = k0 + 1;
        const double v0 = k0 == 0 ? 0.0 : ent[i].x;
        bq[padx(k0)] = v0;
        bq[padx(k1)] = ent[i].y;
        if (k0 != 0) bq[padx(M2 - k0)] = -v0;
        else bq[padx(nx)] = 0.0;
        bq[padx(M2 - k1)] = -ent[i].y;
      }
    }
    __syncthreads();
    if (c) lds_read_half<M2, 0, 1>(buf, v, tid);
    else lds_read_half<M2, 0, 0>(buf, v, tid);
  }
  stage_regs<M2, 0, -1>(v, tid, tw);
  run_stages_half<M2, 1, -1>(buf, v, tid, tw);
  constexpr int SL = PL::NSTAGES - 1;
  constexpr int RL = PL::radix(SL);
  const int ja = 1 + slot0 + 2 * q;
  const bool oka = ja <= ny - 1, okb = ja + 1 <= ny - 1;
  double* sa = s + (size_t)ja * P;
  double* sb = sa + P;
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) {
      const int p = out_pos<M2, SL>(tid, b, r);
      if (p >= 1 && p < nx) {
        const double va = -v[b * RL + r].y, vb = v[b * RL + r].x;
        if (oka) sa[p] = va;
        if (okb) sb[p] = vb;
        if (sprev != nullptr) {
          if (oka) {
            const double d = va - sprev[(size_t)ja * P + p];
            acc += d * d;
          }
          if (okb) {
            const double d = vb - sprev[(size_t)(ja + 1) * P + p];
            acc += d * d;
          }
        }
      }
    }
  if (part != nullptr) {
    __syncthreads();  // the buffer's last readers are done
    double* red = lds;
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = C::THREADS / 2; off > 0; off >>= 1) {
      if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
  }
}

// The forward row pass in the same small-item shape (CFDJ_DST_FWD_NP): the packed transform's
// outputs go through the buffer one component at a time into natural order; an entry of the
// pair's first row needs the imaginary parts only (-Im Z), one of its second row the real
// parts (Re Z).
#ifndef CFDJ_DST_FWD_NP
#define CFDJ_DST_FWD_NP 1
#endif
template <int M2>
constexpr bool dst_fwd_np() { return CFDJ_DST_FWD_NP != 0 && M2 <= CFDJ_DST_NP_MAXM2; }

template <int M2>
__global__ __launch_bounds__(DstNpCfg<M2>::THREADS) void dst_rows_fwd_np_kernel(
    const double* __restrict__ w, int P, int ny, double2* __restrict__ T, int JT, double sgn,
    const double2* __restrict__ tw_) {
  using PL = Plan<M2>;
  using C = DstNpCfg<M2>;
  __shared__ double lds[C::RP * PL::PAD];
  const TwGlobal<M2> tw{tw_};
  const int q = threadIdx.x / PL::T, tid = threadIdx.x % PL::T;
  double* buf = lds + q * PL::PAD;
  const int slot0 = xcd_remap(blockIdx.x, gridDim.x) * C::ROWS;
  double2 v[16];
  load_row_pair<M2>(v, w, P, ny, 1 + slot0 + 2 * q, tid, sgn);
  stage_regs<M2, 0, -1>(v, tid, tw);
  run_stages_half<M2, 1, -1>(buf, v, tid, tw);
  constexpr int SL = PL::NSTAGES - 1;
  constexpr int RL = PL::radix(SL);
  auto entry = [](int i, int& rr, int& kap) {
    const int e = threadIdx.x + i * C::THREADS;
    rr = (e >> 4) % C::ROWS;
    kap = ((e >> 4) / C::ROWS) * 16 + (e & 15);
  };
  double2 o[C::ENTRIES];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
      for (int r = 0; r < RL; ++r)
        buf[padx(out_pos<M2, SL>(tid, b, r))] = c ? v[b * RL + r].y : v[b * RL + r].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < C::ENTRIES; ++i) {
      int rr, kap;
      entry(i, rr, kap);
      if ((rr & 1) != c) {  // second row of a pair: Re Z (c = 0); first row: -Im Z (c = 1)
        const double* bq = lds + (rr >> 1) * PL::PAD;
        const double z0 = bq[padx(2 * kap)], z1 = bq[padx(2 * kap + 1)];
        o[i] = c ? make_double2(-z0, -z1) : make_double2(z0, z1);
      }
    }
  }
  double2* tb = T + __builtin_amdgcn_readfirstlane(slot0);
#pragma unroll
  for (int i = 0; i < C::ENTRIES; ++i) {
    int rr, kap;
    entry(i, rr, kap);
    tb[(unsigned)(kap * JT + rr)] = o[i];
  }
}

// One mode pair per workgroup: packed y-DST, times iden, packed y-DST, in place.
#ifndef CFDJ_DST_COLS_WAVES
#define CFDJ_DST_COLS_WAVES 3
#endif
// Values per thread (16 or 8): a pass has only nx / 2 columns (four per CU at 2048^2), so its
// time is the latency of one column's chain of loads, stages and exchanges times the rounds
// of resident workgroups -- twice the threads per column shorten that chain.
#ifndef CFDJ_DST_COLS_NV
#define CFDJ_DST_COLS_NV 16
#endif
constexpr int kDstNV = CFDJ_DST_COLS_NV;
// Wavefronts per SIMD the kernel is compiled for (the register cap): one per resident
// 256-thread workgroup at M2 = 4096.
template <int M2>
constexpr int dst_cols_waves() {
  return kDstNV == 8 ? 4 : (M2 <= 4096 ? CFDJ_DST_COLS_WAVES : 2);
}

template <int M2>
__global__ __launch_bounds__((Plan<M2, kDstNV>::T))
    __attribute__((amdgpu_waves_per_eu(dst_cols_waves<M2>(), dst_cols_waves<M2>()))) void dst_cols_kernel(double2* __restrict__ T, int JT,
                                                             const double* __restrict__ tx,
                                                             const double* __restrict__ ty,
                                                             double scale,
                                                             const double2* __restrict__ tw_) {
  constexpr int NV = kDstNV;
  using PL = Plan<M2, NV>;
  static_assert(PL::NSTAGES >= 2, "column length");
  constexpr int ny = M2 / 2;
  __shared__ double lds[PL::PAD];  // one component at a time (exchange_half): 3 per CU
  const TwGlobal<M2> tw{tw_};
  const int tid = threadIdx.x;
  const int kap = xcd_remap(blockIdx.x, gridDim.x);
  double2* col = T + (size_t)kap * JT;  // row j in slot j - 1

  double2 a[NV];
  constexpr int R0 = PL::radix(0);
#pragma unroll
  for (int b = 0; b < NV / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int p = in_pos<M2, 0, NV>(tid, b, r);
      const bool zero = (p & (ny - 1)) == 0;
      const int j = p < ny ? p : M2 - p;
      const double2 c = col[zero ? 0 : j - 1];
      const double s = p < ny ? 1.0 : -1.0;
      a[b * R0 + r] = zero ? make_double2(0.0, 0.0) : make_double2(s * c.x, s * c.y);
    }
  stage_regs<M2, 0, -1>(a, tid, tw);
  run_stages_half<M2, 1, -1>(lds, a, tid, tw);  // last stage stays in registers

  double2 v[NV];
  fwd_to_inv<M2>(a, v);  // v[r] = Z[p], p = tid + T r
  const double txa = tx[2 * kap], txb = tx[2 * kap + 1];
#pragma unroll
  for (int r = 0; r < NV; ++r) {
    const int p = tid + PL::T * r;
    const bool zero = (p & (ny - 1)) == 0;
    const double t = ty[p];  // even in p about ny (the table holds the extension)
    // S_a = -Im Z, S_b = Re Z; times iden (lid_driven_cavity.jl:17), then the second
    // transform's input ext(S_a iden_a) + i ext(S_b iden_b): the oddness is already there
    const double ia = recip_nr(fd_symbol(txa, 1.0, t));
    const double ib = recip_nr(fd_symbol(txb, 1.0, t));
    const double2 z = make_double2((-v[r].y * ia) * scale, (v[r].x * ib) * scale);
    v[r] = zero ? make_double2(0.0, 0.0) : z;
  }
  stage_regs<M2, 0, -1>(v, tid, tw);
  run_stages_half<M2, 1, -1>(lds, v, tid, tw);
  constexpr int SL = PL::NSTAGES - 1;
  constexpr int RL = PL::radix(SL);
#pragma unroll
  for (int b = 0; b < NV / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) {
      const int p = out_pos<M2, SL, NV>(tid, b, r);
      if (p >= 1 && p < ny) col[p - 1] = make_double2(-v[b * RL + r].y, v[b * RL + r].x);
    }
}

// ---------------------------------------------------------------------------------------
// Half-length DST-I.  The kernels above transform the odd extension of a row: a complex FFT
// of length 2n for two rows of n - 1 values.  The ones below get the same coefficients from a
// complex FFT of length n (half the arithmetic, half the LDS): with y_0 = 0,
//   y_j = sin(pi j / n) (x_j + x_{n-j}) + (x_j - x_{n-j}) / 2,   j = 1 .. n-1,
// and Y = FFT_n(y) = R + i I, the sine coefficients S_k = 2 sum_j x_j sin(pi j k / n) are
//   S_{2k} = -2 I_k,      S_{2k+1} = S_{2k-1} + 2 R_k   (S_1 = R_0),
// i.e. the odd ones are a running sum over k.  Two rows a, b ride one complex transform
// z = y_a + i y_b; their spectra separate by pairing Z_k with conj Z_{n-k}.  Round-off grows
// with the running sum: 3-5e-15 of max|S| at n = 2048..4096 against scipy's DST-I (the
// odd-extension route: 4e-16), far inside the 1e-12 the solve is held to.
//
// Z in natural order -> (S_a, S_b) at the even modes 2k (ev) and the odd modes 2k + 1 (od),
// k = tid + T i, i < 8, of a team of T = N / 16 threads.  buf: the team's exchange buffer
// (Plan<N>::PAD doubles); wtot: W = T / 64 double2 per team (unused where T <= 64).
template <int N>
__device__ __forceinline__ void dsth_post(double* buf, double2* wtot, const double2 (&v)[16],
                                          int tid, double2 (&ev)[8], double2 (&od)[8]) {
  using PL = Plan<N>;
  constexpr int T = PL::T, SL = PL::NSTAGES - 1, W = T / 64 < 1 ? 1 : T / 64;
  constexpr int WIDTH = T < 64 ? T : 64;
  double2 zk[8], zm[8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();
    if (c) lds_write_half<N, SL, 1>(buf, v, tid);
    else lds_write_half<N, SL, 0>(buf, v, tid);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = tid + T * i;
      const double a = buf[padx(k)], b = buf[padx((N - k) & (N - 1))];
      if (c) {
        zk[i].y = a;
        zm[i].y = b;
      } else {
        zk[i].x = a;
        zm[i].x = b;
      }
    }
  }
  // Y_a = (Z_k + conj Z_{n-k}) / 2, Y_b = (Z_k - conj Z_{n-k}) / (2i)
  double2 r[8];  // 2 R_k of rows a, b (k = 0: R_0)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ev[i] = make_double2(zm[i].y - zk[i].y, zk[i].x - zm[i].x);  // -2 I_k
    r[i] = make_double2(zk[i].x + zm[i].x, zk[i].y + zm[i].y);
    if (i == 0 && tid == 0) r[i] = make_double2(0.5 * r[i].x, 0.5 * r[i].y);
  }
  // running sum over k through the buffer: row a's terms at k, row b's at N/2 + k; a thread
  // sums the 8 consecutive k of its chunk, the chunks' totals are scanned across the team
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    buf[padx(tid + T * i)] = r[i].x;
    buf[padx(N / 2 + tid + T * i)] = r[i].y;
  }
  __syncthreads();
  double2 c8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    c8[j] = make_double2(buf[padx(8 * tid + j)], buf[padx(N / 2 + 8 * tid + j)]);
#pragma unroll
  for (int j = 1; j < 8; ++j) c8[j] = make_double2(c8[j].x + c8[j - 1].x, c8[j].y + c8[j - 1].y);
  double2 tot = c8[7];  // inclusive scan of the chunk totals over the wavefront's team lanes
  const int ln = tid & (WIDTH - 1);
#pragma unroll
  for (int d = 1; d < WIDTH; d <<= 1) {
    const double tx = __shfl_up(tot.x, d, WIDTH), ty = __shfl_up(tot.y, d, WIDTH);
    if (ln >= d) tot = make_double2(tot.x + tx, tot.y + ty);
  }
  double2 carry = make_double2(tot.x - c8[7].x, tot.y - c8[7].y);  // exclusive
  if constexpr (W > 1) {
    const int wv = tid / 64;
    if (ln == 63) wtot[wv] = tot;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < W - 1; ++w)
      if (w < wv) carry = make_double2(carry.x + wtot[w].x, carry.y + wtot[w].y);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    buf[padx(8 * tid + j)] = c8[j].x + carry.x;
    buf[padx(N / 2 + 8 * tid + j)] = c8[j].y + carry.y;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i)
    od[i] = make_double2(buf[padx(tid + T * i)], buf[padx(N / 2 + tid + T * i)]);
}

// W_N^e from the table of W_2N.
template <int N>
struct TwEven {
  const double2* __restrict__ t;
  __device__ __forceinline__ double2 w(int e) const { return t[2 * e]; }
};

// y of the definition above from x_p and x_{n-p}; sn = sin(pi p / n).
__device__ __forceinline__ double dsth_y(double x1, double x2, double sn) {
  return sn * (x1 + x2) + 0.5 * (x1 - x2);
}

template <int N>
struct DsthCfg {
  static constexpr int T = Plan<N>::T;
  static constexpr int RP = 256 / T < 1 ? 1 : 256 / T;  // row pairs per workgroup
  static constexpr int ROWS = 2 * RP;
  static constexpr int THREADS = RP * T;
  static constexpr int W = T / 64 < 1 ? 1 : T / 64;
};

// Forward row pass: rows ja, ja + 1 of the node array -> T[kappa][row] = (S_2kappa, S_2kappa+1).
template <int N>
__global__ __launch_bounds__(DsthCfg<N>::THREADS) void dsth_rows_fwd_kernel(
    const double* __restrict__ w, int P, int ny, double2* __restrict__ Tt, int JT, double sgn,
    const double2* __restrict__ tw2n) {
  using PL = Plan<N>;
  using C = DsthCfg<N>;
  __shared__ double lds[C::RP * PL::PAD];
  __shared__ double2 wtot[C::RP][C::W];
  const TwEven<N> tw{tw2n};
  const int q = threadIdx.x / C::T, tid = threadIdx.x % C::T;
  double* buf = lds + q * PL::PAD;
  const int slot0 = xcd_remap(blockIdx.x, gridDim.x) * C::ROWS;
  const int ja = 1 + slot0 + 2 * q;
  const bool oka = ja <= ny - 1, okb = ja + 1 <= ny - 1;
  const double* ra = w + (size_t)(oka ? ja : 1) * P;
  const double* rb = w + (size_t)(okb ? ja + 1 : 1) * P;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = tid + C::T * r;
    const int p1 = p == 0 ? 1 : p, p2 = p == 0 ? 1 : N - p;  // (p = 0: y = 0)
    const double sn = -tw2n[p].y;  // sin(pi p / N)
    const double ya = dsth_y(ra[p1], ra[p2], sn), yb = dsth_y(rb[p1], rb[p2], sn);
    v[r] = make_double2(p == 0 || !oka ? 0.0 : sgn * ya, p == 0 || !okb ? 0.0 : sgn * yb);
  }
  stage_regs<N, 0, -1>(v, tid, tw);
  run_stages_half<N, 1, -1>(buf, v, tid, tw);
  double2 ev[8], od[8];
  dsth_post<N>(buf, wtot[q], v, tid, ev, od);
  double2* tb = Tt + __builtin_amdgcn_readfirstlane(slot0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const unsigned o = (unsigned)((tid + C::T * i) * JT + 2 * q);
    tb[o] = make_double2(ev[i].x, od[i].x);
    tb[o + 1] = make_double2(ev[i].y, od[i].y);
  }
}

// Inverse row pass: T[kappa][row] -> rows ja, ja + 1 of s (interior nodes), and the partial
// sums of (s_new - sprev)^2 as in dst_rows_inv_np_kernel.
template <int N>
__global__ __launch_bounds__(DsthCfg<N>::THREADS) void dsth_rows_inv_kernel(
    const double2* __restrict__ Tt, int JT, double* __restrict__ s, int P, int ny,
    const double2* __restrict__ tw2n, const double* __restrict__ sprev,
    double* __restrict__ part) {
  using PL = Plan<N>;
  using C = DsthCfg<N>;
  __shared__ double lds[C::RP * PL::PAD];
  __shared__ double2 wtot[C::RP][C::W];
  const TwEven<N> tw{tw2n};
  const int q = threadIdx.x / C::T, tid = threadIdx.x % C::T;
  double* buf = lds + q * PL::PAD;
  const int slot0 = xcd_remap(blockIdx.x, gridDim.x) * C::ROWS;
  const double2* tb = Tt + __builtin_amdgcn_readfirstlane(slot0);
  double2 ea[8], eb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const unsigned o = (unsigned)((tid + C::T * i) * JT + 2 * q);
    ea[i] = tb[o];
    eb[i] = tb[o + 1];
  }
  if (tid == 0) ea[0].x = eb[0].x = 0.0;  // mode 0 of a sine series does not exist
  // the rows' coefficients in natural order, one row at a time, read back at p and n - p
  double2 v[16];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = tid + C::T * i;
      buf[padx(2 * k)] = c ? eb[i].x : ea[i].x;
      buf[padx(2 * k + 1)] = c ? eb[i].y : ea[i].y;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = tid + C::T * r;
      const double y = dsth_y(buf[padx(p)], buf[padx((N - p) & (N - 1))], -tw2n[p].y);
      if (c) v[r].y = y;
      else v[r].x = y;
    }
  }
  stage_regs<N, 0, -1>(v, tid, tw);
  run_stages_half<N, 1, -1>(buf, v, tid, tw);
  double2 ev[8], od[8];
  dsth_post<N>(buf, wtot[q], v, tid, ev, od);
  const int ja = 1 + slot0 + 2 * q;
  const bool oka = ja <= ny - 1, okb = ja + 1 <= ny - 1;
  double* sa = s + (size_t)ja * P;
  double* sb = sa + P;
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = 2 * (tid + C::T * i);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (p + h >= 1) {
        const double va = h ? od[i].x : ev[i].x, vb = h ? od[i].y : ev[i].y;
        if (oka) sa[p + h] = va;
        if (okb) sb[p + h] = vb;
        if (sprev != nullptr) {
          if (oka) {
            const double d = va - sprev[(size_t)ja * P + p + h];
            acc += d * d;
          }
          if (okb) {
            const double d = vb - sprev[(size_t)(ja + 1) * P + p + h];
            acc += d * d;
          }
        }
      }
    }
  }
  if (part != nullptr) {
    __syncthreads();  // the buffer's last readers are done
    double* red = lds;
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = C::THREADS / 2; off > 0; off >>= 1) {
      if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
  }
}

// Column pass: one mode pair per workgroup (its column holds two real columns as the
// components of a double2): y-DST, times iden, y-DST, in place.
#ifndef CFDJ_DSTH_COLS_WAVES
#define CFDJ_DSTH_COLS_WAVES 3
#endif
template <int N>
__global__ __launch_bounds__((Plan<N>::T))
    __attribute__((amdgpu_waves_per_eu(CFDJ_DSTH_COLS_WAVES, CFDJ_DSTH_COLS_WAVES))) void dsth_cols_kernel(
        double2* __restrict__ Tt, int JT, const double* __restrict__ tx,
        const double* __restrict__ ty, double scale, const double2* __restrict__ tw2n) {
  using PL = Plan<N>;
  constexpr int T = PL::T, W = T / 64 < 1 ? 1 : T / 64;
  __shared__ double buf[PL::PAD];
  __shared__ double2 wtot[W];
  const TwEven<N> tw{tw2n};
  const int tid = threadIdx.x;
  const int kap = xcd_remap(blockIdx.x, gridDim.x);
  double2* col = Tt + (size_t)kap * JT;  // row j in slot j - 1
  double2 v[16];
  {
    // x_p into v, x_{n-p} into c2, y in place; p = 0 (thread 0's first element: y = 0) reads
    // slot 0 for both, so its difference is zero like its sine
    double2 c2[16];
    const int z0 = tid == 0 ? 1 : 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = col[(unsigned)(tid + T * r - 1 + (r == 0 ? z0 : 0))];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      c2[r] = col[(unsigned)(N - 1 - tid - T * r - (r == 0 ? z0 * (N - 1) : 0))];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const double sn = -tw2n[tid + T * r].y;
      v[r] = make_double2(dsth_y(v[r].x, c2[r].x, sn), dsth_y(v[r].y, c2[r].y, sn));
    }
  }
  stage_regs<N, 0, -1>(v, tid, tw);
  run_stages_half<N, 1, -1>(buf, v, tid, tw);
  double2 ev[8], od[8];
  dsth_post<N>(buf, wtot, v, tid, ev, od);
  // times iden (lid_driven_cavity.jl:17) and the transforms' normalisation
  const double txa = tx[2 * kap], txb = tx[2 * kap + 1];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = 2 * (tid + T * i);
    const double t0 = ty[p], t1 = ty[p + 1];
    const double2 e = ev[i], o = od[i];
    ev[i] = p == 0 ? make_double2(0.0, 0.0)
                   : make_double2((e.x * recip_nr(fd_symbol(txa, 1.0, t0))) * scale,
                                  (e.y * recip_nr(fd_symbol(txb, 1.0, t0))) * scale);
    od[i] = make_double2((o.x * recip_nr(fd_symbol(txa, 1.0, t1))) * scale,
                         (o.y * recip_nr(fd_symbol(txb, 1.0, t1))) * scale);
  }
  // second transform: the products in natural order, one component at a time.  It works from
  // an opaque copy of the thread index: the twiddles, sines and buffer addresses of the first
  // transform are formed again instead of staying in registers (or spilled) across both.
  int t2 = tid;
  asm volatile("" : "+v"(t2));
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = t2 + T * i;
      buf[padx(2 * k)] = c ? ev[i].y : ev[i].x;
      buf[padx(2 * k + 1)] = c ? od[i].y : od[i].x;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = t2 + T * r;
      const double y = dsth_y(buf[padx(p)], buf[padx((N - p) & (N - 1))], -tw2n[p].y);
      if (c) v[r].y = y;
      else v[r].x = y;
    }
  }
  stage_regs<N, 0, -1>(v, t2, tw);
  run_stages_half<N, 1, -1>(buf, v, t2, tw);
  dsth_post<N>(buf, wtot, v, t2, ev, od);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const unsigned p = 2 * (t2 + T * i);
    if (p >= 1) col[p - 1] = ev[i];
    col[p] = od[i];
  }
}

template <int M2>
int dst_rows_grid_t(int ny, int ncu) {
  using C = DstRowCfg<M2>;
  int nb = ncu - ncu % 8;
  if (nb < 8) nb = 8;
  const int items = ny / C::ROWS;
  return nb < items ? nb : items;
}

// The inverse pass's grid: one workgroup per small item where the non-persistent kernel
// applies (transforms of up to 4096 points, CFDJ_DST_INV_NP != 0), else the persistent grid.
#ifndef CFDJ_DST_INV_NP
#define CFDJ_DST_INV_NP 1
#endif
template <int M2>
constexpr bool dst_inv_np() { return CFDJ_DST_INV_NP != 0 && M2 <= CFDJ_DST_NP_MAXM2; }
template <int M2>
int dst_rows_inv_grid_t(int ny, int ncu) {
  if (dst_inv_np<M2>() && ny % DstNpCfg<M2>::ROWS == 0) return ny / DstNpCfg<M2>::ROWS;
  return dst_rows_grid_t<M2>(ny, ncu);
}

template <int M2>
void launch_dst_rows(int pass, const DstPoissonArgs& a, hipStream_t st) {
  using C = DstRowCfg<M2>;
  const dim3 grid(dst_rows_grid_t<M2>(a.ny, a.ncu));
  if (pass == 0 && dst_fwd_np<M2>() && a.ny % DstNpCfg<M2>::ROWS == 0) {
    hipLaunchKernelGGL((dst_rows_fwd_np_kernel<M2>), dim3(a.ny / DstNpCfg<M2>::ROWS),
                       dim3(DstNpCfg<M2>::THREADS), 0, st, a.w, a.P, a.ny, a.T, a.JT,
                       a.neg ? -1.0 : 1.0, a.twX);
  } else if (pass == 0) {
    hipLaunchKernelGGL((dst_rows_fwd_kernel<M2>), grid, dim3(C::THREADS), 0, st, a.w, a.P, a.ny,
                       a.T, a.JT, a.neg ? -1.0 : 1.0, a.twX);
  } else if (dst_inv_np<M2>() && a.ny % DstNpCfg<M2>::ROWS == 0) {
    hipLaunchKernelGGL((dst_rows_inv_np_kernel<M2>), dim3(a.ny / DstNpCfg<M2>::ROWS),
                       dim3(DstNpCfg<M2>::THREADS), 0, st, a.T, a.JT, a.s, a.P, a.ny, a.twX,
                       a.sprev, a.sprev ? a.part : nullptr);
  } else {
    hipLaunchKernelGGL((dst_rows_inv_kernel<M2>), grid, dim3(C::THREADS), 0, st, a.T, a.JT, a.s,
                       a.P, a.ny, a.twX, a.sprev, a.sprev ? a.part : nullptr);
  }
}

template <int M2>
void launch_dst_cols(const DstPoissonArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((dst_cols_kernel<M2>), dim3(a.nx / 2), dim3(Plan<M2, kDstNV>::T), 0, st, a.T, a.JT,
                     a.tx, a.ty, a.scale, a.twY);
}

constexpr bool pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

template <int N>
void launch_dsth(int pass, const DstPoissonArgs& a, hipStream_t st) {
  using C = DsthCfg<N>;
  if (pass == 1) {
    hipLaunchKernelGGL((dsth_cols_kernel<N>), dim3(a.nx / 2), dim3(Plan<N>::T), 0, st, a.T, a.JT,
                       a.tx, a.ty, a.scale, a.twY);
  } else if (pass == 0) {
    hipLaunchKernelGGL((dsth_rows_fwd_kernel<N>), dim3(a.ny / C::ROWS), dim3(C::THREADS), 0, st,
                       a.w, a.P, a.ny, a.T, a.JT, a.neg ? -1.0 : 1.0, a.twX);
  } else {
    hipLaunchKernelGGL((dsth_rows_inv_kernel<N>), dim3(a.ny / C::ROWS), dim3(C::THREADS), 0, st,
                       a.T, a.JT, a.s, a.P, a.ny, a.twX, a.sprev, a.sprev ? a.part : nullptr);
  }
}

template <int N>
int dsth_rows_grid_t(int ny) { return ny / DsthCfg<N>::ROWS; }

}  // namespace

bool dst_poisson_supported(int nx, int ny) {
  return pow2(nx) && pow2(ny) && nx >= 512 && nx <= 4096 && ny >= 512 && ny <= 4096;
}

// Workgroups of the inverse row pass = entries of its `part` output (at most 2048).
int dst_half_passes(int nx, int ny) {
  const char* e = std::getenv("CFDJ_DST_HALF");
  if (e && e[0] == '0') return 0;
  if (e && e[0] == '1') return 7;
  if (e && e[0] == 'm') return std::atoi(e + 1) & 7;  // (A/B: a mask of passes)
  // columns from 2048 points on; rows never: at nx = 4096 the small-item odd-extension kernels
  // (8192-point transforms, two 512-thread workgroups per CU since the remainder stage's
  // twiddles stopped costing 24-47 registers) take 100 / 98 us per pass of a 4096^2 solve
  // against the half-length kernels' 105 / 108
  (void)nx;
  return ny >= 2048 ? 2 : 0;
}

int dst_rows_grid(int nx, int ny, int ncu, int half) {
  if (half & 4) {
    switch (nx) {
      case 512: return dsth_rows_grid_t<512>(ny);
      case 1024: return dsth_rows_grid_t<1024>(ny);
      case 2048: return dsth_rows_grid_t<2048>(ny);
      default: return dsth_rows_grid_t<4096>(ny);
    }
  }
  switch (2 * nx) {
    case 1024: return dst_rows_inv_grid_t<1024>(ny, ncu);
    case 2048: return dst_rows_inv_grid_t<2048>(ny, ncu);
    case 4096: return dst_rows_inv_grid_t<4096>(ny, ncu);
    default: return dst_rows_inv_grid_t<8192>(ny, ncu);
  }
}

void launch_dst_poisson_pass(int pass, const DstPoissonArgs& a, hipStream_t st) {
  if (!dst_poisson_supported(a.nx, a.ny) || a.JT < a.ny || a.P < a.nx + 1)
    throw Error{CFDJ_ERR_ARG, "DST Poisson: unsupported size"};
  const int n = pass == 1 ? a.ny : a.nx;
  if (pass < 0 || pass > 2) throw Error{CFDJ_ERR_ARG, "DST Poisson: bad pass"};
  if ((a.half >> pass) & 1) {
    switch (n) {
      case 512: launch_dsth<512>(pass, a, st); break;
      case 1024: launch_dsth<1024>(pass, a, st); break;
      case 2048: launch_dsth<2048>(pass, a, st); break;
      default: launch_dsth<4096>(pass, a, st); break;
    }
    CFDJ_HIP(hipGetLastError());
    return;
  }
  switch (2 * n) {
    case 1024: pass == 1 ? launch_dst_cols<1024>(a, st) : launch_dst_rows<1024>(pass, a, st); break;
    case 2048: pass == 1 ? launch_dst_cols<2048>(a, st) : launch_dst_rows<2048>(pass, a, st); break;
    case 4096: pass == 1 ? launch_dst_cols<4096>(a, st) : launch_dst_rows<4096>(pass, a, st); break;
    default: pass == 1 ? launch_dst_cols<8192>(a, st) : launch_dst_rows<8192>(pass, a, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
