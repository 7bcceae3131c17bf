// Hand-written fused FD-FFT Poisson solver for square power-of-two grids (gfx950).
//
// Replaces rocFFT D2Z + divide + Z2D (8 rocFFT passes + 1 divide pass over HBM at 4096^2)
// with THREE passes (Common.jl:97-125 semantics):
//
//   rows_fwd   : each row of the real field f (N reals) is read as N/2 complex z[n] =
//                f[2n] + i f[2n+1], FFT'd (length L = N/2, Stockham radix-16 in LDS), and
//                post-processed into the real-FFT half spectrum X[m], m = 0..L-1, with the
//                two real coefficients X[0] (DC) and X[L] (Nyquist) packed into slot 0 as
//                X[0] + i X[L].  Output is written COLUMN-MAJOR, H[m][y] (y contiguous):
//                a workgroup owns XR = 4 consecutive rows, so every column piece it writes
//                is a full 64-B segment, and the column pass reads one contiguous 64 KB
//                column.
//   cols       : one workgroup per column: forward FFT along y (length M), the
//                spectral divide by the FD symbol aa + bb cos kx + cc cos ky (Common.jl:119-
//                121; packed column 0 is split into its DC and Nyquist halves with the
//                Z[k], Z[-k] symmetry, each divided by its own symbol), the inverse FFT, all
//                in LDS; written back in place.  1/(N M) is folded into the divide.
//   rows_inv   : c2r of each row (pre-processing inverse of the above + inverse FFT),
//                writing the real streamfunction.
//
// Twiddles come from host-built tables (long-double accurate) read through L1/L2.  FMA
// contraction is allowed here: the FFT is not bit-comparable to FFTW / pocketfft anyway
// (tolerance 1e-12 relative on psi, tests/test_gpu_parity.py).
#pragma clang fp contract(fast)
#include <cstdlib>
#include <type_traits>

#include "colsum.hpp"
#include "fft_lds.hpp"

namespace cfdj {

namespace {

// ---------------------------------------------------------------------------------------
// Pass 1: rows, real -> packed half spectrum, column-major output H[m][y].
// ---------------------------------------------------------------------------------------
template <int L, bool FWD = true>
struct RowCfg {
  static constexpr int T = Plan<L>::T;
  // rows per work item: >= 4 (64-B column segments) where the LDS holds them, fewer for
  // the long rows of the multi-GPU grids (L = 4096: 2, L = 8192: 1 -- 136 KB per row)
  // (separately for the forward and the inverse pass: the segment size is an access
  // pattern of each pass, not a property of the spectrum layout)
#ifndef CFDJ_ROWS_FWD_XR_MIN
#define CFDJ_ROWS_FWD_XR_MIN 4
#endif
#ifndef CFDJ_ROWS_INV_XR_MIN
#define CFDJ_ROWS_INV_XR_MIN 4
#endif
  static constexpr int XR_MIN = FWD ? CFDJ_ROWS_FWD_XR_MIN : CFDJ_ROWS_INV_XR_MIN;
  static constexpr int XR_WANT = (256 / T) > XR_MIN ? (256 / T) : XR_MIN;
  static constexpr int XR_FIT = (140 * 1024) / (Plan<L>::ROWSTRIDE * 16);
  static constexpr int XR = XR_WANT < XR_FIT ? XR_WANT : XR_FIT;
  static_assert(XR >= 1, "row does not fit the LDS");
  static constexpr int THREADS = XR * T;
  static constexpr int PAIRS = (L / 2) * XR / THREADS;  // (m, L-m) pairs per thread
};

// Element pair p of a work item: row qq, columns m and L-m (m = p in [0, L/2)).  Lanes take
// 16 consecutive m of one row, so both LDS accesses are contiguous per row and both global
// accesses cover whole XR*16-B column segments.
template <int L, bool FWD>
__device__ __forceinline__ void pair_index(int e, int& qq, int& m) {
  using C = RowCfg<L, FWD>;
  qq = (e >> 4) % C::XR;
  m = ((e >> 4) / C::XR) * 16 + (e & 15);
}

// Element (m, y) of a half spectrum with `M` rows: column-major (m M + y) or, for the
// substructured y-slab path, in 8-mode tiles (((m/8) M + y) 8 + m%8): a row's modes are
// whole 128-B lines, and the Schur kernels' column reads of 8 neighbouring modes share
// them in L2 (TILE = true).
template <bool TILE>
__device__ __forceinline__ size_t sidx(int m, int y, int M) {
  if constexpr (TILE) return ((((size_t)(m >> 3)) * M + y) << 3) + (m & 7);
  else return (size_t)m * M + y;
}

// Prefetch loads use a wave-uniform base pointer and unsigned 32-bit element offsets, so
// each load needs one offset VGPR (global_load ... saddr) instead of a 64-bit address pair.
template <int L, bool NT>
__device__ __forceinline__ void load_row_z(double2 (&v)[16], const double* __restrict__ f,
                                           int y, int tid) {
  // y is wave-uniform only when a row spans whole wavefronts (T >= 64)
  const int yu = Plan<L>::T >= 64 ? __builtin_amdgcn_readfirstlane(y) : y;
  const double2* z = reinterpret_cast<const double2*>(f) + (size_t)yu * L;
  constexpr int R0 = Plan<L>::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) v[b * R0 + r] = load_stream<NT>(z + (unsigned)in_pos<L, 0>(tid, b, r));
}

// One work item (XR rows) of the forward row pass: stage 0 on the prefetched rows in `nxt`,
// LDS write, refill `nxt` with the next item's rows (next_y0 >= 0), remaining stages,
// post-processing, stores.  The 16 stores per thread are unconditional and fully unrolled,
// and the kernel peels its first item, so every entry into the item loop carries the same
// queue of vector-memory operations (the 16 prefetch loads, then the 16 stores): the wait
// for the prefetched rows at the top of an item is then a counted `vmcnt` that leaves the
// previous item's stores in flight -- their drain overlaps stage 0 instead of stalling it
// (vmcnt completes in order; a conservative vmcnt(0) there cost a quarter of the pass).
template <int L, bool TILE, bool NT>
__device__ __forceinline__ void rows_fwd_item(double2 (&nxt)[16], double2* lds, double2* buf,
                                              const double* __restrict__ f,
                                              double2* __restrict__ H, int M, int y0,
                                              int next_y0, int q, int tid,
                                              const TwLds<L>& twL, const TwLds<2 * L>& twN) {
  using P = Plan<L>;
  using C = RowCfg<L, true>;
  stage_regs<L, 0, -1>(nxt, tid, twL);
  lds_write<L, 0>(buf, nxt, tid);
  if (next_y0 >= 0) load_row_z<L, NT>(nxt, f, next_y0 + q, tid);
  __syncthreads();
  double2 v[16];
  run_stages<L, 1, -1, true>(buf, v, tid, twL);

  // post-process, two outputs per pair: X[m] = E[m] + W^m O[m], X[L-m] likewise;
  // slot 0 = X[0] + i X[L]; m = L/2 is its own partner (stored by the m = 0 lane, which
  // can only occur in pair 0: later pairs start at m >= 16).  Stores go through a
  // wave-uniform base (row y0) and 32-bit element offsets: one offset VGPR per store.
  double2* hb = H + sidx<TILE>(0, __builtin_amdgcn_readfirstlane(y0), M);
#pragma unroll
  for (int i = 0; i < C::PAIRS; ++i) {
    int qq, m;
    pair_index<L, true>(threadIdx.x + i * C::THREADS, qq, m);
    const bool z0 = i == 0 && m == 0;
    const int mp = z0 ? L / 2 : L - m;
    const double2* bq = lds + qq * P::ROWSTRIDE;
    const double2 Zm = bq[padx(m)];
    const double2 Zp = bq[padx(mp)];
    const double2 Zc = cconj(Zp);
    const double2 E = make_double2(0.5 * (Zm.x + Zc.x), 0.5 * (Zm.y + Zc.y));
    const double2 D = csub(Zm, Zc);                       // = 2i O[m]
    const double2 O = make_double2(0.5 * D.y, -0.5 * D.x);  // D / (2i)
    const double2 WO = cmul(twN.w(m), O);
    double2 o1 = cadd(E, WO);
    // X[L-m] = conj(E[m]) + W^{L-m} conj(O[m]) = conj(E[m] - W^m O[m])
    double2 o2 = cconj(csub(E, WO));
    if (i == 0) {
      if (z0) {  // X[L/2] = E + W^{L/2} O, W^{L/2} = -i: conj(Z[L/2])
        o1 = make_double2(Zm.x + Zm.y, Zm.x - Zm.y);
        o2 = Zc;
      }
    }
    hb[(unsigned)sidx<TILE>(m, qq, M)] = o1;
    hb[(unsigned)sidx<TILE>(mp, qq, M)] = o2;
  }
  __syncthreads();  // LDS is rewritten by the next item
}

template <int L, bool TILE, bool NT>
__global__ __launch_bounds__((RowCfg<L, true>::THREADS)) void rows_fwd_kernel(
    const double* __restrict__ f, double2* __restrict__ H, int M,
    const double2* __restrict__ twL_, const double2* __restrict__ twN_) {
  using P = Plan<L>;
  using C = RowCfg<L, true>;
  __shared__ double2 lds[C::XR * P::ROWSTRIDE];
  __shared__ TwLds<L> twL;      // W_L (row FFT stages)
  __shared__ TwLds<2 * L> twN;  // W_N (r2c post-processing)
  const int q = threadIdx.x / P::T;
  const int tid = threadIdx.x % P::T;
  double2* buf = lds + q * P::ROWSTRIDE;
  const Range rg = persistent_range(blockIdx.x, gridDim.x, M / C::XR);

  // register double buffer: stage 0 runs on the prefetched rows in place; once its output
  // is in LDS the registers are refilled with the next item while stages 1.. run.  The
  // first item's loads are issued right behind the (older) twiddle-table loads, so the
  // table fill's wait does not serialise them.
  twL.fill(twL_);
  twN.fill(twN_);
  if (rg.count <= 0) return;
  double2 nxt[16];
  load_row_z<L, NT>(nxt, f, rg.first * C::XR + q, tid);
  __syncthreads();
  auto item_y0 = [&](int it) { return (rg.first + it * rg.stride) * C::XR; };
  rows_fwd_item<L, TILE, NT>(nxt, lds, buf, f, H, M, item_y0(0),
                             rg.count > 1 ? item_y0(1) : -1, q, tid, twL, twN);
  for (int it = 1; it < rg.count; ++it)
    rows_fwd_item<L, TILE, NT>(nxt, lds, buf, f, H, M, item_y0(it),
                               it + 1 < rg.count ? item_y0(it + 1) : -1, q, tid, twL, twN);
}

// ---------------------------------------------------------------------------------------
// Pass 2: one column at a time: forward FFT, divide, inverse FFT, in place.
// ---------------------------------------------------------------------------------------
struct DivArgs {
  const double* cx;         // cos(kx[m]), m <= L (global m)
  const double* cy;         // cos(ky[k]), k < M
  const double* cy_mirror;  // cy[(M - k) % M] when the symbol is not even in ky (ny < nx)
  double aa, bb, cc, scale;
  int L;
  int neg;
  int recip;
  int m0;         // global index of this buffer's first column (y-slabs: rank * L/P)
  int rl_log2;    // rows per segment (y-slabs: rows per rank; one GPU: M)
  unsigned seg;   // elements between the segments of one column (y-slabs: (L/P) * rows)
};

// v / d as v * (1/d) (recip_nr: the divide is the column pass's costliest step), for the
// FD symbol and for the Dirichlet (DST-I) multiplier of lid_driven_cavity.jl:17 alike; or
// the Hermitian projection (v/d + v/d2)/2 of a symbol that is not even in ky: what
// real(ifft(...)) keeps of a non-Hermitian quotient (Common.jl:123 with ny < nx).  The
// sign is applied first, as divide_kernel does.
__device__ __forceinline__ double2 sym_apply(double2 v, double d, double d2, double sgn,
                                             bool mirror) {
  const double x = sgn * v.x, y = sgn * v.y;
  const double id = recip_nr(d);
  if (mirror) {
    const double id2 = recip_nr(d2);
    return make_double2(0.5 * (x * id + x * id2), 0.5 * (y * id + y * id2));
  }
  return make_double2(x * id, y * id);
}

// Element k of the packed column: Z = Z[k], Zp = Z[-k].  A = (Z + conj Zp)/2 belongs to the
// kx = eps column, B = (Z - conj Zp)/(2i) to kx = -pi; each is divided by its own symbol
// and the pair re-packed as A' + i B'.
struct DivArgs;
__device__ __forceinline__ double2 packed_divide(double2 Z, double2 Zp, int k, double ax,
                                              double axL, const DivArgs& da, double sgn,
                                              bool mirror);

// Element y of a column: rows are stored in segments of 2^rl_log2 (one per source rank of
// the y-slab all-to-all), `seg` elements apart; on one GPU the column is one segment.
__device__ __forceinline__ unsigned col_off(int y, int rl_log2, unsigned seg) {
  return (unsigned)(y >> rl_log2) * seg + (unsigned)(y & ((1 << rl_log2) - 1));
}

__device__ __forceinline__ double2 packed_divide(double2 Z, double2 Zp, int k, double ax,
                                              double axL, const DivArgs& da, double sgn,
                                              bool mirror) {
  const double2 Zc = cconj(Zp);
  const double2 A = make_double2(0.5 * (Z.x + Zc.x), 0.5 * (Z.y + Zc.y));
  const double2 D = csub(Z, Zc);
  const double2 B = make_double2(0.5 * D.y, -0.5 * D.x);
  const double cyk = da.cy[k];
  const double cym = mirror ? da.cy_mirror[k] : cyk;
  const double d0 = fd_symbol(ax, da.cc, cyk);   // kx = eps column
  const double dL = fd_symbol(axL, da.cc, cyk);  // kx = -pi column
  const double d0m = fd_symbol(ax, da.cc, cym);
  const double dLm = fd_symbol(axL, da.cc, cym);
  const double2 A2 = k == 0 ? make_double2(0.0, 0.0)  // e[1,1] = 0 (Common.jl:118)
                            : sym_apply(A, d0, d0m, sgn, mirror);
  const double2 B2 = sym_apply(B, dL, dLm, sgn, mirror);
  return make_double2((A2.x - B2.y) * da.scale, (A2.y + B2.x) * da.scale);
}

template <int M, int NV>
__device__ __forceinline__ void load_col(double2 (&a)[NV], const double2* __restrict__ col,
                                         int tid, int rl_log2, unsigned seg) {
  constexpr int R0 = Plan<M, NV>::radix(0);
#pragma unroll
  for (int b = 0; b < NV / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r)
      a[b * R0 + r] = col[col_off(in_pos<M, 0, NV>(tid, b, r), rl_log2, seg)];
}

// The column kernel's shape: NV values per thread (M / NV threads per column) and the LDS
// exchange, component-wise (HALF: one double per element) or complex.
#ifndef CFDJ_COLS_NV
#define CFDJ_COLS_NV 16
#endif
#ifndef CFDJ_COLS_HALF
#define CFDJ_COLS_HALF 1
#endif
constexpr int kColsNV = CFDJ_COLS_NV;
constexpr bool kColsHalf = CFDJ_COLS_HALF != 0;

// Stages 0.. of a length-M transform on v; the last stage's outputs stay in v.  The LDS
// buffer may still be read by the previous transform's last stage.
template <int M, int DIR, bool HALF, class TW, int NV>
__device__ __forceinline__ void col_fft(void* lds, double2 (&v)[NV], int tid, const TW& tw) {
  stage_regs<M, 0, DIR>(v, tid, tw);
  if constexpr (HALF) {
    run_stages_half<M, 1, DIR>(static_cast<double*>(lds), v, tid, tw);
  } else {
    __syncthreads();
    lds_write<M, 0>(static_cast<double2*>(lds), v, tid);
    __syncthreads();
    run_stages<M, 1, DIR, false>(static_cast<double2*>(lds), v, tid, tw);
  }
}

// One column: forward FFT, divide, inverse FFT.  PACKED = the column of slot 0, Z =
// FFT_y(X_dc + i X_nyq): split with the partner Z[-k] into the DC and the Nyquist column,
// each divided by its own symbol (kx = eps and kx = -pi), re-packed.  One workgroup in L
// does this and it must not set the kernel's register count: it is a separate instantiation
// of the whole body (no merge of two versions of the registers), its spectrum goes through
// the output column in global memory and a rolled loop over the pairs (k, M - k) transforms
// it in place.
template <int M, bool MIRROR, bool PACKED, int NV, bool HALF>
__device__ __forceinline__ void cols_column(void* lds, const double2* __restrict__ col,
                                            double2* __restrict__ ocol, int m, int tid,
                                            const TwGlobal<M>& twM, const DivArgs& da) {
  using P = Plan<M, NV>;
  const double sgn = da.neg ? -1.0 : 1.0;
  constexpr bool mirror = MIRROR;  // symbol not even in ky (ny < nx): a template flag, so
                                  // the square-grid kernel carries no cy_mirror loads
  double2 a[NV];
  load_col<M>(a, col, tid, da.rl_log2, da.seg);
  col_fft<M, -1, HALF>(lds, a, tid, twM);

  double2 v[NV];
  fwd_to_inv<M>(a, v);  // v[r] = spectrum at k = tid + T*r, natural order
  const double ax = fd_symbol_x(da.aa, da.bb, da.cx[m]);
  // From here on the thread index is an opaque copy that exists only once the forward
  // transform is done: the loads that depend on nothing else (cos(ky) of the divide, the
  // inverse stages' twiddles) would otherwise be hoisted to the top of the kernel and
  // their registers stay live through the whole forward transform (170 -> 144 VGPRs).
  int tk = tid;
  asm volatile("" : "+v"(tk) : "v"(v[NV - 1].x));
  if constexpr (!PACKED) {
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      const int k = tk + P::T * r;
      const double d = fd_symbol(ax, da.cc, da.cy[k]);
      const double d2 = mirror ? fd_symbol(ax, da.cc, da.cy_mirror[k]) : d;
      const double2 q = sym_apply(v[r], d, d2, sgn, mirror);
      v[r] = make_double2(q.x * da.scale, q.y * da.scale);
    }
  } else {
#pragma unroll
    for (int r = 0; r < NV; ++r) ocol[col_off(tid + P::T * r, da.rl_log2, da.seg)] = v[r];
    __syncthreads();  // workgroup-scope release / acquire of the global stores
    const double axL = fd_symbol_x(da.aa, da.bb, da.cx[da.L]);
#pragma unroll 1
    for (int k = tid; k <= M / 2; k += P::T) {
      const int kp = (M - k) & (M - 1);
      double2* pk = ocol + col_off(k, da.rl_log2, da.seg);
      double2* pp = ocol + col_off(kp, da.rl_log2, da.seg);
      const double2 Zk = *pk, Zq = *pp;
      *pk = packed_divide(Zk, Zq, k, ax, axL, da, sgn, mirror);
      if (kp != k) *pp = packed_divide(Zq, Zk, kp, ax, axL, da, sgn, mirror);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NV; ++r) v[r] = ocol[col_off(tid + P::T * r, da.rl_log2, da.seg)];
    __syncthreads();  // every reload precedes the final stores to the same column
  }
  col_fft<M, 1, HALF>(lds, v, tk, twM);
  // last inverse stage: outputs j + r*NS are in natural order -> straight to HBM
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
#pragma unroll
  for (int b = 0; b < NV / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r)
      ocol[col_off(out_pos<M, SL, NV>(tk, b, r), da.rl_log2, da.seg)] = v[b * RL + r];
}

// Wavefronts per SIMD the column kernel is compiled for (its register cap): with 16 values
// per thread one per resident workgroup when a workgroup is 4 wavefronts (M = 4096: LDS
// allows 4, registers 3); with 8 values per thread, 4.
#ifndef CFDJ_COLS_WAVES
#define CFDJ_COLS_WAVES 3
#endif
template <int M>
constexpr int cols_waves() {
  return kColsNV == 8 ? 4 : (Plan<M>::T == 256 && M <= 4096 ? CFDJ_COLS_WAVES : 2);
}

template <int M, bool MIRROR>
__global__ __launch_bounds__((Plan<M, kColsNV>::T))
    __attribute__((amdgpu_waves_per_eu(cols_waves<M>(), cols_waves<M>()))) void cols_kernel(const double2* __restrict__ C,
                                                        double2* __restrict__ Cout,
                                                        const double2* __restrict__ twM_,
                                                        const DivArgs da) {
  // One column per workgroup: not persistent, because the divide's cy[k] loads would queue
  // behind a next-column prefetch (vmcnt is in order).  The workgroups of a CU overlap each
  // other's memory and FFT phases instead, so their number matters: the LDS buffer holds one
  // double per element and the stages exchange real and imaginary parts one after the other
  // (exchange_half), 34 KB at M = 4096 -- three workgroups per CU (the registers' limit)
  // where a complex buffer allows two.
  using P = Plan<M, kColsNV>;
  static_assert(P::NSTAGES >= 2, "column length");
  __shared__ double2 lds[kColsHalf ? (P::PAD + 1) / 2 : P::PAD];
  const TwGlobal<M> twM{twM_};
  const int tid = threadIdx.x;
  const int ml = xcd_remap(blockIdx.x, gridDim.x);
  const int m = da.m0 + ml;  // global x-mode
  const double2* col = C + ((size_t)ml << da.rl_log2);
  double2* ocol = Cout + ((size_t)ml << da.rl_log2);
  if (m == 0) {
    cols_column<M, MIRROR, true, kColsNV, kColsHalf>(lds, col, ocol, m, tid, twM, da);
    return;
  }
  cols_column<M, MIRROR, false, kColsNV, kColsHalf>(lds, col, ocol, m, tid, twM, da);
}

// The packed column alone, for the y-slab path (every rank solves the gathered column
// redundantly, on its step's critical path): one workgroup, the whole column in a complex LDS
// buffer, the partner Z[-k] of the packed divide read back from that buffer -- no round trip
// through global memory as in cols_column's packed branch (which must not cost the other 2047
// columns' workgroups any registers).  Element y of the column comes from segment y >> rl_log2
// of `src` (the all-gather's receive layout), the result goes to the dense column `dst`.
template <int M>
__global__ __launch_bounds__((Plan<M>::T)) void col0_solve_kernel(
    const double2* __restrict__ src, size_t seg_stride, int rl_log2, double2* __restrict__ dst,
    const double2* __restrict__ twM_, const DivArgs da) {
  using P = Plan<M>;
  __shared__ double2 lds[P::PAD];
  const TwGlobal<M> twM{twM_};
  const int tid = threadIdx.x;
  const double sgn = da.neg ? -1.0 : 1.0;
  double2 a[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int y = in_pos<M, 0>(tid, b, r);
      a[b * R0 + r] = src[(size_t)(y >> rl_log2) * seg_stride + (y & ((1 << rl_log2) - 1))];
    }
  col_fft<M, -1, false>(lds, a, tid, twM);
  double2 v[16];
  fwd_to_inv<M>(a, v);  // v[r] = Z[k], k = tid + T r
  __syncthreads();       // the forward transform's last LDS reads
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[padx(tid + P::T * r)] = v[r];
  __syncthreads();
  const double ax = fd_symbol_x(da.aa, da.bb, da.cx[0]);
  const double axL = fd_symbol_x(da.aa, da.bb, da.cx[da.L]);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int k = tid + P::T * r;
    const double2 Zp = lds[padx((M - k) & (M - 1))];
    v[r] = packed_divide(v[r], Zp, k, ax, axL, da, sgn, false);
  }
  col_fft<M, 1, false>(lds, v, tid, twM);  // (its first LDS write is behind a barrier)
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) dst[out_pos<M, SL>(tid, b, r)] = v[b * RL + r];
}

// The same solve as two workgroups, one per real column (c = 0: the kx = eps column, the real
// parts of the packed column; c = 1: kx = -pi, the imaginary parts): a real transform of
// length M as a complex one of length H = M/2 on z[j] = x[2j] + i x[2j+1],
//   X[k] = E + W_M^k O,  X[H-k] = conj(E - W_M^k O),
//   E = (Z[k] + conj Z[H-k]) / 2,  O = (Z[k] - conj Z[H-k]) / (2i),
// both divided by the column's own symbol, and back through
//   Z'[k] = (Y[k] + conj Y[H-k]) + i conj(W_M^k) (Y[k] - conj Y[H-k]),
// whose inverse transform of length H is y[2j] + i y[2j+1] of the length-M inverse.  Half
// the transform length per workgroup, on two CUs: this kernel sits alone on every rank's
// critical path between the all-gather and the row pass.
template <int H>
struct TwEvery2nd {  // W_H^e out of the table of W_2H
  const double2* __restrict__ t;
  __device__ __forceinline__ double2 w(int e) const { return t[2 * e]; }
};
#ifndef CFDJ_COL0_SPLIT
#define CFDJ_COL0_SPLIT 1
#endif
template <int M>
__global__ __launch_bounds__((Plan<M / 2>::T)) void col0_split_kernel(
    const double2* __restrict__ src, size_t seg_stride, int rl_log2, double2* __restrict__ dst,
    const double2* __restrict__ twM_, const DivArgs da, const double2* __restrict__ cs_src,
    int cs_ranks, double2* __restrict__ csT) {
  constexpr int H = M / 2;
  using P = Plan<H>;
  __shared__ double2 lds[P::PAD];
  const TwEvery2nd<H> twH{twM_};
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const double sgn = da.neg ? -1.0 : 1.0;
  double2 a[16];
  constexpr int R0 = P::radix(0);
  if (c == 2) {
    // third workgroup (square grids: rows are as long as columns): the ranks' column-sum rows
    // added up, rank 0 first, and the sum's half spectrum X[1 .. H-1] -- the same real
    // transform, forward only
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = make_double2(0.0, 0.0);
#pragma unroll 1
    for (int q = 0; q < cs_ranks; ++q) {
      const double2* z = cs_src + (size_t)q * seg_stride;
#pragma unroll
      for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
        for (int r = 0; r < R0; ++r) a[b * R0 + r] = cadd(a[b * R0 + r], z[in_pos<H, 0>(tid, b, r)]);
    }
    col_fft<H, -1, false>(lds, a, tid, twH);
    double2 v[16];
    fwd_to_inv<H>(a, v);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[padx(tid + P::T * r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = tid + P::T * r;
      const double2 Zc = cconj(lds[padx((H - k) & (H - 1))]);
      const double2 E = make_double2(0.5 * (v[r].x + Zc.x), 0.5 * (v[r].y + Zc.y));
      const double2 D = csub(v[r], Zc);
      csT[k] = cadd(E, cmul(twM_[k], make_double2(0.5 * D.y, -0.5 * D.x)));
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int y = 2 * in_pos<H, 0>(tid, b, r);  // (y and y + 1 share a segment)
      const double* e = reinterpret_cast<const double*>(
          src + (size_t)(y >> rl_log2) * seg_stride + (y & ((1 << rl_log2) - 1)));
      a[b * R0 + r] = make_double2(e[c], e[2 + c]);
    }
  col_fft<H, -1, false>(lds, a, tid, twH);
  double2 v[16];
  fwd_to_inv<H>(a, v);  // v[r] = Z[k], k = tid + T r
  __syncthreads();       // the forward transform's last LDS reads
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[padx(tid + P::T * r)] = v[r];
  __syncthreads();
  const double ax = fd_symbol_x(da.aa, da.bb, da.cx[c ? da.L : 0]);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int k = tid + P::T * r;
    const double2 Zc = cconj(lds[padx((H - k) & (H - 1))]);
    const double2 w = twM_[k];
    const double2 E = make_double2(0.5 * (v[r].x + Zc.x), 0.5 * (v[r].y + Zc.y));
    const double2 D = csub(v[r], Zc);
    const double2 Q = cmul(w, make_double2(0.5 * D.y, -0.5 * D.x));
    const double dk = fd_symbol(ax, da.cc, da.cy[k]);
    const double dp = fd_symbol(ax, da.cc, da.cy[H - k]);
    double2 Yk = sym_apply(cadd(E, Q), dk, dk, sgn, false);
    const double2 Yp = sym_apply(csub(E, Q), dp, dp, sgn, false);  // conj Y[H-k]
    if (c == 0 && k == 0) Yk = make_double2(0.0, 0.0);              // e[1,1] = 0 (Common.jl:118)
    const double2 S = cadd(Yk, Yp), U = cmul(cconj(w), csub(Yk, Yp));
    v[r] = make_double2((S.x - U.y) * da.scale, (S.y + U.x) * da.scale);
  }
  col_fft<H, 1, false>(lds, v, tid, twH);  // (its first LDS write is behind a barrier)
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  double* out = reinterpret_cast<double*>(dst) + c;
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) {
      const int j = out_pos<H, SL>(tid, b, r);
      out[4 * j] = v[b * RL + r].x;
      out[4 * j + 2] = v[b * RL + r].y;
    }
}

// ---------------------------------------------------------------------------------------
// Pass 3: rows, packed half spectrum -> real (c2r).
// ---------------------------------------------------------------------------------------
// One pair (m, L-m) per slot: Z[m] = (X[m] + conj X[L-m]) + i W_N^{-m} (X[m] - conj X[L-m]),
// Z[L-m] = conj of the same expression with m and L-m swapped.
template <int L>
struct InvLoads {
  double2 xm[RowCfg<L, false>::PAIRS], xp[RowCfg<L, false>::PAIRS];
  double2 xh;  // X[L/2] for the thread that owns m = 0
};
template <int L, bool TILE>
__device__ __forceinline__ void load_inv(InvLoads<L>& ld, const double2* __restrict__ H, int M,
                                         int y0) {
  using C = RowCfg<L, false>;
  // uniform row offset in the base pointer, 32-bit per-lane offsets (sidx(m, y0 + qq) =
  // sidx(m, qq) + sidx(0, y0) in both layouts)
  const double2* base = H + sidx<TILE>(0, __builtin_amdgcn_readfirstlane(y0), M);
  // the lane offsets are recomputed at every call from an opaque copy of the thread index:
  // hoisted out of the item loop they were 16 64-bit addresses, spilled to scratch and
  // reloaded between the prefetch loads (each reload waiting behind the earlier loads)
  int tx = threadIdx.x;
  asm volatile("" : "+v"(tx));
#pragma unroll
  for (int i = 0; i < C::PAIRS; ++i) {
    int qq, m;
    pair_index<L, false>(tx + i * C::THREADS, qq, m);
    ld.xm[i] = base[(unsigned)sidx<TILE>(m, qq, M)];
    ld.xp[i] = base[(unsigned)sidx<TILE>((L - m) & (L - 1), qq, M)];  // m = 0: unused
    // m = 0 occurs in pair 0 only (later pairs start at m >= 16); every lane loads, the
    // others a second copy of X[m] that is never used: 17 unconditional loads per item
    if (i == 0) ld.xh = base[(unsigned)sidx<TILE>(m == 0 ? L / 2 : m, qq, M)];
  }
}

// One work item (XR rows) of the inverse row pass: c2r pre-processing of the prefetched
// spectrum pairs into LDS, refill of `nxt` with the next item (next_y0 >= 0), inverse FFT,
// real rows out.  Branch-free with 17 loads and 16 stores per thread, first item peeled by
// the kernel: see rows_fwd_item for why (counted vmcnt at the top of an item).
template <int L, bool TILE>
__device__ __forceinline__ void rows_inv_item(InvLoads<L>& nxt, double2* lds, double2* buf,
                                              const double2* __restrict__ H,
                                              double* __restrict__ f, int M, int y0,
                                              int next_y0, int q, int tid,
                                              const TwLds<L>& twL, const TwLds<2 * L>& twN) {
  using P = Plan<L>;
  using C = RowCfg<L, false>;
#pragma unroll
  for (int i = 0; i < C::PAIRS; ++i) {
    int qq, m;
    pair_index<L, false>(threadIdx.x + i * C::THREADS, qq, m);
    const bool z0 = i == 0 && m == 0;
    double2* bq = lds + qq * P::ROWSTRIDE;
    const double2 Xm = nxt.xm[i];
    const double2 Xp = cconj(nxt.xp[i]);  // conj X[L-m]
    const double2 S = cadd(Xm, Xp);
    const double2 D = cmul(cconj(twN.w(m)), csub(Xm, Xp));
    double2 o1 = make_double2(S.x - D.y, S.y + D.x);
    // Z[L-m] = S' + i D' with S' = conj(S), D' = W^{-(L-m)} (X[L-m] - conj X[m]) = conj(D)
    double2 o2 = make_double2(S.x + D.y, D.x - S.y);
    if (i == 0) {
      if (z0) {  // slot 0 = (X[0], X[L]), both real; Z[L/2] = 2 conj(X[L/2])
        o1 = make_double2(Xm.x + Xm.y, Xm.x - Xm.y);
        o2 = make_double2(2.0 * nxt.xh.x, -2.0 * nxt.xh.y);
      }
    }
    bq[padx(m)] = o1;
    bq[padx(z0 ? L / 2 : L - m)] = o2;
  }
  if (next_y0 >= 0) load_inv<L, TILE>(nxt, H, M, next_y0);
  __syncthreads();

  double2 v[16];
  run_stages<L, 0, 1, false>(buf, v, tid, twL);
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  double2* z = reinterpret_cast<double2*>(f + (size_t)(y0 + q) * (2 * L));
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) z[out_pos<L, SL>(tid, b, r)] = v[b * RL + r];
  __syncthreads();  // LDS is rewritten by the next item
}

template <int L, bool TILE>
__global__ __launch_bounds__((RowCfg<L, false>::THREADS)) void rows_inv_kernel(
    const double2* __restrict__ H, double* __restrict__ f, int M,
    const double2* __restrict__ twL_, const double2* __restrict__ twN_) {
  using P = Plan<L>;
  using C = RowCfg<L, false>;
  __shared__ double2 lds[C::XR * P::ROWSTRIDE];
  __shared__ TwLds<L> twL;
  __shared__ TwLds<2 * L> twN;
  const int q = threadIdx.x / P::T;
  const int tid = threadIdx.x % P::T;
  double2* buf = lds + q * P::ROWSTRIDE;
  const Range rg = persistent_range(blockIdx.x, gridDim.x, M / C::XR);

  // register double buffer: the prefetched spectrum pairs are consumed into LDS, then the
  // registers are refilled with the next item while the FFT runs.
  twL.fill(twL_);
  twN.fill(twN_);
  if (rg.count <= 0) return;
  InvLoads<L> nxt;
  load_inv<L, TILE>(nxt, H, M, rg.first * C::XR);
  __syncthreads();
  auto item_y0 = [&](int it) { return (rg.first + it * rg.stride) * C::XR; };
  rows_inv_item<L, TILE>(nxt, lds, buf, H, f, M, item_y0(0), rg.count > 1 ? item_y0(1) : -1, q,
                         tid, twL, twN);
  for (int it = 1; it < rg.count; ++it)
    rows_inv_item<L, TILE>(nxt, lds, buf, H, f, M, item_y0(it),
                           it + 1 < rg.count ? item_y0(it + 1) : -1, q, tid, twL, twN);
}

// The inverse row pass of the one-GPU column-major spectrum for rows of up to 4096 reals:
// ONE small item (XR rows: 2 at L = 2048, 256 threads) per workgroup, not persistent, the
// LDS buffer component-wise (35 KB), 128 registers -- four workgroups per CU overlap each
// other's loads, transforms and stores, which a single persistent workgroup with its next
// item prefetched into registers does less well (59 -> 49 us per launch in the step at
// 4096^2).  The c2r pre-processing of a pair (m, L - m) is formed in registers and goes
// through the buffer one component at a time, straight into stage 0's input order.
// CFDJ_ROWS_INV_NP=0 builds without it (the persistent kernel everywhere).  The forward
// pass keeps the persistent 4-row items: its column-segment WRITES would shrink to 32 B
// with 2-row items, which measured slower (85 us in the step).
#ifndef CFDJ_ROWS_INV_NP_CM_MAXL
#define CFDJ_ROWS_INV_NP_CM_MAXL 2048  // column-major layout: longest half row it takes
#endif
#ifndef CFDJ_ROWS_INV_NP
#define CFDJ_ROWS_INV_NP 1
#endif
// Rows per item: 256 threads' worth, at least 2 in the column-major layout (32-B column
// segments); in the 8-mode-tile layout of the y-slab path a single row is whole 128-B lines.
#ifndef CFDJ_ROWS_NP_XR_MIN
#define CFDJ_ROWS_NP_XR_MIN 2
#endif
// Minimum wavefronts per SIMD the small-item row kernels are compiled for (1: no constraint).
// Rows of 8192 complex points are 512-thread workgroups, two wavefronts per SIMD each: a
// second workgroup per CU needs the kernel within 128 registers.  With eight loaded twiddles
// of the radix-2 last stage held across the exchange they wanted 142-154 and the cap spilled
// 19-33 (158-162 us per pass at 16384 x 2048 against 147-148 uncapped); with that stage's
// twiddles formed from one table value (fft_lds.hpp: lazy_last) they fit without spills.
#ifndef CFDJ_ROWS_NP_WAVES_8192
#define CFDJ_ROWS_NP_WAVES_8192 4
#endif
// Rows of 4096 complex points (256-thread workgroups, 35 KB of LDS: four per CU): the forward
// kernel of the y-slab path wants 138 registers, three workgroups per CU; capped at 128 it
// spills one and runs 8192 x 1024 (1152 workgroups: one round and an eighth instead of one and
// a half) in 25.8 us instead of 30.7, 8192 x 2048 unchanged.
#ifndef CFDJ_ROWS_NP_WAVES_4096
#define CFDJ_ROWS_NP_WAVES_4096 4
#endif
// (rows of 512 complex points, eight per 256-thread workgroup: the inverse kernel is at 129)
#ifndef CFDJ_ROWS_NP_WAVES_512
#define CFDJ_ROWS_NP_WAVES_512 4
#endif
template <int L>
constexpr int rows_np_waves() {
  return L >= 8192 ? CFDJ_ROWS_NP_WAVES_8192 : L == 4096 ? CFDJ_ROWS_NP_WAVES_4096 :
         L == 512 ? CFDJ_ROWS_NP_WAVES_512 : 1;
}

template <int L, bool TILE>
constexpr int rows_np_xr() {
  constexpr int byT = 256 / Plan<L>::T;
  return TILE ? (byT > 1 ? byT : 1) : (byT > CFDJ_ROWS_NP_XR_MIN ? byT : CFDJ_ROWS_NP_XR_MIN);
}

// BAND: the spectrum is zero in the columns above `mmax` (the spectral solvers' 2/3 rule):
// they are not read.
// NTS: the real rows by streaming stores.  psi (134 MB at 4096^2) is the next kernel's input,
// but written the plain way its dirty lines sit in the caches while that kernel streams four
// other arrays through them: stage kernels 87 -> 83 us, this pass 49 -> 47 (0.742 -> 0.727 ms
// per step).  Chosen like the streaming loads: only where the fields outgrow the caches.
// COL0 (y-slab path): the packed column 0 comes from the dense array col0[row] (where the
// gathered column's solve leaves it) instead of the spectrum; and, where hx.H is set, the
// workgroups beyond the slab's rows transform the first two rows of that 8-row tiled spectrum
// (psi-hat of the rows just outside the slab, from the substructured solve) into the slab's
// two halo rows hx.lo / hx.hi, their packed column 0 from hx.c0lo / hx.c0hi.
struct HaloRows {
  const double2* H;
  double* lo;
  double* hi;
  const double2* c0lo;
  const double2* c0hi;
};
template <int L, int XR, bool TILE, bool BAND = false, bool NTS = false, bool COL0 = false>
__global__ __launch_bounds__(XR* Plan<L>::T)
    __attribute__((amdgpu_waves_per_eu(rows_np_waves<L>()))) void rows_inv_np_kernel(
    const double2* __restrict__ H, double* __restrict__ f, int M,
    const double2* __restrict__ twL_, const double2* __restrict__ twN_, int mmax,
    const double2* __restrict__ col0, const HaloRows hx) {
  using P = Plan<L>;
  constexpr int THREADS = XR * P::T, PAIRS = (L / 2) * XR / THREADS;
  __shared__ double lds[XR * P::PAD];
  const TwGlobal<L> twL{twL_};
  const TwGlobal<2 * L> twN{twN_};
  const int q = threadIdx.x / P::T, tid = threadIdx.x % P::T;
  double* buf = lds + q * P::PAD;
  int y0 = xcd_remap(blockIdx.x, gridDim.x) * XR;
  bool extra = false;
  if constexpr (COL0) {
    if (y0 >= M) {  // the blocks whose index the (bijective) remap puts beyond the rows
      extra = true;
      y0 -= M;
      H = hx.H;
      M = 8;
    }
  }
  const double2* base = H + sidx<TILE>(0, __builtin_amdgcn_readfirstlane(y0), M);
  double2 o1[PAIRS], o2[PAIRS];
  // pair i of the thread: row qq, columns m and L - m (16 consecutive lanes take 16
  // consecutive m of one row; m = 0, with partner L/2, occurs in pair 0 only)
  auto pair = [](int i, int& qq, int& m) {
    const int e = threadIdx.x + i * THREADS;
    qq = (e >> 4) % XR;
    m = ((e >> 4) / XR) * 16 + (e & 15);
  };
#pragma unroll
  for (int i = 0; i < PAIRS; ++i) {
    int qq, m;
    pair(i, qq, m);
    const bool z0 = i == 0 && m == 0;
    const int mq = z0 ? L / 2 : L - m;
    double2 Xm = make_double2(0.0, 0.0), Xq = Xm;
    if (!BAND || m <= mmax) Xm = base[(unsigned)sidx<TILE>(m, qq, M)];
    if (!BAND || mq <= mmax) Xq = base[(unsigned)sidx<TILE>(mq, qq, M)];
    if constexpr (COL0)
      if (z0) Xm = !extra ? col0[y0 + qq] : (y0 + qq == 0 ? *hx.c0lo : *hx.c0hi);
    const double2 Xp = cconj(Xq);
    const double2 S = cadd(Xm, Xp);
    const double2 D = cmul(cconj(twN.w(m)), csub(Xm, Xp));
    o1[i] = make_double2(S.x - D.y, S.y + D.x);
    o2[i] = make_double2(S.x + D.y, D.x - S.y);
    if (z0) {  // slot 0 = (X[0], X[L]), both real; Z[L/2] = 2 conj(X[L/2])
      o1[i] = make_double2(Xm.x + Xm.y, Xm.x - Xm.y);
      o2[i] = make_double2(2.0 * Xq.x, -2.0 * Xq.y);
    }
  }
  double2 v[16];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c) __syncthreads();
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      int qq, m;
      pair(i, qq, m);
      double* bq = lds + qq * P::PAD;
      bq[padx(m)] = c ? o1[i].y : o1[i].x;
      bq[padx(i == 0 && m == 0 ? L / 2 : L - m)] = c ? o2[i].y : o2[i].x;
    }
    __syncthreads();
    if (c) lds_read_half<L, 0, 1>(buf, v, tid);
    else lds_read_half<L, 0, 0>(buf, v, tid);
  }
  stage_regs<L, 0, 1>(v, tid, twL);
  run_stages_half<L, 1, 1>(buf, v, tid, twL);
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  double2* z = reinterpret_cast<double2*>(f + (size_t)(y0 + q) * (2 * L));
  if constexpr (COL0) {
    if (extra) {  // rows 0 and 1 of the extra spectrum are the halo rows; the rest is padding
      if (y0 + q > 1) return;
      z = reinterpret_cast<double2*>(y0 + q == 0 ? hx.lo : hx.hi);
    }
  }
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) store_stream<NTS>(z + out_pos<L, SL>(tid, b, r), v[b * RL + r]);
}

// The forward row pass in the same shape (one small item per workgroup, component-wise LDS,
// four workgroups per CU), used with the 8-mode-tile layout of the y-slab path, where one
// row's modes are whole 128-B lines; in the column-major layout a small item's column
// segments are too short to write (see above) and the persistent kernel stays.
// COL0 (y-slab path): the packed column 0 goes to the dense array col0[row] as well, the
// send buffer of that column's all-gather; and one workgroup beyond the slab's rows transforms
// the first XR rows of the 8-row array fx (the slab's column-sum row and zeros) into the
// 8-row tiled spectrum Hx, which would otherwise be a launch of its own between two others.
template <int L, int XR, bool TILE, bool NT, bool COL0 = false>
__global__ __launch_bounds__(XR* Plan<L>::T)
    __attribute__((amdgpu_waves_per_eu(rows_np_waves<L>()))) void rows_fwd_np_kernel(
    const double* __restrict__ f, double2* __restrict__ H, int M,
    const double2* __restrict__ twL_, const double2* __restrict__ twN_,
    double2* __restrict__ col0, const double* __restrict__ fx, double2* __restrict__ Hx,
    double2* __restrict__ wrows, const double* __restrict__ cp, int ncp,
    double* __restrict__ csout) {
  using P = Plan<L>;
  constexpr int THREADS = XR * P::T, PAIRS = (L / 2) * XR / THREADS;
  __shared__ double lds[XR * P::PAD];
  const TwGlobal<L> twL{twL_};
  const TwGlobal<2 * L> twN{twN_};
  const int q = threadIdx.x / P::T, tid = threadIdx.x % P::T;
  double* buf = lds + q * P::PAD;
  int bid = blockIdx.x, nbl = gridDim.x;
  if constexpr (COL0 && THREADS >= 256) {
    if (cp != nullptr) {
      // the first 2L/64 workgroups (dispatched first: their chain of load round trips runs
      // beside the row items instead of after them): 64 columns each of the field's
      // column-sum partial rows added up -- no transform, the sums travel with the
      // all-gather; as a launch of its own this costs 5 us on the step
      constexpr int NCS = (2 * L + 63) / 64;
      if (bid < NCS) {
        const int x0 = bid * 64;
        const double t = colsum_block(cp, ncp, 2 * L, x0, reinterpret_cast<double(*)[64]>(lds));
        if (threadIdx.x < 64 && x0 + (int)threadIdx.x < 2 * L) csout[x0 + threadIdx.x] = t;
        return;
      }
      bid -= NCS;
      nbl -= NCS;
    }
  }
  int y0 = xcd_remap(bid, nbl) * XR;
  bool extra = false;
  if constexpr (COL0) {
    if (y0 >= M) {  // the one block whose index the (bijective) remap puts beyond the rows
      extra = true;
      f = fx;
      H = Hx;
      M = 8;
      y0 = 0;
    }
  }
  double2 v[16];
  {
    const double2* z = reinterpret_cast<const double2*>(f) + (size_t)(y0 + q) * L;
    constexpr int R0 = P::radix(0);
#pragma unroll
    for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
      for (int r = 0; r < R0; ++r)
        v[b * R0 + r] = load_stream<NT>(z + (unsigned)in_pos<L, 0>(tid, b, r));
    // COL0 with wrows: the slab's first and last rows also go, as they are, to wrows[0 .. L)
    // and wrows[L .. 2L) -- the neighbours' halo rows of this field, sent with the gather
    if constexpr (COL0) {
      if (wrows != nullptr && !extra && (y0 + q == 0 || y0 + q == M - 1)) {
        double2* wr = wrows + (y0 + q == 0 ? 0 : L);
#pragma unroll
        for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
          for (int r = 0; r < R0; ++r) wr[in_pos<L, 0>(tid, b, r)] = v[b * R0 + r];
      }
    }
  }
  stage_regs<L, 0, -1>(v, tid, twL);
  run_stages_half<L, 1, -1>(buf, v, tid, twL);
  // the transform's outputs, in natural order, through the buffer one component at a time;
  // pair i of the thread: row qq, columns m and L - m (m = 0 pairs with L/2, pair 0 only)
  constexpr int SL = P::NSTAGES - 1;
  auto pair = [](int i, int& qq, int& m) {
    const int e = threadIdx.x + i * THREADS;
    qq = (e >> 4) % XR;
    m = ((e >> 4) / XR) * 16 + (e & 15);
  };
  double2 Zm[PAIRS], Zp[PAIRS];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();
    if (c) lds_write_half<L, SL, 1>(buf, v, tid);
    else lds_write_half<L, SL, 0>(buf, v, tid);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      int qq, m;
      pair(i, qq, m);
      const double* bq = lds + qq * P::PAD;
      const double a = bq[padx(m)], b = bq[padx(i == 0 && m == 0 ? L / 2 : L - m)];
      if (c) {
        Zm[i].y = a;
        Zp[i].y = b;
      } else {
        Zm[i].x = a;
        Zp[i].x = b;
      }
    }
  }
  double2* hb = H + sidx<TILE>(0, __builtin_amdgcn_readfirstlane(y0), M);
#pragma unroll
  for (int i = 0; i < PAIRS; ++i) {
    int qq, m;
    pair(i, qq, m);
    const bool z0 = i == 0 && m == 0;
    const int mp = z0 ? L / 2 : L - m;
    const double2 Zc = cconj(Zp[i]);
    const double2 E = make_double2(0.5 * (Zm[i].x + Zc.x), 0.5 * (Zm[i].y + Zc.y));
    const double2 D = csub(Zm[i], Zc);                      // = 2i O[m]
    const double2 O = make_double2(0.5 * D.y, -0.5 * D.x);  // D / (2i)
    const double2 WO = cmul(twN.w(m), O);
    double2 o1 = cadd(E, WO);
    double2 o2 = cconj(csub(E, WO));
    if (z0) {  // slot 0 = X[0] + i X[L]; X[L/2] = conj(Z[L/2])
      o1 = make_double2(Zm[i].x + Zm[i].y, Zm[i].x - Zm[i].y);
      o2 = Zc;
      if constexpr (COL0)
        if (!extra) col0[y0 + qq] = o1;
    }
    hb[(unsigned)sidx<TILE>(m, qq, M)] = o1;
    hb[(unsigned)sidx<TILE>(mp, qq, M)] = o2;
  }
}

// The 2/3-rule solver's product rows (pseudospectral_23_rule.jl:134-140): the inverse row pass
// of the fourth derivative field (band-limited half spectrum H4, column-major), the product
// j1 j2 - j3 j4 with the three fields already in physical space (R: three arrays of M rows of
// 2L reals), and the product's forward row pass (-> Hout, column-major packed half spectrum)
// in one kernel: the fourth field and the product never reach HBM.  The inverse transform's
// last stage leaves a thread the elements the forward transform's stage 0 reads (fwd_to_inv),
// so the product is formed in registers with no exchange between the transforms.  Each factor
// is scaled by inv_np = 1 / (nx ny) first, as the reference's ifft does.
template <int L, int XR, bool NT>
__global__ __launch_bounds__(XR* Plan<L>::T) void rows_jac_np_kernel(
    const double2* __restrict__ H4, const double* __restrict__ R, double2* __restrict__ Hout,
    int M, const double2* __restrict__ twL_, const double2* __restrict__ twN_, int mmax,
    double inv_np) {
  using P = Plan<L>;
  constexpr int THREADS = XR * P::T, PAIRS = (L / 2) * XR / THREADS;
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  __shared__ double lds[XR * P::PAD];
  const TwGlobal<L> twL{twL_};
  const TwGlobal<2 * L> twN{twN_};
  const int y0 = xcd_remap(blockIdx.x, gridDim.x) * XR;
  double2 v[16];
  {  // ---- c2r of rows y0 .. y0 + XR - 1 of H4 (rows_inv_np_kernel's steps)
    const int tx = threadIdx.x;
    const int q = tx / P::T, tid = tx % P::T;
    double* buf = lds + q * P::PAD;
    const double2* base = H4 + __builtin_amdgcn_readfirstlane(y0);
    double2 o1[PAIRS], o2[PAIRS];
    auto pair = [tx](int i, int& qq, int& m) {
      const int e = tx + i * THREADS;
      qq = (e >> 4) % XR;
      m = ((e >> 4) / XR) * 16 + (e & 15);
    };
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      int qq, m;
      pair(i, qq, m);
      const bool z0 = i == 0 && m == 0;
      const int mq = z0 ? L / 2 : L - m;
      double2 Xm = make_double2(0.0, 0.0), Xq = Xm;
      if (m <= mmax) Xm = base[(unsigned)(m * M + qq)];
      if (mq <= mmax) Xq = base[(unsigned)(mq * M + qq)];
      const double2 Xp = cconj(Xq);
      const double2 S = cadd(Xm, Xp);
      const double2 D = cmul(cconj(twN.w(m)), csub(Xm, Xp));
      o1[i] = make_double2(S.x - D.y, S.y + D.x);
      o2[i] = make_double2(S.x + D.y, D.x - S.y);
      if (z0) {  // slot 0 = (X[0], X[L]), both real; Z[L/2] = 2 conj(X[L/2])
        o1[i] = make_double2(Xm.x + Xm.y, Xm.x - Xm.y);
        o2[i] = make_double2(2.0 * Xq.x, -2.0 * Xq.y);
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (c) __syncthreads();
#pragma unroll
      for (int i = 0; i < PAIRS; ++i) {
        int qq, m;
        pair(i, qq, m);
        double* bq = lds + qq * P::PAD;
        bq[padx(m)] = c ? o1[i].y : o1[i].x;
        bq[padx(i == 0 && m == 0 ? L / 2 : L - m)] = c ? o2[i].y : o2[i].x;
      }
      __syncthreads();
      if (c) lds_read_half<L, 0, 1>(buf, v, tid);
      else lds_read_half<L, 0, 0>(buf, v, tid);
    }
    stage_regs<L, 0, 1>(v, tid, twL);
    run_stages_half<L, 1, 1>(buf, v, tid, twL);
  }
  // Each phase works from its own opaque copy of the thread index: what depends only on it
  // (pair offsets, buffer addresses, twiddles) is formed again where it is used instead of
  // staying in registers from one transform to the other; the product's loads stay behind
  // the inverse transform.
  __builtin_amdgcn_sched_barrier(0);
  int tx = threadIdx.x;
  asm volatile("" : "+v"(tx));
  {  // ---- product: v = (f1 inv)(f2 inv) - (f3 inv)(v inv) at the thread's elements
    const int q = tx / P::T, tid = tx % P::T;
    const size_t full = (size_t)M * L;  // complex elements per real array
    const double2* r1 = reinterpret_cast<const double2*>(R) +
                        (size_t)__builtin_amdgcn_readfirstlane(y0) * L;
    const double2* r2 = r1 + full;
    const double2* r3 = r2 + full;
#pragma unroll
    for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
      for (int r = 0; r < RL; ++r) {
        const unsigned off = (unsigned)(q * L + out_pos<L, SL>(tid, b, r));
        const double2 f1 = load_stream<NT>(r1 + off), f2 = load_stream<NT>(r2 + off);
        const double2 f3 = load_stream<NT>(r3 + off);
        double2& d = v[b * RL + r];
        d.x = (f1.x * inv_np) * (f2.x * inv_np) - (f3.x * inv_np) * (d.x * inv_np);
        d.y = (f1.y * inv_np) * (f2.y * inv_np) - (f3.y * inv_np) * (d.y * inv_np);
        // formed here, not where the next exchange first uses them (their factors would
        // stay in registers until then)
        asm volatile("" : "+v"(d.x), "+v"(d.y));
      }
  }
  __builtin_amdgcn_sched_barrier(0);
  int tx2 = tx;
  asm volatile("" : "+v"(tx2));
  {  // ---- r2c of the product rows (rows_fwd_np_kernel's steps)
    const int q = tx2 / P::T, tid = tx2 % P::T;
    double* buf = lds + q * P::PAD;
    double2 a[16];
    fwd_to_inv<L>(v, a);  // a[r] = element tid + T r
    stage_regs<L, 0, -1>(a, tid, twL);
    run_stages_half<L, 1, -1>(buf, a, tid, twL);
    auto pair = [tx2](int i, int& qq, int& m) {
      const int e = tx2 + i * THREADS;
      qq = (e >> 4) % XR;
      m = ((e >> 4) / XR) * 16 + (e & 15);
    };
    double2 Zm[PAIRS], Zp[PAIRS];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      __syncthreads();
      if (c) lds_write_half<L, SL, 1>(buf, a, tid);
      else lds_write_half<L, SL, 0>(buf, a, tid);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < PAIRS; ++i) {
        int qq, m;
        pair(i, qq, m);
        const double* bq = lds + qq * P::PAD;
        const double za = bq[padx(m)], zb = bq[padx(i == 0 && m == 0 ? L / 2 : L - m)];
        if (c) {
          Zm[i].y = za;
          Zp[i].y = zb;
        } else {
          Zm[i].x = za;
          Zp[i].x = zb;
        }
      }
    }
    double2* hb = Hout + __builtin_amdgcn_readfirstlane(y0);
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      int qq, m;
      pair(i, qq, m);
      const bool z0 = i == 0 && m == 0;
      const int mp = z0 ? L / 2 : L - m;
      const double2 Zc = cconj(Zp[i]);
      const double2 E = make_double2(0.5 * (Zm[i].x + Zc.x), 0.5 * (Zm[i].y + Zc.y));
      const double2 D = csub(Zm[i], Zc);                      // = 2i O[m]
      const double2 O = make_double2(0.5 * D.y, -0.5 * D.x);  // D / (2i)
      const double2 WO = cmul(twN.w(m), O);
      double2 o1 = cadd(E, WO);
      double2 o2 = cconj(csub(E, WO));
      if (z0) {  // slot 0 = X[0] + i X[L]; X[L/2] = conj(Z[L/2])
        o1 = make_double2(Zm[i].x + Zm[i].y, Zm[i].x - Zm[i].y);
        o2 = Zc;
      }
      hb[(unsigned)(m * M + qq)] = o1;
      hb[(unsigned)(mp * M + qq)] = o2;
    }
  }
}

// Persistent grid: `per_cu` resident workgroups per CU (LDS-limited), a multiple of 8.
static int persistent_grid(int ncu, int per_cu, int items) {
  int nb = ncu * per_cu;
  nb -= nb % 8;
  if (nb < 8) nb = 8;
  return nb < items ? nb : items;
}

template <int L, bool FWD>
void launch_rows_dir(int pass, const FusedPoissonArgs& a, hipStream_t st);

// CFDJ_FWD_NP=2|4|8 (read once): see launch_rows.
static int fwd_np_rows() {
  static const int v = [] {
    const char* e = std::getenv("CFDJ_FWD_NP");
    const int x = e ? std::atoi(e) : 0;
    return x == 2 || x == 4 || x == 8 ? x : 0;
  }();
  return v;
}

template <int L>
void launch_rows(int pass, const FusedPoissonArgs& a, hipStream_t st) {
#if CFDJ_ROWS_INV_NP > 0
  // the small-item kernels: the inverse pass in both layouts, the forward pass in the
  // 8-mode-tile layout; rows of up to 4096 (column-major) / 8192 (tiles) reals
  if constexpr (L <= 8192) {
    if (a.tile8) {
      constexpr int XR = rows_np_xr<L, true>();
      if (a.rows % XR == 0) {
        const dim3 grid(a.rows / XR), block(XR * Plan<L>::T);
        if (pass == 0) {
          if ((a.fx && !(a.col0 && a.Hx)) || (a.wrows && !a.col0))
            throw Error{CFDJ_ERR_ARG, "fused Poisson: extra row without dense column 0"};
          if (a.cp && (a.fx || !a.col0 || !a.csout || a.ncp < 1 || XR * Plan<L>::T < 256))
            throw Error{CFDJ_ERR_ARG, "fused Poisson: column sums unsupported here"};
          const dim3 gridx(a.rows / XR + (a.fx ? 1 : 0) + (a.cp ? (2 * L + 63) / 64 : 0));
          auto fwd = [&](auto nt, auto c0) {
            hipLaunchKernelGGL((rows_fwd_np_kernel<L, XR, true, nt.value, c0.value>), gridx, block,
                               0, st, a.f, a.H, a.rows, a.twL, a.twN, a.col0, a.fx, a.Hx, a.wrows,
                               a.cp, a.ncp, a.csout);
          };
          using T = std::true_type;
          using F = std::false_type;
          if (a.stream) a.col0 ? fwd(T{}, T{}) : fwd(T{}, F{});
          else a.col0 ? fwd(F{}, T{}) : fwd(F{}, F{});
        } else {
          if (a.hx_H && !(a.col0 && a.hx_lo && a.hx_hi && a.hx_c0lo && a.hx_c0hi))
            throw Error{CFDJ_ERR_ARG, "fused Poisson: halo rows without dense column 0"};
          const HaloRows hx{a.hx_H, a.hx_lo, a.hx_hi, a.hx_c0lo, a.hx_c0hi};
          const dim3 gridi(a.rows / XR + (a.hx_H ? (2 + XR - 1) / XR : 0));
          auto inv = [&](auto nts, auto c0) {
            hipLaunchKernelGGL((rows_inv_np_kernel<L, XR, true, false, nts.value, c0.value>), gridi,
                               block, 0, st, a.H, a.s, a.rows, a.twL, a.twN, 0, a.col0, hx);
          };
          using T = std::true_type;
          using F = std::false_type;
          if (a.stream_out) a.col0 ? inv(T{}, T{}) : inv(T{}, F{});
          else a.col0 ? inv(F{}, T{}) : inv(F{}, F{});
        }
        return;
      }
    }
  }
  if constexpr (L <= 4096) {
    if (a.tile8) {
      // (taken above)
    } else if (pass == 0 && L <= 2048 && fwd_np_rows() > 0) {
      // A/B switch (CFDJ_FWD_NP=2|4|8): the forward pass in the small-item shape on the
      // column-major layout, XR rows per workgroup (column segments of 16 XR bytes)
      const int xr = fwd_np_rows();
      auto go = [&](auto xrc) {
        constexpr int XR = decltype(xrc)::value;
        if constexpr (XR * Plan<L>::T <= 1024) {
          if (a.rows % XR != 0) throw Error{CFDJ_ERR_ARG, "CFDJ_FWD_NP: rows not a multiple"};
          const dim3 grid(a.rows / XR), block(XR * Plan<L>::T);
          if (a.stream)
            hipLaunchKernelGGL((rows_fwd_np_kernel<L, XR, false, true>), grid, block, 0, st, a.f,
                               a.H, a.rows, a.twL, a.twN, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                               nullptr);
          else
            hipLaunchKernelGGL((rows_fwd_np_kernel<L, XR, false, false>), grid, block, 0, st, a.f,
                               a.H, a.rows, a.twL, a.twN, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                               nullptr);
        } else {
          throw Error{CFDJ_ERR_ARG, "CFDJ_FWD_NP: workgroup too large for this row length"};
        }
      };
      if (xr == 2) go(std::integral_constant<int, 2>{});
      else if (xr == 4) go(std::integral_constant<int, 4>{});
      else go(std::integral_constant<int, 8>{});
      return;
    } else if (pass != 0 && L <= CFDJ_ROWS_INV_NP_CM_MAXL) {
      constexpr int XR = rows_np_xr<L, false>();
      if (a.rows % XR == 0) {
        if (a.mmax > 0)  // (the spectral solvers' batches: plain stores measured as fast)
          hipLaunchKernelGGL((rows_inv_np_kernel<L, XR, false, true>), dim3(a.rows / XR),
                             dim3(XR * Plan<L>::T), 0, st, a.H, a.s, a.rows, a.twL, a.twN,
                             a.mmax, nullptr, HaloRows{});
        else if (a.stream_out)
          hipLaunchKernelGGL((rows_inv_np_kernel<L, XR, false, false, true>), dim3(a.rows / XR),
                             dim3(XR * Plan<L>::T), 0, st, a.H, a.s, a.rows, a.twL, a.twN, 0, nullptr,
                             HaloRows{});
        else
          hipLaunchKernelGGL((rows_inv_np_kernel<L, XR, false>), dim3(a.rows / XR),
                             dim3(XR * Plan<L>::T), 0, st, a.H, a.s, a.rows, a.twL, a.twN, 0, nullptr,
                             HaloRows{});
        return;
      }
    }
  }
#endif
  if (a.col0 || a.fx)
    throw Error{CFDJ_ERR_ARG, "fused Poisson: dense column 0 unsupported here"};
  if (pass == 0) launch_rows_dir<L, true>(pass, a, st);
  else launch_rows_dir<L, false>(pass, a, st);
}

template <int L, bool FWD>
void launch_rows_dir(int pass, const FusedPoissonArgs& a, hipStream_t st) {
  using C = RowCfg<L, FWD>;
  constexpr int row_lds = C::XR * Plan<L>::ROWSTRIDE * 16 + sizeof(TwLds<L>) +
                          sizeof(TwLds<2 * L>);
  const int per_cu = (160 * 1024) / row_lds;
  const dim3 grid(persistent_grid(a.ncu, per_cu, a.rows / C::XR));
  if constexpr (FWD) {
    if (a.tile8 && a.stream)
      hipLaunchKernelGGL((rows_fwd_kernel<L, true, true>), grid, dim3(C::THREADS), 0, st, a.f,
                         a.H, a.rows, a.twL, a.twN);
    else if (a.tile8)
      hipLaunchKernelGGL((rows_fwd_kernel<L, true, false>), grid, dim3(C::THREADS), 0, st, a.f,
                         a.H, a.rows, a.twL, a.twN);
    else if (a.stream)
      hipLaunchKernelGGL((rows_fwd_kernel<L, false, true>), grid, dim3(C::THREADS), 0, st, a.f,
                         a.H, a.rows, a.twL, a.twN);
    else
      hipLaunchKernelGGL((rows_fwd_kernel<L, false, false>), grid, dim3(C::THREADS), 0, st, a.f,
                         a.H, a.rows, a.twL, a.twN);
  } else {
    if (a.tile8)
      hipLaunchKernelGGL((rows_inv_kernel<L, true>), grid, dim3(C::THREADS), 0, st, a.H, a.s,
                         a.rows, a.twL, a.twN);
    else
      hipLaunchKernelGGL((rows_inv_kernel<L, false>), grid, dim3(C::THREADS), 0, st, a.H, a.s,
                         a.rows, a.twL, a.twN);
  }
}

template <int M>
void launch_cols(const FusedPoissonArgs& a, hipStream_t st) {
  DivArgs da{a.cx,  a.cy,  a.cy_mirror,        a.aa, a.bb, a.cc,       a.scale,
             a.nx / 2, a.neg ? 1 : 0, a.recip ? 1 : 0, a.m0, a.rl_log2, a.seg};
  double2* out = a.Cout ? a.Cout : a.C;
  if (a.cy_mirror == nullptr)
    hipLaunchKernelGGL((cols_kernel<M, false>), dim3(a.kb), dim3(Plan<M, kColsNV>::T), 0, st, a.C, out, a.twM, da);
  else
    hipLaunchKernelGGL((cols_kernel<M, true>), dim3(a.kb), dim3(Plan<M, kColsNV>::T), 0, st, a.C, out, a.twM, da);
}

constexpr bool pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

}  // namespace

// Row lengths nx = 1024..16384 (half-length L = 512..8192 in one workgroup's LDS), column
// lengths ny = 1024..8192, powers of two; `rows` (this GPU's rows) a multiple of the row
// pass's rows per work item (<= 8).
bool fused_rows_supported(int nx, int rows) {
  return pow2(nx) && nx >= 1024 && nx <= 16384 && rows >= 8 && rows % 8 == 0;
}

// Whether the row passes of the 8-mode-tile layout take FusedPoissonArgs::col0.
bool fused_rows_take_col0(int nx, int rows) {
  return CFDJ_ROWS_INV_NP > 0 && fused_rows_supported(nx, rows) && nx <= 16384;
}

bool fused_poisson_supported(int nx, int ny, int rows) {
  return pow2(nx) && pow2(ny) && nx >= 1024 && nx <= 16384 && ny >= 1024 && ny <= 8192 &&
         rows >= 8 && rows % 8 == 0 && ny % rows == 0;
}

static bool col0_split_on() {
  static const bool split = [] {
    const char* e = std::getenv("CFDJ_COL0_SPLIT");
    return e ? e[0] != '0' : CFDJ_COL0_SPLIT != 0;
  }();
  return split;
}

// (16384: as two half-length real transforms only -- the whole column does not fit the LDS)
bool col0_solve_supported(int ny) {
  return pow2(ny) && ny >= 1024 && (ny <= 8192 || (ny == 16384 && col0_split_on()));
}

bool col0_solve_takes_colsum(int nx, int ny, int rows) {
  return nx == ny && col0_solve_supported(ny) && col0_split_on() && rows >= 2;
}

bool fused_rows_take_colsum(int nx, int rows) {
  if (!fused_rows_take_col0(nx, rows)) return false;
  switch (nx / 2) {  // the row pass's workgroup: 256 threads
    case 512: return rows_np_xr<512, true>() * Plan<512>::T == 256;
    case 1024: return rows_np_xr<1024, true>() * Plan<1024>::T == 256;
    case 2048: return rows_np_xr<2048, true>() * Plan<2048>::T == 256;
    case 4096: return rows_np_xr<4096, true>() * Plan<4096>::T == 256;
    case 8192: return rows_np_xr<8192, true>() * Plan<8192>::T == 512;
    default: return false;
  }
}

void launch_col0_solve(const FusedPoissonArgs& a, const double2* src, size_t seg_stride,
                       int rows, double2* dst, hipStream_t st, const double2* cs_src,
                       int nranks, double2* csT) {
  if (!col0_solve_supported(a.ny) || rows < 1 || !pow2(rows) || a.ny % rows != 0 ||
      a.cy_mirror != nullptr)
    throw Error{CFDJ_ERR_ARG, "packed column solve: unsupported size"};
  if (cs_src && (!col0_solve_takes_colsum(a.nx, a.ny, rows) || nranks < 1 || !csT))
    throw Error{CFDJ_ERR_ARG, "packed column solve: column sums unsupported here"};
  const DivArgs da{a.cx,  a.cy,  nullptr,           a.aa, a.bb, a.cc,       a.scale,
                   a.nx / 2, a.neg ? 1 : 0, a.recip ? 1 : 0, 0, ilog2(rows), 0u};
  const int rl_log2 = ilog2(rows);
  if (col0_split_on() && rows >= 2) {
    const dim3 g(cs_src ? 3 : 2);
    switch (a.ny) {
      case 1024: hipLaunchKernelGGL((col0_split_kernel<1024>), g, dim3(Plan<512>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da, cs_src, nranks, csT); break;
      case 2048: hipLaunchKernelGGL((col0_split_kernel<2048>), g, dim3(Plan<1024>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da, cs_src, nranks, csT); break;
      case 4096: hipLaunchKernelGGL((col0_split_kernel<4096>), g, dim3(Plan<2048>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da, cs_src, nranks, csT); break;
      case 8192: hipLaunchKernelGGL((col0_split_kernel<8192>), g, dim3(Plan<4096>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da, cs_src, nranks, csT); break;
      default: hipLaunchKernelGGL((col0_split_kernel<16384>), g, dim3(Plan<8192>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da, cs_src, nranks, csT); break;
    }
    CFDJ_HIP(hipGetLastError());
    return;
  }
  switch (a.ny) {
    case 1024: hipLaunchKernelGGL((col0_solve_kernel<1024>), dim3(1), dim3(Plan<1024>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da); break;
    case 2048: hipLaunchKernelGGL((col0_solve_kernel<2048>), dim3(1), dim3(Plan<2048>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da); break;
    case 4096: hipLaunchKernelGGL((col0_solve_kernel<4096>), dim3(1), dim3(Plan<4096>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da); break;
    default: hipLaunchKernelGGL((col0_solve_kernel<8192>), dim3(1), dim3(Plan<8192>::T), 0, st, src, seg_stride, rl_log2, dst, a.twM, da); break;
  }
  CFDJ_HIP(hipGetLastError());
}

bool rows_jac_supported(int nx, int rows) {
  return CFDJ_ROWS_INV_NP > 0 && fused_rows_supported(nx, rows) && nx <= 4096;
}

template <int L>
static void launch_rows_jac_t(const FusedPoissonArgs& a, double inv_np, hipStream_t st) {
  constexpr int XR = 4 * Plan<L>::T <= 1024 ? 4 : 2;
  const dim3 grid(a.rows / XR), block(XR * Plan<L>::T);
  if (a.stream)
    hipLaunchKernelGGL((rows_jac_np_kernel<L, XR, true>), grid, block, 0, st, a.H, a.f, a.C, a.rows,
                       a.twL, a.twN, a.mmax, inv_np);
  else
    hipLaunchKernelGGL((rows_jac_np_kernel<L, XR, false>), grid, block, 0, st, a.H, a.f, a.C, a.rows,
                       a.twL, a.twN, a.mmax, inv_np);
}

// a.H: the fourth field's scratch spectrum (columns 0..a.mmax), a.f: the three real fields,
// a.C: the product's scratch spectrum (must not overlap a.H).
void launch_rows_jac(const FusedPoissonArgs& a, double inv_np, hipStream_t st) {
  if (!rows_jac_supported(a.nx, a.rows) || a.tile8 || a.mmax <= 0 || a.mmax > a.nx / 2 ||
      a.H == nullptr || a.f == nullptr || a.C == nullptr || a.H == a.C)
    throw Error{CFDJ_ERR_ARG, "fused product rows: unsupported arguments"};
  switch (a.nx) {
    case 1024: launch_rows_jac_t<512>(a, inv_np, st); break;
    case 2048: launch_rows_jac_t<1024>(a, inv_np, st); break;
    default: launch_rows_jac_t<2048>(a, inv_np, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_fused_poisson_pass(int pass, const FusedPoissonArgs& a, hipStream_t st) {
  const bool ok = pass == 1 ? !a.tile8 && fused_poisson_supported(a.nx, a.ny, a.rows) && a.kb >= 1 &&
                                 (1 << a.rl_log2) <= a.ny
                           : fused_rows_supported(a.nx, a.rows);
  if (!ok) throw Error{CFDJ_ERR_ARG, "fused Poisson: unsupported size"};
  // the band limit exists in the small-item inverse row kernel only
  if (a.mmax > 0 && !(pass == 2 && !a.tile8 && a.nx <= 4096 && CFDJ_ROWS_INV_NP > 0))
    throw Error{CFDJ_ERR_ARG, "fused Poisson: band limit unsupported here"};
  if (pass == 1) {
    switch (a.ny) {
      case 1024: launch_cols<1024>(a, st); break;
      case 2048: launch_cols<2048>(a, st); break;
      case 4096: launch_cols<4096>(a, st); break;
      case 8192: launch_cols<8192>(a, st); break;
    }
  } else {
    switch (a.nx) {
      case 1024: launch_rows<512>(pass, a, st); break;
      case 2048: launch_rows<1024>(pass, a, st); break;
      case 4096: launch_rows<2048>(pass, a, st); break;
      case 8192: launch_rows<4096>(pass, a, st); break;
      case 16384: launch_rows<8192>(pass, a, st); break;
    }
  }
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
