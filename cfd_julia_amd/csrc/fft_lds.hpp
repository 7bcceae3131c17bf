// Building blocks of the hand-written LDS FFTs (poisson_fft.hip, schur.hip): radix-2/4/8/16
// butterflies in registers, Stockham stage plans over an LDS buffer with one pad per 16
// elements, twiddle sources (LDS 2-level tables or the global long-double table), the FD
// symbol evaluated without FMA, and the XCD-aware persistent work split.
//
// Included after `#pragma clang fp contract(fast)` by the FFT translation units: the FFTs
// are not bit-comparable to FFTW / pocketfft anyway (tolerance 1e-12 relative on psi).
#pragma once
#include "cfdj_internal.hpp"

namespace cfdj {

namespace {

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n / 2); }

// exp(-2 pi i k/16) = (kC16[k], -kS16[k])
__device__ constexpr double kC16[16] = {
    1.0, 0.9238795325112867, 0.7071067811865476, 0.3826834323650898,
    0.0, -0.3826834323650898, -0.7071067811865476, -0.9238795325112867,
    -1.0, -0.9238795325112867, -0.7071067811865476, -0.3826834323650898,
    0.0, 0.3826834323650898, 0.7071067811865476, 0.9238795325112867};
__device__ constexpr double kS16[16] = {
    0.0, 0.3826834323650898, 0.7071067811865476, 0.9238795325112867,
    1.0, 0.9238795325112867, 0.7071067811865476, 0.3826834323650898,
    0.0, -0.3826834323650898, -0.7071067811865476, -0.9238795325112867,
    -1.0, -0.9238795325112867, -0.7071067811865476, -0.3826834323650898};

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }

// v * W16^K (DIR = -1 forward, +1 inverse)
template <int K, int DIR>
__device__ __forceinline__ double2 tw16(double2 v) {
  constexpr int k = K & 15;
  if constexpr (k == 0) {
    return v;
  } else if constexpr (k == 4) {  // -i (fwd) / +i (inv)
    return DIR < 0 ? make_double2(v.y, -v.x) : make_double2(-v.y, v.x);
  } else if constexpr (k == 8) {
    return make_double2(-v.x, -v.y);
  } else if constexpr (k == 12) {
    return DIR < 0 ? make_double2(-v.y, v.x) : make_double2(v.y, -v.x);
  } else {
    constexpr double c = kC16[k];
    constexpr double s = DIR < 0 ? -kS16[k] : kS16[k];
    return make_double2(v.x * c - v.y * s, v.x * s + v.y * c);
  }
}

template <int DIR>
__device__ __forceinline__ void dft2(double2& a, double2& b) {
  const double2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

template <int DIR>
__device__ __forceinline__ void dft4(double2& x0, double2& x1, double2& x2, double2& x3) {
  const double2 s02 = cadd(x0, x2), d02 = csub(x0, x2);
  const double2 s13 = cadd(x1, x3), d13 = tw16<4, DIR>(csub(x1, x3));
  x0 = cadd(s02, s13);
  x2 = csub(s02, s13);
  x1 = cadd(d02, d13);
  x3 = csub(d02, d13);
}

// In-register DFT of length R on v[0..R-1] (natural order in, natural order out).
template <int R, int DIR>
__device__ __forceinline__ void dft(double2* v) {
  if constexpr (R == 2) {
    dft2<DIR>(v[0], v[1]);
  } else if constexpr (R == 4) {
    dft4<DIR>(v[0], v[1], v[2], v[3]);
  } else if constexpr (R == 8) {
    // n = 4 n1 + n2 (n1 < 2, n2 < 4), k = k1 + 2 k2
    double2 a[4][2];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
      a[n2][0] = v[n2];
      a[n2][1] = v[4 + n2];
      dft2<DIR>(a[n2][0], a[n2][1]);
    }
    a[1][1] = tw16<2, DIR>(a[1][1]);
    a[2][1] = tw16<4, DIR>(a[2][1]);
    a[3][1] = tw16<6, DIR>(a[3][1]);
#pragma unroll
    for (int k1 = 0; k1 < 2; ++k1) {
      dft4<DIR>(a[0][k1], a[1][k1], a[2][k1], a[3][k1]);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 2 * k2] = a[k2][k1];
    }
  } else {
    static_assert(R == 16, "radix");
    // n = 4 n1 + n2, k = k1 + 4 k2
    double2 a[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
      a[n2][0] = v[n2];
      a[n2][1] = v[4 + n2];
      a[n2][2] = v[8 + n2];
      a[n2][3] = v[12 + n2];
      dft4<DIR>(a[n2][0], a[n2][1], a[n2][2], a[n2][3]);
    }
    a[1][1] = tw16<1, DIR>(a[1][1]);
    a[1][2] = tw16<2, DIR>(a[1][2]);
    a[1][3] = tw16<3, DIR>(a[1][3]);
    a[2][1] = tw16<2, DIR>(a[2][1]);
    a[2][2] = tw16<4, DIR>(a[2][2]);
    a[2][3] = tw16<6, DIR>(a[2][3]);
    a[3][1] = tw16<3, DIR>(a[3][1]);
    a[3][2] = tw16<6, DIR>(a[3][2]);
    a[3][3] = tw16<9, DIR>(a[3][3]);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      dft4<DIR>(a[0][k1], a[1][k1], a[2][k1], a[3][k1]);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = a[k2][k1];
    }
  }
}

// Stockham plan of a length-L transform with NV values per thread (16, or 8 where more
// wavefronts per transform are wanted): radix-NV stages, then one remainder stage.
template <int L, int NV = 16>
struct Plan {
  static_assert(NV == 16 || NV == 8, "values per thread");
  static constexpr int LOG = ilog2(L);
  static constexpr int LNV = ilog2(NV);
  static constexpr int NFULL = LOG / LNV;
  static constexpr int REM = 1 << (LOG % LNV);
  static constexpr int NSTAGES = NFULL + (REM > 1 ? 1 : 0);
  static constexpr int T = L / NV;  // threads per transform
  static constexpr int radix(int s) { return s < NFULL ? NV : REM; }
  static constexpr int ns(int s) { return s == 0 ? 1 : ns(s - 1) * radix(s - 1); }
#ifdef CFDJ_LDS_PAD32
  static constexpr int PAD = L + L / 32;  // LDS elements per transform (1 pad per 32)
#else
  static constexpr int PAD = L + L / 16;  // LDS elements per transform (1 pad per 16)
#endif
  static constexpr int ROWSTRIDE = PAD;  // rows kernels: row stride (= 0 mod 64 banks)
};

#if defined(CFDJ_LDS_XOR)
__device__ __forceinline__ int padx(int i) { return i ^ ((i >> 4) & 15); }
#elif defined(CFDJ_LDS_PAD32)
__device__ __forceinline__ int padx(int i) { return i + (i >> 5); }
#else
__device__ __forceinline__ int padx(int i) { return i + (i >> 4); }
#endif

// The FD symbol aa + bb cos kx + cc cos ky, evaluated exactly as Common.jl:120 writes it
// (no FMA): for kx = eps the sum cancels to O(1) from terms of O(nx^2), so a contracted
// bb*cx changes psi by ~1e-11 relative at 4096^2 (measured) -- well outside parity.
__device__ __forceinline__ double fd_symbol_x(double aa, double bb, double cx) {
#pragma clang fp contract(off)
  return aa + bb * cx;
}
__device__ __forceinline__ double fd_symbol(double ax, double cc, double cy) {
#pragma clang fp contract(off)
  return ax + cc * cy;
}

// 1/d for the spectral divide: v_rcp_f64 refined by two Newton steps (|rel. error| below
// 2^-52 before the final rounding), i.e. within an ulp of the correctly rounded quotient
// the reference's `e / (...)` (Common.jl:121) forms.  Two true fp64 divisions per complex
// element cost the column pass 15 us of 81 at 4096^2 (measured on cols_kernel variants); d is a
// normal number here (|d| >= ~1e-7 for grids up to 16384^2, never 0 or denormal).
__device__ __forceinline__ double recip_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}

// Twiddles live in LDS as a 2-level table, W_L^e = hi[e >> 6] * lo[e & 63] (one rounding),
// filled once per persistent workgroup from the host-built long-double tables.  Keeping
// them out of the vector-memory stream matters: vmcnt is in order, so a twiddle load issued
// behind the next item's HBM prefetch would wait for that whole prefetch.
template <int L>
struct TwLds {
  static constexpr int HI = L / 64 > 0 ? L / 64 : 1;
  double2 lo[64];
  double2 hi[HI];
  __device__ __forceinline__ void fill(const double2* __restrict__ tw) {
    for (int i = threadIdx.x; i < 64 + HI; i += blockDim.x) {
      if (i < 64) lo[i] = tw[i];
      else hi[i - 64] = tw[(i - 64) * 64];
    }
  }
  __device__ __forceinline__ double2 w(int e) const { return cmul(hi[e >> 6], lo[e & 63]); }
};

// The same interface over the global long-double table (L2-resident): used where no HBM
// prefetch is queued ahead of the twiddle loads (the non-persistent column pass).
template <int L>
struct TwGlobal {
  const double2* __restrict__ t;
  __device__ __forceinline__ double2 w(int e) const { return t[e]; }
};

// Twiddles of one butterfly: w1 = W^e, w4 = W^{4e} (R >= 8) for the stage's base exponent
// e = (j mod NS) * L/(NS*R).
template <int L, int R, int NS>
struct Tw {
  double2 w1, w4;
};
template <int L, int R, int NS, class TW>
__device__ __forceinline__ Tw<L, R, NS> load_tw(int j, const TW& tw) {
  Tw<L, R, NS> t;
  if constexpr (NS > 1) {
    const int e = (j & (NS - 1)) * (L / (NS * R));
    t.w1 = tw.w(e);
    if constexpr (R >= 8) t.w4 = tw.w(4 * e);
  }
  return t;
}

// Twiddle the R inputs of butterfly j (Stockham stage with stride NS) and run the DFT.
template <int L, int R, int NS, int DIR>
__device__ __forceinline__ void butterfly(double2* v, const Tw<L, R, NS>& t) {
  if constexpr (NS > 1) {
    const double2 w1 = DIR < 0 ? t.w1 : cconj(t.w1);
    if constexpr (R == 2) {
      v[1] = cmul(v[1], w1);
    } else {
      const double2 w2 = cmul(w1, w1), w3 = cmul(w2, w1);
      v[1] = cmul(v[1], w1);
      v[2] = cmul(v[2], w2);
      v[3] = cmul(v[3], w3);
      if constexpr (R >= 8) {
        const double2 w4 = DIR < 0 ? t.w4 : cconj(t.w4);
        v[4] = cmul(v[4], w4);
        v[5] = cmul(v[5], cmul(w4, w1));
        v[6] = cmul(v[6], cmul(w4, w2));
        v[7] = cmul(v[7], cmul(w4, w3));
        if constexpr (R == 16) {
          const double2 w8 = cmul(w4, w4), w12 = cmul(w8, w4);
          v[8] = cmul(v[8], w8);
          v[9] = cmul(v[9], cmul(w8, w1));
          v[10] = cmul(v[10], cmul(w8, w2));
          v[11] = cmul(v[11], cmul(w8, w3));
          v[12] = cmul(v[12], w12);
          v[13] = cmul(v[13], cmul(w12, w1));
          v[14] = cmul(v[14], cmul(w12, w2));
          v[15] = cmul(v[15], cmul(w12, w3));
        }
      }
    }
  }
  dft<R, DIR>(v);
}

// Stage S of the plan on the thread's NV registers (NV/R butterflies of radix R):
// inputs v[b*R + r] = element (j_b + r*L/R), j_b = tid + b*T.  NV is deduced from the
// register array wherever one is passed.
template <int L, int S, int NV = 16>
struct StageTw {
  static constexpr int R = Plan<L, NV>::radix(S);
  static constexpr int NS = Plan<L, NV>::ns(S);
  Tw<L, R, NS> t[NV / R];
};
// The remainder stage (the last one; R = 2 or 4: 8 or 4 butterflies per thread): butterfly b's
// base twiddle is W_L^(tid + b T) = W_L^tid * W_16^b (T = L / 16) -- ONE table value, its
// powers shared by the butterflies, and compile-time 16th roots where 16 / R loaded values
// would sit in registers from before the exchange to the butterflies (L = 8192 rows: 142-154
// registers, one 512-thread workgroup per CU, against 120-128).  Not for R = 8 (L = 2048: two
// butterflies, nothing to win, and the seven shared powers cost the row kernels 7 registers
// and an occupancy step).  CFDJ_LAZY_LAST_MAXR=0: every butterfly's twiddles from the table.
#ifndef CFDJ_LAZY_LAST_MAXR
#define CFDJ_LAZY_LAST_MAXR 4
#endif
template <int L, int S, int NV>
constexpr bool lazy_last() {
  constexpr int R = Plan<L, NV>::radix(S);
  return NV == 16 && R <= CFDJ_LAZY_LAST_MAXR && Plan<L, NV>::ns(S) > 1 &&
         Plan<L, NV>::ns(S) * R == L;
}
template <int L, int S, class TW, int NV = 16>
__device__ __forceinline__ StageTw<L, S, NV> stage_tw(int tid, const TW& tw) {
  using ST = StageTw<L, S, NV>;
  ST st;
  if constexpr (lazy_last<L, S, NV>()) {
    st.t[0] = load_tw<L, ST::R, ST::NS, TW>(tid, tw);
  } else {
#pragma unroll
    for (int b = 0; b < NV / ST::R; ++b)
      st.t[b] = load_tw<L, ST::R, ST::NS, TW>(tid + b * Plan<L, NV>::T, tw);
  }
  return st;
}
// input r of butterfly B times base^r (pw[r], shared by the butterflies) times W_16^(r B)
template <int R, int DIR, int B, int Rr>
__device__ __forceinline__ void lazy_last_twiddle(double2* v, const double2* pw) {
  if constexpr (Rr < R) {
    v[B * R + Rr] = tw16<Rr * B, DIR>(cmul(v[B * R + Rr], pw[Rr]));
    lazy_last_twiddle<R, DIR, B, Rr + 1>(v, pw);
  }
}
template <int R, int DIR, int B>
__device__ __forceinline__ void lazy_last_butterflies(double2* v, const double2* pw) {
  if constexpr (B < 16 / R) {
    lazy_last_twiddle<R, DIR, B, 1>(v, pw);
    dft<R, DIR>(&v[B * R]);
    lazy_last_butterflies<R, DIR, B + 1>(v, pw);
  }
}
template <int L, int S, int DIR, int NV>
__device__ __forceinline__ void stage_regs(double2 (&v)[NV], const StageTw<L, S, NV>& st) {
  constexpr int R = Plan<L, NV>::radix(S);
  constexpr int NS = Plan<L, NV>::ns(S);
  if constexpr (lazy_last<L, S, NV>()) {
    // the powers of the base twiddle W_L^tid, in the transform's direction
    double2 pw[R];
    pw[1] = DIR < 0 ? st.t[0].w1 : cconj(st.t[0].w1);
    if constexpr (R >= 4) {
      pw[2] = cmul(pw[1], pw[1]);
      pw[3] = cmul(pw[2], pw[1]);
    }
    if constexpr (R >= 8) {
      pw[4] = DIR < 0 ? st.t[0].w4 : cconj(st.t[0].w4);
      pw[5] = cmul(pw[4], pw[1]);
      pw[6] = cmul(pw[4], pw[2]);
      pw[7] = cmul(pw[4], pw[3]);
    }
    lazy_last_butterflies<R, DIR, 0>(v, pw);
  } else {
#pragma unroll
    for (int b = 0; b < NV / R; ++b) butterfly<L, R, NS, DIR>(&v[b * R], st.t[b]);
  }
}
template <int L, int S, int DIR, class TW, int NV>
__device__ __forceinline__ void stage_regs(double2 (&v)[NV], int tid, const TW& tw) {
  stage_regs<L, S, DIR>(v, stage_tw<L, S, TW, NV>(tid, tw));
}

// Stage input / output positions.
template <int L, int S, int NV = 16>
__device__ __forceinline__ int in_pos(int tid, int b, int r) {
  using P = Plan<L, NV>;
  constexpr int R = P::radix(S);
  return tid + b * P::T + r * (L / R);
}
template <int L, int S, int NV = 16>
__device__ __forceinline__ int out_pos(int tid, int b, int r) {
  using P = Plan<L, NV>;
  constexpr int R = P::radix(S);
  constexpr int NS = P::ns(S);
  const int j = tid + b * P::T;
  return (j / NS) * NS * R + (j & (NS - 1)) + r * NS;
}

// LDS element p of a transform lives at buf[IL * padx(p)]: IL = 1 for one transform per
// buffer (rows), IL = 2 for the two interleaved columns of a tile (cols), so consecutive
// lanes -- (tid, c) pairs -- touch consecutive 16-B slots.
template <int L, int S, int IL = 1, int NV>
__device__ __forceinline__ void lds_write(double2* buf, const double2 (&v)[NV], int tid) {
  constexpr int R = Plan<L, NV>::radix(S);
#pragma unroll
  for (int b = 0; b < NV / R; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) buf[IL * padx(out_pos<L, S, NV>(tid, b, r))] = v[b * R + r];
}
template <int L, int S, int IL = 1, int NV>
__device__ __forceinline__ void lds_read(const double2* buf, double2 (&v)[NV], int tid) {
  constexpr int R = Plan<L, NV>::radix(S);
#pragma unroll
  for (int b = 0; b < NV / R; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) v[b * R + r] = buf[IL * padx(in_pos<L, S, NV>(tid, b, r))];
}

// Middle stages S0..NSTAGES-1 (each: read LDS, barrier, compute, write LDS, barrier).
// The caller has written stage S0-1's output to LDS and synchronised.
template <int L, int S, int DIR, bool LAST_TO_LDS, int IL = 1, class TW, int NV>
__device__ __forceinline__ void run_stages(double2* buf, double2 (&v)[NV], int tid,
                                           const TW& tw) {
  using P = Plan<L, NV>;
  if constexpr (S < P::NSTAGES) {
    const StageTw<L, S, NV> st = stage_tw<L, S, TW, NV>(tid, tw);
    lds_read<L, S, IL>(buf, v, tid);
    __syncthreads();
    stage_regs<L, S, DIR>(v, st);
    if constexpr (S + 1 < P::NSTAGES || LAST_TO_LDS) {
      lds_write<L, S, IL>(buf, v, tid);
      __syncthreads();
    }
    run_stages<L, S + 1, DIR, LAST_TO_LDS, IL>(buf, v, tid, tw);
  }
}

// Component-wise exchange: the transform's LDS buffer holds ONE double per element (half
// the footprint of the complex buffer, so more workgroups fit a CU) and the real and the
// imaginary parts pass through it one after the other.  C = 0: real, 1: imaginary.  IL as
// in lds_write: IL transforms interleaved element by element, `buf` offset by the
// transform's index.
template <int L, int S, int C, int IL = 1, int NV>
__device__ __forceinline__ void lds_write_half(double* buf, const double2 (&v)[NV], int tid) {
  constexpr int R = Plan<L, NV>::radix(S);
#pragma unroll
  for (int b = 0; b < NV / R; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r)
      buf[IL * padx(out_pos<L, S, NV>(tid, b, r))] = C ? v[b * R + r].y : v[b * R + r].x;
}
template <int L, int S, int C, int IL = 1, int NV>
__device__ __forceinline__ void lds_read_half(const double* buf, double2 (&v)[NV], int tid) {
  constexpr int R = Plan<L, NV>::radix(S);
#pragma unroll
  for (int b = 0; b < NV / R; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double t = buf[IL * padx(in_pos<L, S, NV>(tid, b, r))];
      if constexpr (C) v[b * R + r].y = t;
      else v[b * R + r].x = t;
    }
}
// Outputs of stage S-1 (in v) -> inputs of stage S (in v).  The leading barrier protects the
// buffer from readers of the previous exchange.
template <int L, int S, int IL = 1, int NV>
__device__ __forceinline__ void exchange_half(double* buf, double2 (&v)[NV], int tid) {
  __syncthreads();
  lds_write_half<L, S - 1, 0, IL>(buf, v, tid);
  __syncthreads();
  lds_read_half<L, S, 0, IL>(buf, v, tid);
  __syncthreads();
  lds_write_half<L, S - 1, 1, IL>(buf, v, tid);
  __syncthreads();
  lds_read_half<L, S, 1, IL>(buf, v, tid);
}
// Stages S..NSTAGES-1 on stage S-1's outputs held in v; the last stage's outputs stay in v.
template <int L, int S, int DIR, int IL = 1, class TW, int NV>
__device__ __forceinline__ void run_stages_half(double* buf, double2 (&v)[NV], int tid,
                                                const TW& tw) {
  using P = Plan<L, NV>;
  if constexpr (S < P::NSTAGES) {
    const StageTw<L, S, NV> st = stage_tw<L, S, TW, NV>(tid, tw);
    exchange_half<L, S, IL>(buf, v, tid);
    // keep the twiddle powers from being formed before the exchange, where both the old
    // and the new halves of v are live
    __builtin_amdgcn_sched_barrier(0);
    stage_regs<L, S, DIR>(v, st);
    run_stages_half<L, S + 1, DIR, IL>(buf, v, tid, tw);
  }
}

// run_stages for workgroups whose transform groups are not all busy: a group with
// act == false keeps every barrier (they are workgroup-wide, and stay outside the
// branches: act may differ inside one wavefront when T < 64) but touches no LDS.
template <int L, int S, int DIR, bool LAST_TO_LDS, int IL = 1, class TW, int NV>
__device__ __forceinline__ void run_stages_if(double2* buf, double2 (&v)[NV], int tid,
                                              const TW& tw, bool act) {
  using P = Plan<L, NV>;
  if constexpr (S < P::NSTAGES) {
    StageTw<L, S, NV> st;
    if (act) {
      st = stage_tw<L, S, TW, NV>(tid, tw);
      lds_read<L, S, IL>(buf, v, tid);
    }
    __syncthreads();
    if (act) stage_regs<L, S, DIR>(v, st);
    if constexpr (S + 1 < P::NSTAGES || LAST_TO_LDS) {
      if (act) lds_write<L, S, IL>(buf, v, tid);
      __syncthreads();
    }
    run_stages_if<L, S + 1, DIR, LAST_TO_LDS, IL>(buf, v, tid, tw, act);
  }
}

// After the forward transform's last stage a thread holds elements (j_b + r*NS), the same
// set the inverse transform's stage 0 reads (tid + T*r'), in a different register order:
// r' = b + (NV/R_last)*r.  fwd_to_inv permutes the registers accordingly.
template <int M, int NV>
__device__ __forceinline__ void fwd_to_inv(const double2 (&a)[NV], double2 (&v)[NV]) {
  using P = Plan<M, NV>;
  constexpr int RL = P::radix(P::NSTAGES - 1);
#pragma unroll
  for (int b = 0; b < NV / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) v[b + (NV / RL) * r] = a[b * RL + r];
}

// Persistent work split: `nb` resident workgroups (a multiple of 8) process items [0, n).
// XCD x = b % 8 owns the contiguous item range [x n/8, (x+1) n/8); its S = nb/8 workgroups
// take that range with stride S, so at any moment an XCD works on S adjacent items (which
// share 128-B lines) -- speed only, any placement is correct.
struct Range {
  int first, stride, count;
};
__device__ __forceinline__ Range persistent_range(int b, int nb, int n) {
  Range r;
  if ((nb & 7) == 0 && (n & 7) == 0 && nb <= n) {
    const int S = nb >> 3, x = b & 7, s = b >> 3, per = n >> 3;
    r.first = x * per + s;
    r.stride = S;
    r.count = s < per ? (per - s + S - 1) / S : 0;
  } else {
    r.first = b;
    r.stride = nb;
    r.count = b < n ? (n - b + nb - 1) / nb : 0;
  }
  return r;
}

}  // namespace

}  // namespace cfdj
