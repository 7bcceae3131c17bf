// Hand-written fused FD-FFT Poisson solver for square power-of-two grids (gfx950).
//
// Replaces rocFFT D2Z + divide + Z2D (8 rocFFT passes + 1 divide pass over HBM at 4096^2)
// with THREE passes (Common.jl:97-125 semantics):
//
//   rows_fwd   : each row of the real field f (N reals) is read as N/2 complex z[n] =
//                f[2n] + i f[2n+1], FFT'd (length L = N/2, Stockham radix-16 in LDS), and
//                post-processed into the real-FFT half spectrum X[m], m = 0..L-1, with the
//                two real coefficients X[0] (DC) and X[L] (Nyquist) packed into slot 0 as
//                X[0] + i X[L].  Output is written COLUMN-TILED: tile t holds columns
//                m = 2t, 2t+1 for all rows, H[t][y][c] (32 B per row, 128 KB per tile), so
//                the column pass reads one contiguous block.
//   cols       : one workgroup per 2-column tile: forward FFT along y (length M), the
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
#include "cfdj_internal.hpp"

#pragma clang fp contract(fast)

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

// Stockham plan of a length-L transform: radix-16 stages, then one remainder stage.
template <int L>
struct Plan {
  static constexpr int LOG = ilog2(L);
  static constexpr int N16 = LOG / 4;
  static constexpr int REM = 1 << (LOG % 4);
  static constexpr int NSTAGES = N16 + (REM > 1 ? 1 : 0);
  static constexpr int T = L / 16;  // threads per transform
  static constexpr int radix(int s) { return s < N16 ? 16 : REM; }
  static constexpr int ns(int s) { return s == 0 ? 1 : ns(s - 1) * radix(s - 1); }
  static constexpr int PAD = L + L / 16;  // LDS elements per transform (1 pad per 16)
  static constexpr int ROWSTRIDE = PAD + 2;  // rows kernels: stagger banks between rows
};

__device__ __forceinline__ int padx(int i) { return i + (i >> 4); }

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

// Twiddles of one butterfly: w[0] = W^e, w[1] = W^{4e} (R >= 8) for the stage's base
// exponent e = (j mod NS) * L/(NS*R); tw[i] = exp(-2 pi i i / L).  Loaded early (before the
// stage's LDS reads and barrier) so the L2 latency overlaps them.
template <int L, int R, int NS>
struct Tw {
  double2 w1, w4;
};
template <int L, int R, int NS>
__device__ __forceinline__ Tw<L, R, NS> load_tw(int j, const double2* __restrict__ tw) {
  Tw<L, R, NS> t;
  if constexpr (NS > 1) {
    const int e = (j & (NS - 1)) * (L / (NS * R));
    t.w1 = tw[e];
    if constexpr (R >= 8) t.w4 = tw[4 * e];
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

// Stage S of the plan on the thread's 16 registers (16/R butterflies of radix R):
// inputs v[b*R + r] = element (j_b + r*L/R), j_b = tid + b*T.
template <int L, int S>
struct StageTw {
  static constexpr int R = Plan<L>::radix(S);
  static constexpr int NS = Plan<L>::ns(S);
  Tw<L, R, NS> t[16 / R];
};
template <int L, int S>
__device__ __forceinline__ StageTw<L, S> stage_tw(int tid, const double2* __restrict__ tw) {
  StageTw<L, S> st;
#pragma unroll
  for (int b = 0; b < 16 / StageTw<L, S>::R; ++b)
    st.t[b] = load_tw<L, StageTw<L, S>::R, StageTw<L, S>::NS>(tid + b * Plan<L>::T, tw);
  return st;
}
template <int L, int S, int DIR>
__device__ __forceinline__ void stage_regs(double2 (&v)[16], const StageTw<L, S>& st) {
  constexpr int R = Plan<L>::radix(S);
  constexpr int NS = Plan<L>::ns(S);
#pragma unroll
  for (int b = 0; b < 16 / R; ++b) butterfly<L, R, NS, DIR>(&v[b * R], st.t[b]);
}
template <int L, int S, int DIR>
__device__ __forceinline__ void stage_regs(double2 (&v)[16], int tid,
                                           const double2* __restrict__ tw) {
  stage_regs<L, S, DIR>(v, stage_tw<L, S>(tid, tw));
}

// Stage input / output positions.
template <int L, int S>
__device__ __forceinline__ int in_pos(int tid, int b, int r) {
  using P = Plan<L>;
  constexpr int R = P::radix(S);
  return tid + b * P::T + r * (L / R);
}
template <int L, int S>
__device__ __forceinline__ int out_pos(int tid, int b, int r) {
  using P = Plan<L>;
  constexpr int R = P::radix(S);
  constexpr int NS = P::ns(S);
  const int j = tid + b * P::T;
  return (j / NS) * NS * R + (j & (NS - 1)) + r * NS;
}

// LDS element p of a transform lives at buf[IL * padx(p)]: IL = 1 for one transform per
// buffer (rows), IL = 2 for the two interleaved columns of a tile (cols), so consecutive
// lanes -- (tid, c) pairs -- touch consecutive 16-B slots.
template <int L, int S, int IL = 1>
__device__ __forceinline__ void lds_write(double2* buf, const double2 (&v)[16], int tid) {
  constexpr int R = Plan<L>::radix(S);
#pragma unroll
  for (int b = 0; b < 16 / R; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) buf[IL * padx(out_pos<L, S>(tid, b, r))] = v[b * R + r];
}
template <int L, int S, int IL = 1>
__device__ __forceinline__ void lds_read(const double2* buf, double2 (&v)[16], int tid) {
  constexpr int R = Plan<L>::radix(S);
#pragma unroll
  for (int b = 0; b < 16 / R; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) v[b * R + r] = buf[IL * padx(in_pos<L, S>(tid, b, r))];
}

// Middle stages S0..NSTAGES-1 (each: read LDS, barrier, compute, write LDS, barrier).
// The caller has written stage S0-1's output to LDS and synchronised.
template <int L, int S, int DIR, bool LAST_TO_LDS, int IL = 1>
__device__ __forceinline__ void run_stages(double2* buf, double2 (&v)[16], int tid,
                                           const double2* __restrict__ tw) {
  using P = Plan<L>;
  if constexpr (S < P::NSTAGES) {
    const StageTw<L, S> st = stage_tw<L, S>(tid, tw);
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

// ---------------------------------------------------------------------------------------
// Pass 1: rows, real -> packed half spectrum, column-tiled output.
// ---------------------------------------------------------------------------------------
template <int L>
struct RowCfg {
  static constexpr int T = Plan<L>::T;
  static constexpr int XR = (256 / T) > 4 ? (256 / T) : 4;  // rows per workgroup
  static constexpr int THREADS = XR * T;
};

template <int L>
__global__ __launch_bounds__(RowCfg<L>::THREADS) void rows_fwd_kernel(
    const double* __restrict__ f, double2* __restrict__ H, int M,
    const double2* __restrict__ twL, const double2* __restrict__ twN) {
  using P = Plan<L>;
  using C = RowCfg<L>;
  __shared__ double2 lds[C::XR * P::ROWSTRIDE];
  const int q = threadIdx.x / P::T;
  const int tid = threadIdx.x % P::T;
  const int y0 = blockIdx.x * C::XR;
  double2* buf = lds + q * P::ROWSTRIDE;

  // stage 0 straight from HBM: z[n] = f[2n] + i f[2n+1]
  const double2* z = reinterpret_cast<const double2*>(f + (size_t)(y0 + q) * (2 * L));
  double2 v[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) v[b * R0 + r] = z[in_pos<L, 0>(tid, b, r)];
  stage_regs<L, 0, -1>(v, tid, twL);
  lds_write<L, 0>(buf, v, tid);
  __syncthreads();
  run_stages<L, 1, -1, true>(buf, v, tid, twL);

  // post-process: X[m] = E[m] + W_N^m O[m]; slot 0 = X[0] + i X[L].  Thread <-> element
  // assignment chosen so consecutive lanes write consecutive addresses of a tile.
  constexpr int PER = (L * C::XR) / C::THREADS;  // = 16
#pragma unroll 4
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * C::THREADS;
    const int c = e & 1;
    const int qq = (e >> 1) % C::XR;
    const int t = (e >> 1) / C::XR;
    const int m = 2 * t + c;
    const double2* bq = lds + qq * P::ROWSTRIDE;
    const double2 Zm = bq[padx(m)];
    double2 X;
    if (m == 0) {
      X = make_double2(Zm.x + Zm.y, Zm.x - Zm.y);
    } else {
      const double2 Zc = cconj(bq[padx(L - m)]);
      const double2 E = make_double2(0.5 * (Zm.x + Zc.x), 0.5 * (Zm.y + Zc.y));
      const double2 D = csub(Zm, Zc);                       // = 2i O
      const double2 O = make_double2(0.5 * D.y, -0.5 * D.x);  // D / (2i)
      X = cadd(E, cmul(twN[m], O));
    }
    H[((size_t)t * M + y0 + qq) * 2 + c] = X;
  }
}

// ---------------------------------------------------------------------------------------
// Pass 2: columns of one 2-column tile: forward FFT, divide, inverse FFT, in place.
// ---------------------------------------------------------------------------------------
struct DivArgs {
  const double* cx;  // cos(kx[m]), m <= L
  const double* cy;  // cos(ky[k]), k < M
  double aa, bb, cc, scale;
  int L;
  int neg;
};

template <int M>
__global__ __launch_bounds__(2 * Plan<M>::T) void cols_kernel(double2* __restrict__ H,
                                                            const double2* __restrict__ twM,
                                                            const DivArgs da) {
  using P = Plan<M>;
  __shared__ double2 lds[2 * P::PAD];
  const int c = threadIdx.x & 1;
  const int tid = threadIdx.x >> 1;
  const int t = blockIdx.x;
  double2* buf = lds + c;                      // interleaved columns: buf[2*padx(p)]
  double2* tile = H + (size_t)t * M * 2 + c;  // element y at tile[2*y]

  double2 v[16];
  constexpr int R0 = P::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) v[b * R0 + r] = tile[2 * in_pos<M, 0>(tid, b, r)];
  stage_regs<M, 0, -1>(v, tid, twM);
  lds_write<M, 0, 2>(buf, v, tid);
  __syncthreads();
  run_stages<M, 1, -1, true, 2>(buf, v, tid, twM);  // natural-order spectrum in LDS

  // divide (Common.jl:118-121) fused into the first inverse stage's loads
  const int m = 2 * t + c;
  const double sgn = da.neg ? -1.0 : 1.0;
  const double ax = fd_symbol_x(da.aa, da.bb, da.cx[m]);
  const double axL = fd_symbol_x(da.aa, da.bb, da.cx[da.L]);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int k = in_pos<M, 0>(tid, b, r);
      const double2 Z = buf[2 * padx(k)];
      const double cyk = da.cy[k];
      double2 o;
      if (m != 0) {
        const double d = fd_symbol(ax, da.cc, cyk);
        o = make_double2((sgn * Z.x / d) * da.scale, (sgn * Z.y / d) * da.scale);
      } else {
        // packed column: Z = FFT_y(X_dc + i X_nyq); split, divide each, re-pack
        const double2 Zc = cconj(buf[2 * padx((M - k) & (M - 1))]);
        const double2 A = make_double2(0.5 * (Z.x + Zc.x), 0.5 * (Z.y + Zc.y));
        const double2 D = csub(Z, Zc);
        const double2 B = make_double2(0.5 * D.y, -0.5 * D.x);
        const double d0 = fd_symbol(ax, da.cc, cyk);   // kx = eps column
        const double dL = fd_symbol(axL, da.cc, cyk);  // kx = -pi column
        const double2 A2 = k == 0 ? make_double2(0.0, 0.0)  // e[1,1] = 0
                                  : make_double2(sgn * A.x / d0, sgn * A.y / d0);
        const double2 B2 = make_double2(sgn * B.x / dL, sgn * B.y / dL);
        o = make_double2((A2.x - B2.y) * da.scale, (A2.y + B2.x) * da.scale);
      }
      v[b * R0 + r] = o;
    }
  __syncthreads();
  stage_regs<M, 0, 1>(v, tid, twM);
  if constexpr (P::NSTAGES > 1) {
    lds_write<M, 0, 2>(buf, v, tid);
    __syncthreads();
    run_stages<M, 1, 1, false, 2>(buf, v, tid, twM);
  }
  // last inverse stage: outputs j + r*NS are in natural order -> straight to HBM
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) tile[2 * out_pos<M, SL>(tid, b, r)] = v[b * RL + r];
}

// ---------------------------------------------------------------------------------------
// Pass 3: rows, packed half spectrum -> real (c2r).
// ---------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(RowCfg<L>::THREADS) void rows_inv_kernel(
    const double2* __restrict__ H, double* __restrict__ f, int M,
    const double2* __restrict__ twL, const double2* __restrict__ twN) {
  using P = Plan<L>;
  using C = RowCfg<L>;
  __shared__ double2 lds[C::XR * P::ROWSTRIDE];
  const int y0 = blockIdx.x * C::XR;

  // pre-process: Z[m] = (X[m] + conj X[L-m]) + i W_N^{-m} (X[m] - conj X[L-m])
  constexpr int PER = (L * C::XR) / C::THREADS;
#pragma unroll 4
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * C::THREADS;
    const int c = e & 1;
    const int qq = (e >> 1) % C::XR;
    const int t = (e >> 1) / C::XR;
    const int m = 2 * t + c;
    const double2 Xm = H[((size_t)t * M + y0 + qq) * 2 + c];
    double2 Z;
    if (m == 0) {  // slot 0 = (X[0], X[L]), both real
      Z = make_double2(Xm.x + Xm.y, Xm.x - Xm.y);
    } else {
      const int mp = L - m;
      const double2 Xp = cconj(H[((size_t)(mp >> 1) * M + y0 + qq) * 2 + (mp & 1)]);
      const double2 S = cadd(Xm, Xp);
      const double2 D = cmul(cconj(twN[m]), csub(Xm, Xp));
      Z = make_double2(S.x - D.y, S.y + D.x);
    }
    lds[qq * P::ROWSTRIDE + padx(m)] = Z;
  }
  __syncthreads();

  const int q = threadIdx.x / P::T;
  const int tid = threadIdx.x % P::T;
  double2* buf = lds + q * P::ROWSTRIDE;
  double2 v[16];
  run_stages<L, 0, 1, false>(buf, v, tid, twL);
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  double2* z = reinterpret_cast<double2*>(f + (size_t)(y0 + q) * (2 * L));
#pragma unroll
  for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
    for (int r = 0; r < RL; ++r) z[out_pos<L, SL>(tid, b, r)] = v[b * RL + r];
}

template <int N>
void launch_fused_n(int pass, const FusedPoissonArgs& a, hipStream_t st) {
  constexpr int L = N / 2;
  using C = RowCfg<L>;
  const int M = N;
  if (pass == 0) {
    hipLaunchKernelGGL(rows_fwd_kernel<L>, dim3(M / C::XR), dim3(C::THREADS), 0, st, a.f, a.H,
                       M, a.twL, a.twN);
  } else if (pass == 1) {
    DivArgs da{a.cx, a.cy, a.aa, a.bb, a.cc, a.scale, L, a.neg ? 1 : 0};
    hipLaunchKernelGGL(cols_kernel<N>, dim3(L / 2), dim3(2 * Plan<N>::T), 0, st, a.H, a.twN,
                       da);
  } else {
    hipLaunchKernelGGL(rows_inv_kernel<L>, dim3(M / C::XR), dim3(C::THREADS), 0, st, a.H, a.s,
                       M, a.twL, a.twN);
  }
  CFDJ_HIP(hipGetLastError());
}

}  // namespace

bool fused_poisson_supported(int nx, int ny) {
  return nx == ny && (nx == 1024 || nx == 2048 || nx == 4096);
}

void launch_fused_poisson_pass(int pass, const FusedPoissonArgs& a, hipStream_t st) {
  switch (a.n) {
    case 1024: launch_fused_n<1024>(pass, a, st); break;
    case 2048: launch_fused_n<2048>(pass, a, st); break;
    case 4096: launch_fused_n<4096>(pass, a, st); break;
    default: throw Error{CFDJ_ERR_ARG, "fused Poisson: unsupported size"};
  }
}

}  // namespace cfdj
