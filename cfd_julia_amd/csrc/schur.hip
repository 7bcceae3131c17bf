// Substructured y-solve of the multi-GPU (y-slab) FFT Poisson path.
//
// Common.jl:97-125 divides the 2-D spectrum by D(m, k) = aa + bb cos kx_m + cc cos ky_k.
// After the real FFT along x (rows_fwd_kernel, local to a slab), each x-mode m >= 1 needs
// the y-direction operator psi[j-1]/dy^2 + d_m psi[j] + psi[j+1]/dy^2 (d_m = aa + bb
// cos kx_m) inverted on the periodic column -- a tridiagonal circulant whose eigenvalues are
// D(m, k), except at k = 0 where the reference's ky[1] = eps shifts the constant mode (a
// rank-one correction, `corr`).  Instead of transposing the whole spectrum between GPUs
// (two all-to-alls of nx*ny/2 complex per solve), every slab
//   pass 0 (schur_trace_kernel): the two boundary values of its interior rows' solution with
//          zero Dirichlet data (dot products with the tabulated interior Green's function),
//          its separator row f[0] and its column sum;
//   (the host all-gathers those 4 numbers per mode: 64 B x nx/2 per rank)
//   pass 1 (schur_solve_kernel): solves the P x P circulant separator system for its two
//          separator values (precomputed inverse), solves the interior rows 1..rl-1 with
//          them as Dirichlet data (DST-I = FFT of length 2 rl on the odd extension, in LDS)
//          and writes psi-hat (plus the constant-mode correction) in place.
// The x-modes 0 and nx/2 (packed in column 0) are solved separately: the column is gathered
// and FFT'd along y with the reference symbol (packed_divide_kernel).
// Host-side tables (long double): e_m, q_k, the circulant inverse, corr -- host_common.hpp.
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

namespace cfdj {

namespace {

__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }

// Odd extension of interior rows 1..RL-1 of a slab column (length M2 = 2 RL), stage-0
// order; `fix1` / `fixn` are subtracted from rows 1 and RL-1 (Dirichlet data of pass 1).
// Returns the sum of the loaded interior values in `fs`.
template <int M2>
__device__ __forceinline__ void load_odd(double2 (&v)[16], const double2* __restrict__ col,
                                         int cs, int tid, double2 fix1, double2 fixn,
                                         double2& fs) {
  constexpr int RL = M2 / 2;
  constexpr int R0 = Plan<M2>::radix(0);
#pragma unroll
  for (int b = 0; b < 16 / R0; ++b)
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int j = in_pos<M2, 0>(tid, b, r);
      const int i = j < RL ? j : M2 - j;  // interior row of this element
      double2 x = make_double2(0.0, 0.0);
      if (i != 0 && i != RL) {
        x = col[(size_t)i * cs];
        if (i == 1) x = csub(x, fix1);
        if (i == RL - 1) x = csub(x, fixn);
        if (j < RL) fs = cadd(fs, x);
        else x = make_double2(-x.x, -x.y);
      }
      v[b * R0 + r] = x;
    }
}

// W_k = Y_k / lambda_k, lambda_k = e_m - cc q_|k| (no cancellation: both terms <= 0);
// k = 0 and k = RL carry nothing (odd extension).
template <int M2>
__device__ __forceinline__ double2 dst_divide(double2 y, int k, double em, double cc,
                                              const double* __restrict__ q) {
  constexpr int RL = M2 / 2;
  if (k == 0 || k == RL) return make_double2(0.0, 0.0);
  const int kk = k < RL ? k : M2 - k;
  const double lam = em - cc * q[kk];
  return make_double2(y.x / lam, y.y / lam);
}

// Column m of the slab spectrum: base pointer and element stride (column-major, or the
// 8-mode tiles of poisson_fft.hip's sidx: element (m, j) at ((m/8) rl + j) 8 + m%8).
__device__ __forceinline__ double2* slab_col(const SchurArgs& a, int m, int& cs) {
  cs = a.tile8 ? 8 : 1;
  return a.H + (a.tile8 ? ((((size_t)(m >> 3)) * a.rl) << 3) + (m & 7) : (size_t)m * a.rl);
}

// Pass 0: one workgroup per 8-mode tile of the spectrum (8 x-modes, element (m, j) at
// ((m/8) rl + j) 8 + m%8, rows_fwd_kernel's tiled output), so every wavefront load is 8
// whole rows of the tile, 1 KB contiguous.  The zero-Dirichlet interior solution's
// boundary values are rows of the interior Green's function, (T_int^-1)[1, j] =
// -dy^2 gL(j) and (T_int^-1)[n, j] = -dy^2 gL(rl - j) (gL: the homogeneous solution with
// gL(0) = 1, gL(rl) = 0, tabulated on the host in long double, same tiling), so the
// traces are two dot products over the slab column -- one streaming read, no transform.
// Lane = (row r, mode mi): mi = tid % 8, rows j = 1 + tid/8, + 32, ...
constexpr int kTraceThreads = 256;
__global__ __launch_bounds__(kTraceThreads) void schur_trace_kernel(const SchurArgs a) {
  const int tb = xcd_remap(blockIdx.x, gridDim.x);  // tile: modes 8 tb .. 8 tb + 7
  const int mi = threadIdx.x & 7, r0 = threadIdx.x >> 3;
  const int m = 8 * tb + mi;
  const int rl = a.rl;
  const double2* tile = a.H + (((size_t)tb * rl) << 3);
  const double* g = a.g + (((size_t)tb * (rl + 1)) << 3) + mi;
  double2 t1 = make_double2(0.0, 0.0), tn = t1, fs = t1;
  for (int j = 1 + r0; j < rl; j += kTraceThreads / 8) {
    const double2 f = tile[((size_t)j << 3) + mi];
    t1 = cadd(t1, cscale(f, g[(size_t)j << 3]));
    tn = cadd(tn, cscale(f, g[(size_t)(rl - j) << 3]));
    fs = cadd(fs, f);
  }
  // sum over the 8 row lanes of a wavefront with the same mode, then over the 4 waves
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    t1.x += __shfl_xor(t1.x, o);
    t1.y += __shfl_xor(t1.y, o);
    tn.x += __shfl_xor(tn.x, o);
    tn.y += __shfl_xor(tn.y, o);
    fs.x += __shfl_xor(fs.x, o);
    fs.y += __shfl_xor(fs.y, o);
  }
  constexpr int W = kTraceThreads / 64;
  __shared__ double2 red[3][W][8];
  const int wv = threadIdx.x / 64, ln = threadIdx.x % 64;
  if (ln < 8) {
    red[0][wv][ln] = t1;
    red[1][wv][ln] = tn;
    red[2][wv][ln] = fs;
  }
  __syncthreads();
  if (threadIdx.x < 8 && m >= 1) {
    t1 = tn = fs = make_double2(0.0, 0.0);
    for (int w = 0; w < W; ++w) {
      t1 = cadd(t1, red[0][w][mi]);
      tn = cadd(tn, red[1][w][mi]);
      fs = cadd(fs, red[2][w][mi]);
    }
    const double2 fsep = tile[mi];
    const double mdy2 = -1.0 / a.inv_dy2;
    double2* out = a.T + ((size_t)a.rank * a.L + m) * 4;
    out[0] = fsep;
    out[1] = cscale(t1, mdy2);
    out[2] = cscale(tn, mdy2);
    out[3] = cadd(fs, fsep);
  }
}

template <int M2>
__global__ __launch_bounds__(Plan<M2>::T) void schur_solve_kernel(const SchurArgs a) {
  using P = Plan<M2>;
  constexpr int RL = M2 / 2;
  __shared__ double2 lds[P::PAD];
  const TwGlobal<M2> tw{a.tw};
  const int tid = threadIdx.x;
  const int m = 1 + xcd_remap(blockIdx.x, gridDim.x);
  int cs;
  double2* col = slab_col(a, m, cs);

  // separator values s_rank, s_rank+1 from every rank's traces (P <= a few dozen)
  double2 sp = make_double2(0.0, 0.0), sq = sp, fb = sp;
  const double* ci = a.cinv + (size_t)m * a.P;
  for (int qq = 0; qq < a.P; ++qq) {
    const double2* Tq = a.T + ((size_t)qq * a.L + m) * 4;
    const double2* Tm = a.T + ((size_t)((qq + a.P - 1) % a.P) * a.L + m) * 4;
    const double2 rhs = csub(Tq[0], cscale(cadd(Tm[2], Tq[1]), a.inv_dy2));
    sp = cadd(sp, cscale(rhs, ci[(qq - a.rank + a.P) % a.P]));
    sq = cadd(sq, cscale(rhs, ci[(qq - a.rank - 1 + 2 * a.P) % a.P]));
    fb = cadd(fb, Tq[3]);
  }
  const double2 cst = cscale(fb, a.corr[m] * a.inv_ny);

  double2 v[16];
  double2 fs = make_double2(0.0, 0.0);
  load_odd<M2>(v, col, cs, tid, cscale(sp, a.inv_dy2), cscale(sq, a.inv_dy2), fs);
  stage_regs<M2, 0, -1>(v, tid, tw);
  lds_write<M2, 0>(lds, v, tid);
  __syncthreads();
  run_stages<M2, 1, -1, false>(lds, v, tid, tw);
  double2 w[16];
  fwd_to_inv<M2>(v, w);
  const double em = a.e[m];
#pragma unroll
  for (int r = 0; r < 16; ++r) w[r] = dst_divide<M2>(w[r], tid + P::T * r, em, a.cc, a.q);
  __syncthreads();  // LDS is rewritten by the inverse stage 0
  stage_regs<M2, 0, 1>(w, tid, tw);
  lds_write<M2, 0>(lds, w, tid);
  __syncthreads();
  run_stages<M2, 1, 1, false>(lds, w, tid, tw);
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RLAST = P::radix(SL);
  const double s = a.out_scale;
#pragma unroll
  for (int b = 0; b < 16 / RLAST; ++b)
#pragma unroll
    for (int r = 0; r < RLAST; ++r) {
      const int j = out_pos<M2, SL>(tid, b, r);
      if (j >= 1 && j < RL) {
        const double2 x = w[b * RLAST + r];
        col[(size_t)j * cs] =
            make_double2((x.x * (1.0 / M2) + cst.x) * s, (x.y * (1.0 / M2) + cst.y) * s);
      }
    }
  if (tid == 0) col[0] = make_double2((sp.x + cst.x) * s, (sp.y + cst.y) * s);
}

__global__ __launch_bounds__(256) void packed_divide_kernel(const PackedDivParams p) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > p.ny / 2) return;
  const int kp = (p.ny - k) & (p.ny - 1);
  const double sgn = p.neg ? -1.0 : 1.0;
  const double ax0 = fd_symbol_x(p.aa, p.bb, p.cx[0]);    // kx = eps
  const double axL = fd_symbol_x(p.aa, p.bb, p.cx[p.L]);  // kx = -pi
  const double2 Zk = p.Z[k], Zp = p.Z[kp];
  auto one = [&](double2 Z, double2 Zpart, int kk) {
    const double2 Zc = cconj(Zpart);
    const double2 A = make_double2(0.5 * (Z.x + Zc.x), 0.5 * (Z.y + Zc.y));
    const double2 D = csub(Z, Zc);
    const double2 B = make_double2(0.5 * D.y, -0.5 * D.x);
    const double cyk = p.cy[kk];
    const double d0 = fd_symbol(ax0, p.cc, cyk);
    const double dL = fd_symbol(axL, p.cc, cyk);
    const double2 A2 = kk == 0 ? make_double2(0.0, 0.0)  // e[1,1] = 0 (Common.jl:118)
                               : make_double2(sgn * A.x / d0, sgn * A.y / d0);
    const double2 B2 = make_double2(sgn * B.x / dL, sgn * B.y / dL);
    return make_double2((A2.x - B2.y) * p.scale, (A2.y + B2.x) * p.scale);
  };
  const double2 ok = one(Zk, Zp, k);
  const double2 op = one(Zp, Zk, kp);
  p.Z[k] = ok;
  if (kp != k) p.Z[kp] = op;
}

template <int M2>
void launch_schur_n(int pass, const SchurArgs& a, hipStream_t st) {
  const dim3 grid(a.L - 1), block(Plan<M2>::T);
  if (pass == 0)
    hipLaunchKernelGGL(schur_trace_kernel, dim3(a.L / 8), dim3(kTraceThreads), 0, st, a);
  else
    hipLaunchKernelGGL(schur_solve_kernel<M2>, grid, block, 0, st, a);
}

}  // namespace

// Slab heights whose odd extension (2 rl) is one of the in-LDS FFT lengths.
bool schur_supported(int rl) { return rl == 512 || rl == 1024 || rl == 2048 || rl == 4096; }

void launch_schur_pass(int pass, const SchurArgs& a, hipStream_t st) {
  if (!schur_supported(a.rl) || a.L < 8 || a.L % 8 != 0 || !a.tile8 || a.P < 1 ||
      a.rank < 0 || a.rank >= a.P)
    throw Error{CFDJ_ERR_ARG, "substructured Poisson: unsupported slab"};
  switch (a.rl) {
    case 512: launch_schur_n<1024>(pass, a, st); break;
    case 1024: launch_schur_n<2048>(pass, a, st); break;
    case 2048: launch_schur_n<4096>(pass, a, st); break;
    case 4096: launch_schur_n<8192>(pass, a, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_packed_divide(const PackedDivParams& p, hipStream_t st) {
  const int n = p.ny / 2 + 1;
  hipLaunchKernelGGL(packed_divide_kernel, dim3((n + 255) / 256), dim3(256), 0, st, p);
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
