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
//          separator values (precomputed inverse), then the interior rows 1..rl-1 with
//          them as Dirichlet data -- a constant-coefficient tridiagonal system per mode,
//          solved directly in 32-row chunks + a reduced interface system -- and writes
//          psi-hat (plus the constant-mode correction) in place.
// The x-modes 0 and nx/2 (packed in column 0) are solved separately: the column is gathered
// and solved along y with the reference symbol (columns of up to 8192: the single-GPU column
// pass of poisson_fft.hip on that one column; longer: library transforms around
// packed_divide_kernel).
// Host-side tables (long double): the circulant inverse, corr, the Green's function of the
// trace pass, the chunk / interface pivots and homogeneous solutions -- host_common.hpp.
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

namespace cfdj {

namespace {

__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }

// Pass 0: one workgroup per 8-mode tile of the spectrum (8 x-modes, element (m, j) at
// ((m/8) rl + j) 8 + m%8, rows_fwd_kernel's tiled output), so every wavefront load is 8
// whole rows of the tile, 1 KB contiguous.  The zero-Dirichlet interior solution's
// boundary values are rows of the interior Green's function, (T_int^-1)[1, j] =
// -dy^2 gL(j) and (T_int^-1)[n, j] = -dy^2 gL(rl - j) (gL: the homogeneous solution with
// gL(0) = 1, gL(rl) = 0, tabulated on the host in long double, same tiling), so the
// traces are two dot products over the slab column -- one streaming read, no transform.
// Lane = (row r, mode mi): mi = tid % 8, rows j = 1 + tid/8, + 32, ...
// (256 threads: with 1024 -- the slowest modes' whole-column tiles in one batch of loads --
// the kernel measured 11.2 us against 8.9 at 8192 x 1024, 15.6 against 14.4 at 8192 x 2048)
#ifndef CFDJ_TRACE_THREADS
#define CFDJ_TRACE_THREADS 256
#endif
constexpr int kTraceThreads = CFDJ_TRACE_THREADS;
#ifndef CFDJ_TRACE_MODES
#define CFDJ_TRACE_MODES 8
#endif
// Modes per workgroup (8 = a whole tile, 128-B row pieces; fewer = more row lanes per mode).
// The kernel's duration is its slowest workgroup's: the lowest modes' tiles read their whole
// column, rl / (threads / modes) rows per lane in batches of U with a load round trip each.
constexpr int kTraceModes = CFDJ_TRACE_MODES;
__global__ __launch_bounds__(kTraceThreads) void schur_trace_kernel(const SchurArgs a) {
  constexpr int MPW = kTraceModes, PER = 8 / MPW;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tb = lb / PER;  // tile: modes 8 tb .. 8 tb + 7
  const int mi = (lb % PER) * MPW + threadIdx.x % MPW, r0 = threadIdx.x / MPW;
  const int m = 8 * tb + mi;
  const int rl = a.rl;
  const double2* tile = a.H + (((size_t)tb * rl) << 3);
  const double* g = a.g + (((size_t)tb * (rl + 1)) << 3) + mi;
  // gL decays like e^{-j th_m}: only the first / last jt rows of the tile's modes carry
  // trace terms above round-off (host-tabulated, jt = rl for the slowest modes); the
  // column sum comes from the stage kernel's column partials (a.cs), not from this pass
  double2 t1 = make_double2(0.0, 0.0), tn = t1;
  const int J = a.jt[tb];
  constexpr int RS = kTraceThreads / MPW;
  // loads in batches of U rows per lane (the lane's rows still summed in increasing j, so
  // the result does not depend on U): the slowest tiles' full-column loop is load-latency
  // bound, one batch in flight per iteration
#ifndef CFDJ_TRACE_U
#define CFDJ_TRACE_U 8
#endif
  constexpr int U = CFDJ_TRACE_U;
  auto sweep = [&](int jb, int je, bool first, bool last) {
    for (int j0 = jb + r0; j0 < je; j0 += U * RS) {
      double2 f[U];
      double g1[U], gn[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * RS;
        const bool ok = j < je;
        const int jj = ok ? j : jb;
        f[u] = ok ? tile[((size_t)jj << 3) + mi] : make_double2(0.0, 0.0);
        g1[u] = first ? g[(size_t)jj << 3] : 0.0;
        gn[u] = last ? g[(size_t)(rl - jj) << 3] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j0 + u * RS < je) {
          if (first) t1 = cadd(t1, cscale(f[u], g1[u]));
          if (last) tn = cadd(tn, cscale(f[u], gn[u]));
        }
      }
    }
  };
  if (2 * J >= rl - 1) {
    sweep(1, rl, true, true);
  } else {
    sweep(1, J + 1, true, false);
    sweep(rl - J, rl, false, true);
  }
  // sum over the row lanes of a wavefront with the same mode, then over the waves
#pragma unroll
  for (int o = MPW; o < 64; o <<= 1) {
    t1.x += __shfl_xor(t1.x, o);
    t1.y += __shfl_xor(t1.y, o);
    tn.x += __shfl_xor(tn.x, o);
    tn.y += __shfl_xor(tn.y, o);
  }
  constexpr int W = kTraceThreads / 64;
  __shared__ double2 red[2][W][MPW];
  const int wv = threadIdx.x / 64, ln = threadIdx.x % 64;
  if (ln < MPW) {
    red[0][wv][ln] = t1;
    red[1][wv][ln] = tn;
  }
  __syncthreads();
  if (threadIdx.x < MPW && m >= 1) {
    t1 = tn = make_double2(0.0, 0.0);
    for (int w = 0; w < W; ++w) {
      t1 = cadd(t1, red[0][w][threadIdx.x]);
      tn = cadd(tn, red[1][w][threadIdx.x]);
    }
    const double2 fsep = tile[mi];
    const double mdy2 = -1.0 / a.inv_dy2;
    double2* out = a.T + (size_t)a.rank * a.tstride + (size_t)m * a.tnum;
    out[0] = fsep;
    out[1] = cscale(t1, mdy2);
    out[2] = cscale(tn, mdy2);
    // column sum over all rows of the slab, separator included: the row r2c of the
    // slab's column-sum row (element (m, 0) of the 8-row tile spectrum a.cs) -- unless the
    // sums travel untransformed and the solve gets the total's spectrum (tnum == 3)
    if (a.tnum == 4) out[3] = a.cs[((size_t)(m >> 3) << 6) + (m & 7)];
  }
}

// Pass 1: the interior rows 1 .. rl-1 of every x-mode m >= 1 with the separator values
// s_p (row 0) and s_q (row rl, the next slab's row 0) as Dirichlet data, i.e. the
// tridiagonal system (psi[j-1] + psi[j+1]) / dy^2 + d_m psi[j] = f[j], solved directly
// (no transform), one workgroup per 8-mode tile:
//   * rows are cut into K chunks of kChunk rows: chunk k = interface row k C plus the
//     C - 1 rows after it; thread (mode mi, chunk k) solves its C - 1 rows with zero
//     boundary values by the Thomas algorithm (tabulated inverse pivots, the system scaled
//     by dy^2 so the off-diagonal is 1) -- the particular solution u;
//   * psi = u + v_k g(i) + v_{k+1} g(C - i) on chunk k, g the homogeneous solution with
//     g(0) = 1, g(C) = 0 (tabulated), v_k = psi at interface row k C (v_0 = s_p, v_K = s_q);
//   * the interface rows give a K-1 tridiagonal system in v, A v_{k-1} + B v_k + A v_{k+1}
//     = dy^2 f[kC] - u^{(k-1)}_{C-1} - u^{(k)}_1, solved by one lane per mode (tabulated
//     inverse pivots).
// Reads and writes each element once, whole 128-B tile rows per 8 lanes.  All pivots and
// coefficients are built on the host in long double from e_m = d_m + 2/dy^2 (exact), so
// the near-singular low modes lose nothing to cancellation (host_common.hpp).
constexpr int kChunk = CFDJ_SCHUR_CHUNK;

// K chunks per mode, MW modes per workgroup (8 = a whole tile; 4 = half a tile for the
// 128-chunk slabs, so MW K stays within the 1024-thread / register budget).
template <int K, int MW>
__global__ __launch_bounds__(MW * K) void schur_solve_kernel(const SchurArgs a) {
  constexpr int C = kChunk;
  constexpr int PER = 8 / MW;  // workgroups per tile
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tb = lb / PER;
  const int mi = threadIdx.x % MW, k = threadIdx.x / MW;
  const int m8 = (lb % PER) * MW + mi;  // mode within the tile
  const int m = 8 * tb + m8;
  const bool act = m >= 1;  // m = 0 (packed DC / Nyquist) is solved on the gathered column
  const int mm = act ? m : 1;
  double2* tile = a.H + (((size_t)tb * a.rl) << 3) + m8;  // row j at tile[8 j]
  __shared__ double2 fst[K][MW], lst[K][MW], rint[K][MW], V[K + 1][MW];
  __shared__ double sip[MW][C], sg[MW][C + 1];

  // this workgroup's pivots and homogeneous solutions into LDS (read in the sweeps)
  for (int t = threadIdx.x; t < MW * (2 * C + 1); t += MW * K) {
    const int w = t / (2 * C + 1), r = t % (2 * C + 1);
    const int mw = 8 * tb + (lb % PER) * MW + w;
    const int mr = mw >= 1 ? mw : 1;
    if (r < C) sip[w][r] = a.tip[(size_t)mr * C + r];
    else sg[w][r - C] = a.tg[(size_t)mr * (C + 1) + (r - C)];
  }

  // separator values s_rank, s_rank+1 from every rank's traces (as the reference's
  // periodic circulant), and the constant-mode correction
  double2 sp = make_double2(0.0, 0.0), sq = sp, fb = sp;
  const double* ci = a.cinv + (size_t)mm * a.P;
  for (int qq = 0; qq < a.P; ++qq) {
    const double2* Tq = a.T + (size_t)qq * a.tstride + (size_t)mm * a.tnum;
    const double2* Tm = a.T + (size_t)((qq + a.P - 1) % a.P) * a.tstride + (size_t)mm * a.tnum;
    const double2 rhs = csub(Tq[0], cscale(cadd(Tm[2], Tq[1]), a.inv_dy2));
    sp = cadd(sp, cscale(rhs, ci[(qq - a.rank + a.P) % a.P]));
    sq = cadd(sq, cscale(rhs, ci[(qq - a.rank - 1 + 2 * a.P) % a.P]));
    if (a.csT == nullptr) fb = cadd(fb, Tq[3]);
  }
  if (a.csT != nullptr) fb = a.csT[mm];
  const double2 cst = cscale(fb, a.corr[mm] * a.inv_ny);

  // chunk rows, scaled by dy^2
  const double sc = a.dy2;
  double2 y[C - 1];
#pragma unroll
  for (int i = 1; i < C; ++i) y[i - 1] = cscale(tile[(size_t)(k * C + i) << 3], sc);
  const double2 fint = cscale(tile[(size_t)(k * C) << 3], sc);
  __syncthreads();  // tables

  // Thomas with zero boundary values: y_i -= y_{i-1} / p_{i-1}; u_i = (y_i - u_{i+1}) / p_i
  const double* ip = sip[mi];  // 1 / p_i at [i - 1]
#pragma unroll
  for (int i = 1; i < C - 1; ++i) y[i] = csub(y[i], cscale(y[i - 1], ip[i - 1]));
  y[C - 2] = cscale(y[C - 2], ip[C - 2]);
#pragma unroll
  for (int i = C - 3; i >= 0; --i) y[i] = cscale(csub(y[i], y[i + 1]), ip[i]);
  fst[k][mi] = y[0];
  lst[k][mi] = y[C - 2];
  rint[k][mi] = fint;
  __syncthreads();

  // the K-1 interface values by parallel cyclic reduction, lane (mi, k) owning v_k:
  // a v_{k-s} + b v_k + c v_{k+s} = r, starting from (A, B, A) with v_0 = s_p and v_K = s_q
  // folded into r; every step eliminates the couplings at distance s (log2 K steps).
  // Lanes k = 0 carry the identity row.
  __shared__ double sa[K][MW], sb[K][MW], sc2[K][MW];
  {
    const double A = a.tA[mm], B = a.tB[mm];
    double ca = 0.0, cb = 1.0, cc = 0.0;
    double2 r = make_double2(0.0, 0.0);
    if (k >= 1) {
      ca = k == 1 ? 0.0 : A;
      cb = B;
      cc = k == K - 1 ? 0.0 : A;
      r = csub(rint[k][mi], cadd(lst[k - 1][mi], fst[k][mi]));
      if (k == 1) r = csub(r, cscale(sp, A));
      if (k == K - 1) r = csub(r, cscale(sq, A));
    }
#pragma unroll 1
    for (int st = 1; st < K; st <<= 1) {
      sa[k][mi] = ca;
      sb[k][mi] = cb;
      sc2[k][mi] = cc;
      V[k][mi] = r;
      __syncthreads();
      const int lo = k - st, hi = k + st;
      double al = 0.0, ga = 0.0, alo = 0.0, clo = 0.0, ahi = 0.0, chi = 0.0;
      double2 rlo = make_double2(0.0, 0.0), rhi = rlo;
      if (k >= 1 && lo >= 1) {
        al = -ca / sb[lo][mi];
        alo = sa[lo][mi];
        clo = sc2[lo][mi];
        rlo = V[lo][mi];
      }
      if (k >= 1 && hi <= K - 1) {
        ga = -cc / sb[hi][mi];
        ahi = sa[hi][mi];
        chi = sc2[hi][mi];
        rhi = V[hi][mi];
      }
      __syncthreads();
      if (k >= 1) {
        cb = cb + al * clo + ga * ahi;
        ca = al * alo;
        cc = ga * chi;
        r = cadd(r, cadd(cscale(rlo, al), cscale(rhi, ga)));
      }
    }
    V[k][mi] = k >= 1 ? make_double2(r.x / cb, r.y / cb) : sp;
    if (k == 0) V[K][mi] = sq;
  }
  __syncthreads();

  if (!act) return;
  const double s = a.out_scale;
  const double2 v0 = V[k][mi], v1 = V[k + 1][mi];
  const double* g = sg[mi];
  // psi-hat of the two rows just outside the slab: the next slab's separator value is known
  // here (s_q), the previous slab's last row follows from the operator's equation at this
  // slab's separator row, psi[-1] + psi[1] - (2 + ep) psi[0] = dy^2 f[0] (f[0] from the
  // interface buffer, psi[1] formed here: nothing stays in registers for it)
  if (a.halo8 != nullptr && k == 0) {
    const double2 p1 = cadd(y[0], cadd(cscale(v0, g[1]), cscale(v1, g[C - 1])));
    const double2 lo = csub(cadd(rint[0][mi], cscale(v0, a.tD[mm])), p1);
    const double2 hi = V[K][mi];
    double2* h8 = a.halo8 + (((size_t)tb * 8) << 3) + m8;  // row j at h8[8 j]
    h8[0] = make_double2((lo.x + cst.x) * s, (lo.y + cst.y) * s);
    h8[8] = make_double2((hi.x + cst.x) * s, (hi.y + cst.y) * s);
  }
  tile[(size_t)(k * C) << 3] = make_double2((v0.x + cst.x) * s, (v0.y + cst.y) * s);
#pragma unroll
  for (int i = 1; i < C; ++i) {
    const double2 p = cadd(y[i - 1], cadd(cscale(v0, g[i]), cscale(v1, g[C - i])));
    tile[(size_t)(k * C + i) << 3] = make_double2((p.x + cst.x) * s, (p.y + cst.y) * s);
  }
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

template <int K>
void launch_schur_n(int pass, const SchurArgs& a, hipStream_t st) {
  if (pass == 0)
    hipLaunchKernelGGL(schur_trace_kernel, dim3(a.L / kTraceModes), dim3(kTraceThreads), 0, st, a);
  else
  {
#ifndef CFDJ_SCHUR_MW64
#define CFDJ_SCHUR_MW64 4
#endif
#ifndef CFDJ_SCHUR_MW128
#define CFDJ_SCHUR_MW128 4
#endif
    constexpr int MW = K >= 256 ? 4 : K >= 128 ? CFDJ_SCHUR_MW128 : (K >= 64 ? CFDJ_SCHUR_MW64 : 8);
    hipLaunchKernelGGL((schur_solve_kernel<K, MW>), dim3(a.L / MW), dim3(MW * K), 0, st, a);
  }
}

}  // namespace

// Slab heights of 16 .. 128 chunks (one workgroup of 8 K <= 1024 threads per tile).
bool schur_supported(int rl) { return rl == 512 || rl == 1024 || rl == 2048 || rl == 4096; }

void launch_schur_pass(int pass, const SchurArgs& a, hipStream_t st) {
  if (!schur_supported(a.rl) || a.L < 8 || a.L % 8 != 0 || !a.tile8 || a.P < 1 ||
      a.rank < 0 || a.rank >= a.P)
    throw Error{CFDJ_ERR_ARG, "substructured Poisson: unsupported slab"};
  switch (a.rl) {
    case 512: launch_schur_n<512 / kChunk>(pass, a, st); break;
    case 1024: launch_schur_n<1024 / kChunk>(pass, a, st); break;
    case 2048: launch_schur_n<2048 / kChunk>(pass, a, st); break;
    case 4096: launch_schur_n<4096 / kChunk>(pass, a, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_packed_divide(const PackedDivParams& p, hipStream_t st) {
  const int n = p.ny / 2 + 1;
  hipLaunchKernelGGL(packed_divide_kernel, dim3((n + 255) / 256), dim3(256), 0, st, p);
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
