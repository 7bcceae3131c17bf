// 2-D real <-> half-spectrum transforms on grids of 3 * 2^k points a side (1536, 3072, 6144):
// the product grid of the 3/2-rule solver (21_NS2D_PseudoSpectral_32_Rule/
// pseudospectral_32_rule.jl:124-125 pads nx to 1.5 nx), which the power-of-two passes of
// poisson_fft.hip / fft2d_r2c.hip do not cover.
//
// A transform of length L = 3 L3 (L3 a power of two) is three independent length-L3 Stockham
// transforms (the radix-16 plans of fft_lds.hpp) of the decimated inputs x[3 n + r], one per
// third of the workgroup's team, followed by the L3 radix-3 butterflies of a decimation-in-time
// step: X[k + s L3] = F_0[k] + w3^s W_L^k F_1[k] + w3^2s W_L^2k F_2[k], s < 3.  The team's LDS
// buffer holds one double per element (real and imaginary parts pass through it one after the
// other, as in the column pass of the Poisson solver): it serves as the three sub-transforms'
// exchange buffers, as the exchange of the radix-3 step (a thread reads the three F_r[k] of
// each of its five or six butterflies), and as the natural-order buffer of the (m, L - m)
// pairs of the real-transform pre/post-processing.
//
// The 3/2-rule solver's own kernels are here too: column passes that pad and form the
// derivative spectra on load / unpad on store (cols3_ps32_*), and the row kernel that keeps
// the fourth field and the product in the workgroup (rows3_jac_kernel).
//
// Layout of the half spectrum between the passes: column-major, element (m, y) at m n + y
// (ky contiguous), columns m = 0 .. mmax only -- the padded spectrum is zero beyond the
// unpadded grid's Nyquist column, so neither pass touches those columns.  Slot 0 of a row's
// packed spectrum holds X[0] alone: the padded grid's own Nyquist mode is zero on the way in
// and dropped on the way out (pseudospectral_32_rule.jl:171-178 does not unpad it).
//
// Both directions are unnormalised, like the library transforms they stand in for.
#pragma clang fp contract(fast)
#include "fft_lds.hpp"

namespace cfdj {

namespace {

// exp(-2 pi i j / 32), j < 8: the real-transform post-processing's W_N^m of pair i is that of
// pair 0 times this constant (m = m0 + TT i, TT / N = 1/32): one table load per thread instead
// of one per pair.  (The radix-3 step's twiddles use exp(-2 pi i b / 16) of fft_lds.hpp the
// same way.)
__device__ constexpr double kC32[8] = {1.0, 0.98078528040323043, 0.92387953251128674,
                                       0.83146961230254524, 0.70710678118654757,
                                       0.55557023301960229, 0.38268343236508984,
                                       0.19509032201612833};
__device__ constexpr double kS32[8] = {0.0, 0.19509032201612825, 0.38268343236508978,
                                       0.55557023301960218, 0.70710678118654746,
                                       0.83146961230254524, 0.92387953251128674,
                                       0.98078528040323043};

template <int L3>
struct Cfg3 {
  static constexpr int L = 3 * L3;
  static constexpr int T3 = Plan<L3>::T;       // threads per sub-transform
  static constexpr int TT = 3 * T3;            // threads per transform (team)
  static constexpr int PAD3 = Plan<L3>::PAD;   // doubles per sub-transform buffer
  static constexpr int PADL = 3 * PAD3;        // doubles per team buffer (>= padx(L - 1) + 1)
  static_assert(Plan<L3>::NSTAGES >= 2 && Plan<L3>::radix(0) == 16, "sub-transform length");
};

// The sub-transform of branch q on its decimated inputs in v (v[r] = x[3 (tid + T3 r) + q]);
// on return v holds F_q[k] at the last stage's output positions k.
template <int L3, int DIR>
__device__ __forceinline__ void sub_fft(double* team_buf, double2 (&v)[16], int q, int tid,
                                        const double2* __restrict__ tw3_) {
  const TwGlobal<L3> tw3{tw3_};
  stage_regs<L3, 0, DIR>(v, tid, tw3);
  run_stages_half<L3, 1, DIR>(team_buf + q * Cfg3<L3>::PAD3, v, tid, tw3);
}

// The radix-3 step: the three sub-transforms' outputs F_r[k] (in v, r = q) -> the team's
// L3 radix-3 butterflies X[k + s L3] = F_0[k] + w3^s W_L^k F_1[k] + w3^2s W_L^2k F_2[k], s < 3
// (w3 = exp(-+2 pi i / 3); conjugated twiddles for the inverse).  Butterfly k belongs to the
// team's thread tt = q T3 + tid = k mod TT: five butterflies per thread, k = tt + TT b, b < 5,
// and a sixth (b = 5) in the first sub-team, q = 0 (L3 = 5 TT + T3).  out[3 b + s] =
// X[tt + TT b + s L3]: consecutive lanes hold consecutive elements.  The F_r go through the
// team buffer one component at a time (F_r[k] at r L3 + k).  W_L^k = W_L^tt times the
// constant W_16^b (TT / L = 1/16): one table load per thread.
// Offset of a thread's butterfly b from its butterfly 0.  Outside the first sub-team there is
// no sixth: b = 5 maps to butterfly 0 again, so the register arrays are filled and used
// without predication (a predicated element of a register array costs a select per element
// and its registers twice); only stores of out[15..17] are guarded, by has3(b, q).
template <int L3>
__device__ __forceinline__ int boff3(int b, int q) {
  return b < 5 ? Cfg3<L3>::TT * b : (q == 0 ? 5 * Cfg3<L3>::TT : 0);
}
__device__ __forceinline__ bool has3(int b, int q) { return b < 5 || q == 0; }

template <int L3, int DIR>
__device__ __forceinline__ void combine3(double* team_buf, const double2 (&v)[16], int q,
                                         int tid, const double2* __restrict__ twL,
                                         double2 (&out)[18]) {
  using C = Cfg3<L3>;
  using P = Plan<L3>;
  static_assert(5 * C::TT + C::T3 == L3, "butterflies per thread");
  constexpr int SL = P::NSTAGES - 1;
  constexpr int RL = P::radix(SL);
  const int tt = q * C::T3 + tid;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();  // the buffer's previous readers
#pragma unroll
    for (int b = 0; b < 16 / RL; ++b)
#pragma unroll
      for (int r = 0; r < RL; ++r)
        team_buf[padx(q * L3 + out_pos<L3, SL>(tid, b, r))] = c ? v[b * RL + r].y : v[b * RL + r].x;
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int k = tt + boff3<L3>(b, q);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double f = team_buf[padx(r * L3 + k)];
        if (c) out[3 * b + r].y = f;
        else out[3 * b + r].x = f;
      }
    }
  }
  double2 cb = twL[tt];  // W_L^tt
  if (DIR > 0) cb.y = -cb.y;
  constexpr double h3 = 0.8660254037844386;  // sqrt(3) / 2
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    // (b = 5 outside the first sub-team: butterfly 0 again with another twiddle -- unused)
    const double2 w1 = cmul(cb, make_double2(kC16[b], DIR < 0 ? -kS16[b] : kS16[b]));
    const double2 w2 = cmul(w1, w1);
    const double2 f0 = out[3 * b], t1 = cmul(out[3 * b + 1], w1), t2 = cmul(out[3 * b + 2], w2);
    const double2 sm = cadd(t1, t2), df = csub(t1, t2);
    const double2 m = make_double2(f0.x - 0.5 * sm.x, f0.y - 0.5 * sm.y);
    // -+ i (sqrt(3) / 2) (t1 - t2)
    const double2 rot = DIR < 0 ? make_double2(h3 * df.y, -h3 * df.x)
                                : make_double2(-h3 * df.y, h3 * df.x);
    out[3 * b] = cadd(f0, sm);
    out[3 * b + 1] = cadd(m, rot);
    out[3 * b + 2] = csub(m, rot);
  }
}

// ---- columns: one contiguous column of M = 3 M3 elements per workgroup, in place -----------
#ifndef CFDJ_COLS3_WAVES
#define CFDJ_COLS3_WAVES 4  // > 0: wavefronts per SIMD the kernel is compiled for
#endif
#if CFDJ_COLS3_WAVES > 0
#define CFDJ_COLS3_ATTR __attribute__((amdgpu_waves_per_eu(CFDJ_COLS3_WAVES, CFDJ_COLS3_WAVES)))
#else
#define CFDJ_COLS3_ATTR
#endif
template <int M3, int DIR>
__global__ __launch_bounds__((Cfg3<M3>::TT)) CFDJ_COLS3_ATTR void cols3_kernel(
    double2* __restrict__ data, const double2* __restrict__ tw3,
    const double2* __restrict__ twM) {
  using C = Cfg3<M3>;
  __shared__ double lds[C::PADL];
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  double2* col = data + (size_t)id * C::L;
  const int t = threadIdx.x, q = t / C::T3, tid = t % C::T3;
  double2 v[16];
  // the three sub-teams' loads interleave element by element: together whole lines
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = col[(unsigned)(3 * (tid + C::T3 * r) + q)];
  sub_fft<M3, DIR>(lds, v, q, tid, tw3);
  double2 o[18];
  combine3<M3, DIR>(lds, v, q, tid, twM, o);
  // (the DC column of a real field's spectrum transforms to real values up to round-off; the
  // inverse row pass reads the real parts of column 0 only)
#pragma unroll
  for (int b = 0; b < 6; ++b)
    if (has3(b, q))
#pragma unroll
      for (int r = 0; r < 3; ++r) col[(unsigned)(t + C::TT * b + r * M3)] = o[3 * b + r];
}

// ---- columns of the 3/2-rule solver on the half spectrum of its unpadded grid ---------------
// State layout: columns m = 0..N/2 of N = 2 M3 elements (ky contiguous), the modes kx index
// 0..N/2 of the spectrum, followed by the row `ex` of N/2 + 1 elements ex[m] = w_f(-m, N/2).
// The rest of the other half is conj(w_f(-kx, -ky)), as for any real field's spectrum; the ky
// index N/2 is different: the 3/2 rule's unpadding (pseudospectral_32_rule.jl:171-178) fills it
// with the padded grid's mode -N/2, which on that grid is not its own conjugate twin, so
// w_f(-m, N/2) and conj(w_f(m, N/2)) are independent numbers from the first Jacobian on, and
// so are w_f(N/2, j) and conj(w_f(N/2, -j)) -- column N/2 is stored whole anyway.
// The padded column has 3 M3 elements, the unpadded modes in its first and last third
// (pseudospectral_32_rule.jl:109-154).

// Inverse column pass with the four derivative spectra formed where the column is loaded:
// array arr of i kx w_f / k2, i ky w_f, i ky w_f / k2, i kx w_f (pseudospectral_32_rule.jl:
// 109-154), padded, times `scale` = (nxe nye) / (nx ny).  real(ifft(.)) keeps the Hermitian
// part (P(a, b) + conj P(-a, -b)) / 2 of the padded array P; at the padded element p of column
// a0 that is (i/2) (kappa(a0, j) w_f(a0, j) - kappa(-a0, -j) conj w_f(-a0, -j)) (/ k2), j the
// unpadded mode at p, each term present only where the padding puts that mode: the index N/2
// is the mode -N/2 and sits on the negative side only (so column N/2 and the element 2 M3 have
// no first term, the element M3 -- the twin of the other side's 2 M3 -- no second), and kappa
// is not odd at index 0 (kx[1] = eps, Common.jl:199).  EDGE = the columns 0 and N/2, which hold
// both w_f(a0, j) and w_f(-a0, -j) = w_f(a0, -j); elsewhere the second is the conjugate of the
// first, except at the element M3, where it is ex[a0].
template <int M3, bool EDGE>
__device__ __forceinline__ void ps32_load_column(double2 (&v)[16], const double2* __restrict__ col,
                                                 double2 ex, const double* __restrict__ kx, int a0,
                                                 int arr, int q, int tid, double scale) {
#pragma clang fp contract(off)
  using C = Cfg3<M3>;
  constexpr int N = 2 * M3, H = M3;
  const bool fp = a0 < H;
  const double kxa = kx[a0], kxm = kx[(N - a0) & (N - 1)];
  // the table's entries (Common.jl:190-199: kx[1] = eps, else h times the signed index) formed
  // from kx[0] and kx[1] = h instead of two more loads per element
  const double eps = kx[0], h = kx[1];
  const bool xder = arr == 0 || arr == 3, overk2 = arr == 0 || arr == 2;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = 3 * (tid + C::T3 * r) + q;
    const bool kept = p <= H || p >= 2 * H;
    const int j = p <= H ? p : p - H;  // (the middle third maps to a valid index, unused)
    const int jm = (N - j) & (N - 1);
    const double kyj = j == 0 ? eps : h * (double)(j < H ? j : j - N);
    const double kym = jm == 0 ? eps : h * (double)(jm < H ? jm : jm - N);
    const double kap_p = fp && p != H ? (xder ? kxa : kyj) : 0.0;
    const double kap_m = p != 2 * H ? (xder ? kxm : kym) : 0.0;
    double2 u;  // kappa(a0, j) w_f(a0, j) - kappa(-a0, -j) conj(w_f(-a0, -j))
    if constexpr (EDGE) {
      const double2 w0 = col[j], w1 = col[jm];
      u = make_double2(kap_p * w0.x - kap_m * w1.x, kap_p * w0.y + kap_m * w1.y);
    } else {
      double2 w = col[j];
      if (p == H) w = make_double2(ex.x, -ex.y);
      const double keff = kap_p - kap_m;
      u = make_double2(keff * w.x, keff * w.y);
    }
    double f = 0.5 * scale;
    if (overk2) f = f * recip_nr(kxa * kxa + kyj * kyj);
    v[r] = kept ? make_double2(f * -u.y, f * u.x) : make_double2(0.0, 0.0);  // i u f
  }
}

template <int M3>
__global__ __launch_bounds__((Cfg3<M3>::TT)) CFDJ_COLS3_ATTR void cols3_ps32_in_kernel(
    const double2* __restrict__ hs, double2* __restrict__ x, const double* __restrict__ kx,
    double scale, const double2* __restrict__ tw3, const double2* __restrict__ twM) {
  using C = Cfg3<M3>;
  constexpr int N = 2 * M3;
  __shared__ double lds[C::PADL];
  // the four arrays of a column are neighbours (one XCD): the column comes from HBM once
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int a0 = __builtin_amdgcn_readfirstlane(id >> 2), arr = id & 3;
  const double2* col = hs + (size_t)a0 * N;
  const double2 ex = hs[(size_t)(M3 + 1) * N + a0];
  const int t = threadIdx.x, q = t / C::T3, tid = t % C::T3;
  double2 v[16];
  if (a0 == 0 || a0 == M3) ps32_load_column<M3, true>(v, col, ex, kx, a0, arr, q, tid, scale);
  else ps32_load_column<M3, false>(v, col, ex, kx, a0, arr, q, tid, scale);
  sub_fft<M3, 1>(lds, v, q, tid, tw3);
  double2 o[18];
  combine3<M3, 1>(lds, v, q, tid, twM, o);
  double2* out = x + ((size_t)arr * (M3 + 1) + a0) * C::L;  // (wave-uniform)
#pragma unroll
  for (int b = 0; b < 6; ++b)
    if (has3(b, q))
#pragma unroll
      for (int r = 0; r < 3; ++r) out[(unsigned)(t + C::TT * b + r * M3)] = o[3 * b + r];
}

// Forward column pass with the unpadding of pseudospectral_32_rule.jl:171-178 where the column
// is stored, times `scale` = (nx ny) / (nxe nye): the first third of the padded column a0 is
// the state's modes 0..N/2-1 of that column, the last third its modes N/2..N-1; the middle
// third is dropped but for its first element M3, the mode (a0, +N/2), whose conjugate is the
// state's ex[a0] = (-a0, -N/2).  The state's column N/2 is the mode -N/2: mode j there is the
// conjugate of the element -b(j) of the padded column N/2, b(j) the padded index of mode j.
template <int M3>
__global__ __launch_bounds__((Cfg3<M3>::TT)) CFDJ_COLS3_ATTR void cols3_ps32_out_kernel(
    const double2* __restrict__ x, double2* __restrict__ hs, double scale,
    const double2* __restrict__ tw3, const double2* __restrict__ twM) {
  using C = Cfg3<M3>;
  constexpr int N = 2 * M3, H = M3;
  __shared__ double lds[C::PADL];
  const int a0 = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  const double2* col = x + (size_t)a0 * C::L;
  const int t = threadIdx.x, q = t / C::T3, tid = t % C::T3;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = col[(unsigned)(3 * (tid + C::T3 * r) + q)];
  sub_fft<M3, -1>(lds, v, q, tid, tw3);
  double2 o[18];
  combine3<M3, -1>(lds, v, q, tid, twM, o);
  double2* out = hs + (size_t)a0 * N;
  double2* ex = hs + (size_t)(M3 + 1) * N;
  // butterfly k = t + TT b holds the padded elements k (first third), k + M3 (middle third)
  // and k + 2 M3 (last third)
  if (a0 != H) {
#pragma unroll
    for (int b = 0; b < 6; ++b)
      if (has3(b, q)) {
        const int k = t + C::TT * b;
        out[k] = make_double2(o[3 * b].x * scale, o[3 * b].y * scale);
        out[k + M3] = make_double2(o[3 * b + 2].x * scale, o[3 * b + 2].y * scale);
      }
    if (t == 0) ex[a0] = make_double2(o[1].x * scale, -o[1].y * scale);  // element M3
  } else {
    // element p goes to j = -p of the first and the last third; the padding puts -b = N/2 in
    // the last third's twin only: element M3 -> j = N/2 (and ex[N/2], the same mode)
#pragma unroll
    for (int b = 0; b < 6; ++b)
      if (has3(b, q)) {
        const int k = t + C::TT * b;
        out[(N - k) & (N - 1)] = make_double2(o[3 * b].x * scale, -o[3 * b].y * scale);
        if (k != 0) out[M3 - k] = make_double2(o[3 * b + 2].x * scale, -o[3 * b + 2].y * scale);
      }
    if (t == 0) out[H] = ex[H] = make_double2(o[1].x * scale, -o[1].y * scale);
  }
}

// Pair i of a thread in a row workgroup of XR teams: row qq, columns m and L - m; 16
// consecutive lanes take 16 consecutive m of one row (whole XR * 16-B column segments).
template <int L3, int XR>
__device__ __forceinline__ void pair3(int tx, int i, int& qq, int& m) {
  const int e = tx + i * (XR * Cfg3<L3>::TT);
  qq = (e >> 4) % XR;
  m = ((e >> 4) / XR) * 16 + (e & 15);
}

// ---- rows, half spectrum -> real (c2r): XR rows per workgroup ------------------------------
#ifndef CFDJ_ROWS3_INV_WAVES
#define CFDJ_ROWS3_INV_WAVES 4  // > 0: wavefronts per SIMD the kernel is compiled for
#endif
#if CFDJ_ROWS3_INV_WAVES > 0
#define CFDJ_ROWS3_INV_ATTR \
  __attribute__((amdgpu_waves_per_eu(CFDJ_ROWS3_INV_WAVES, CFDJ_ROWS3_INV_WAVES)))
#else
#define CFDJ_ROWS3_INV_ATTR
#endif

// The rows y0 .. y0 + XR - 1 of the half spectrum H (M rows, columns 0..mmax) -> the thread's
// complex outputs o[3 b + s] = (f[2p], f[2p + 1]), p = t + TT b + s L3 (t the thread's index in
// its team; b < 5, and b = 5 where q = 0: combine3), of row y0 + team.
template <int L3, int XR>
__device__ __forceinline__ void c2r_rows3(const double2* __restrict__ H, int M, int mmax, int y0,
                                          double* lds, int tx, const double2* __restrict__ tw3,
                                          const double2* __restrict__ twL,
                                          const double2* __restrict__ twN, double2 (&o)[18]) {
  using C = Cfg3<L3>;
  constexpr int L = C::L, THREADS = XR * C::TT, PAIRS = (L / 2) * XR / THREADS;
  static_assert(PAIRS * THREADS == (L / 2) * XR, "pair mapping");
  const int team = tx / C::TT, t = tx % C::TT, q = t / C::T3, tid = t % C::T3;
  double* buf = lds + team * C::PADL;
  const double2* base = H + __builtin_amdgcn_readfirstlane(y0);
  // c2r pre-processing of the pairs (m, L - m): Z[m] = (X[m] + conj X[L-m]) + i W_N^-m (X[m] -
  // conj X[L-m]); slot 0 = X[0] (the Nyquist mode of this grid is zero), Z[L/2] = 2 conj X[L/2]
  static_assert(PAIRS == 8, "pair twiddle table");
  double2 o1[PAIRS], o2[PAIRS];
  double2 wn0 = make_double2(1.0, 0.0);
#pragma unroll
  for (int i = 0; i < PAIRS; ++i) {
    int qq, m;
    pair3<L3, XR>(tx, i, qq, m);
    const bool z0 = i == 0 && m == 0;
    const int mq = z0 ? L / 2 : L - m;
    double2 Xm = make_double2(0.0, 0.0), Xq = Xm;
    if (m <= mmax) Xm = base[(unsigned)(m * M + qq)];
    if (mq <= mmax) Xq = base[(unsigned)(mq * M + qq)];
    const double2 Xp = cconj(Xq);
    const double2 S = cadd(Xm, Xp);
    if (i == 0) wn0 = cconj(twN[m]);  // W_N^-m of pair 0; pair i: m + TT i
    const double2 D = cmul(cmul(wn0, make_double2(kC32[i], kS32[i])), csub(Xm, Xp));
    o1[i] = make_double2(S.x - D.y, S.y + D.x);
    o2[i] = make_double2(S.x + D.y, D.x - S.y);
    if (z0) {
      o1[i] = make_double2(Xm.x, Xm.x);  // (X[0] + X[L], X[0] - X[L]) with X[L] = 0
      o2[i] = make_double2(2.0 * Xq.x, -2.0 * Xq.y);
    }
  }
  // through the natural-order buffer one component at a time, read back as the
  // sub-transforms' decimated inputs
  double2 v[16];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c) __syncthreads();
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      int qq, m;
      pair3<L3, XR>(tx, i, qq, m);
      double* bq = lds + qq * C::PADL;
      bq[padx(m)] = c ? o1[i].y : o1[i].x;
      bq[padx(i == 0 && m == 0 ? L / 2 : L - m)] = c ? o2[i].y : o2[i].x;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const double a = buf[padx(3 * (tid + C::T3 * r) + q)];
      if (c) v[r].y = a;
      else v[r].x = a;
    }
  }
  sub_fft<L3, 1>(buf, v, q, tid, tw3);
  combine3<L3, 1>(buf, v, q, tid, twL, o);
}

template <int L3, int XR, bool NTS>
__global__ __launch_bounds__((XR * Cfg3<L3>::TT)) CFDJ_ROWS3_INV_ATTR void rows3_inv_kernel(
    const double2* __restrict__ H, double* __restrict__ f, int M, int mmax,
    const double2* __restrict__ tw3, const double2* __restrict__ twL,
    const double2* __restrict__ twN, size_t hstride, size_t fstride) {
  using C = Cfg3<L3>;
  constexpr int L = C::L;
  __shared__ double lds[XR * C::PADL];
  const int team = threadIdx.x / C::TT, t = threadIdx.x % C::TT, q = t / C::T3;
  const int y0 = xcd_remap(blockIdx.x, gridDim.x) * XR;
  // blockIdx.y: the array of a batch (one launch for all of them: one tail instead of one each)
  H += blockIdx.y * hstride;
  f += blockIdx.y * fstride;
  double2 o[18];
  c2r_rows3<L3, XR>(H, M, mmax, y0, lds, threadIdx.x, tw3, twL, twN, o);
  // (a wave-uniform base and 32-bit element offsets: one offset register per access)
  double2* z = reinterpret_cast<double2*>(f) + (size_t)__builtin_amdgcn_readfirstlane(y0) * L;
#pragma unroll
  for (int b = 0; b < 6; ++b)
    if (has3(b, q))
#pragma unroll
      for (int r = 0; r < 3; ++r)
        store_stream<NTS>(z + (unsigned)(team * L + t + C::TT * b + r * L3), o[3 * b + r]);
}

// ---- rows, real -> half spectrum (r2c): XR rows per workgroup ------------------------------
// The thread's decimated inputs v[r] = (f[2p], f[2p + 1]), p = 3 (tid + T3 r) + q, of row
// y0 + team -> the columns 0..mmax of rows y0 .. y0 + XR - 1 of the half spectrum H.
template <int L3, int XR>
__device__ __forceinline__ void r2c_rows3(double2 (&v)[16], double2* __restrict__ H, int M,
                                          int mmax, int y0, double* lds, int tx,
                                          const double2* __restrict__ tw3,
                                          const double2* __restrict__ twL,
                                          const double2* __restrict__ twN) {
  using C = Cfg3<L3>;
  constexpr int L = C::L, THREADS = XR * C::TT, PAIRS = (L / 2) * XR / THREADS;
  const int team = tx / C::TT, t = tx % C::TT, q = t / C::T3, tid = t % C::T3;
  double* buf = lds + team * C::PADL;
  sub_fft<L3, -1>(buf, v, q, tid, tw3);
  double2 o[18];
  combine3<L3, -1>(buf, v, q, tid, twL, o);
  // natural order through the buffer, read back as the pairs (m, L - m) of the r2c
  // post-processing
  double2 Zm[PAIRS], Zp[PAIRS];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 6; ++b)
      if (has3(b, q))
#pragma unroll
        for (int r = 0; r < 3; ++r)
          buf[padx(t + C::TT * b + r * L3)] = c ? o[3 * b + r].y : o[3 * b + r].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      int qq, m;
      pair3<L3, XR>(tx, i, qq, m);
      const double* bq = lds + qq * C::PADL;
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
  double2* hb = H + __builtin_amdgcn_readfirstlane(y0);
  static_assert(PAIRS == 8, "pair twiddle table");
  double2 wn0 = make_double2(1.0, 0.0);
#pragma unroll
  for (int i = 0; i < PAIRS; ++i) {
    int qq, m;
    pair3<L3, XR>(tx, i, qq, m);
    const bool z0 = i == 0 && m == 0;
    const int mp = z0 ? L / 2 : L - m;
    const double2 Zc = cconj(Zp[i]);
    const double2 E = make_double2(0.5 * (Zm[i].x + Zc.x), 0.5 * (Zm[i].y + Zc.y));
    const double2 D = csub(Zm[i], Zc);
    const double2 O = make_double2(0.5 * D.y, -0.5 * D.x);
    if (i == 0) wn0 = twN[m];  // W_N^m of pair 0; pair i: m + TT i
    const double2 WO = cmul(cmul(wn0, make_double2(kC32[i], -kS32[i])), O);
    double2 o1 = cadd(E, WO);
    double2 o2 = cconj(csub(E, WO));
    if (z0) {  // slot 0 = X[0] (this grid's Nyquist mode X[L] is not kept); X[L/2] = conj Z[L/2]
      o1 = make_double2(Zm[i].x + Zm[i].y, 0.0);
      o2 = Zc;
    }
    if (m <= mmax) hb[(unsigned)(m * M + qq)] = o1;
    if (mp <= mmax) hb[(unsigned)(mp * M + qq)] = o2;
  }
}

template <int L3, int XR, bool NT>
__global__ __launch_bounds__((XR * Cfg3<L3>::TT)) CFDJ_ROWS3_INV_ATTR void rows3_fwd_kernel(
    const double* __restrict__ f, double2* __restrict__ H, int M, int mmax,
    const double2* __restrict__ tw3, const double2* __restrict__ twL,
    const double2* __restrict__ twN) {
  using C = Cfg3<L3>;
  constexpr int L = C::L;
  __shared__ double lds[XR * C::PADL];
  const int team = threadIdx.x / C::TT, t = threadIdx.x % C::TT, q = t / C::T3, tid = t % C::T3;
  const int y0 = xcd_remap(blockIdx.x, gridDim.x) * XR;
  const double2* z =
      reinterpret_cast<const double2*>(f) + (size_t)__builtin_amdgcn_readfirstlane(y0) * L;
  double2 v[16];
  // the three sub-teams' loads interleave element by element: together whole lines
#pragma unroll
  for (int r = 0; r < 16; ++r)
    v[r] = load_stream<NT>(z + (unsigned)(team * L + 3 * (tid + C::T3 * r) + q));
  r2c_rows3<L3, XR>(v, H, M, mmax, y0, lds, threadIdx.x, tw3, twL, twN);
}

// ---- rows of the 3/2-rule solver's product (pseudospectral_32_rule.jl:156-169) ---------------
// The fourth field's inverse row pass, the product j1 j2 - j3 j4 with the three fields already
// in physical space (R: three arrays of n x n reals) and the product's forward row pass in one
// kernel: a row of the fourth field and of the product never leaves the workgroup.  Each
// factor is scaled by inv_np = 1 / (nxe nye) first, as the reference's ifft does.
#ifndef CFDJ_ROWS3_JAC_WAVES
#define CFDJ_ROWS3_JAC_WAVES 3
#endif
template <int L3, int XR, bool NT>
__global__ __launch_bounds__((XR * Cfg3<L3>::TT))
    __attribute__((amdgpu_waves_per_eu(CFDJ_ROWS3_JAC_WAVES, CFDJ_ROWS3_JAC_WAVES))) void rows3_jac_kernel(
        const double2* __restrict__ H4, const double* __restrict__ R, double2* __restrict__ Hout,
        int M, int mmax, double inv_np, const double2* __restrict__ tw3,
        const double2* __restrict__ twL, const double2* __restrict__ twN) {
  using C = Cfg3<L3>;
  constexpr int L = C::L;
  __shared__ double lds[XR * C::PADL];
  const int y0 = xcd_remap(blockIdx.x, gridDim.x) * XR;
  double2 o[18];
  c2r_rows3<L3, XR>(H4, M, mmax, y0, lds, threadIdx.x, tw3, twL, twN, o);
  // Each phase below works from its own opaque copy of the thread index, so that what depends
  // only on it (pair offsets, buffer addresses, twiddles) is formed again where it is used
  // instead of staying in registers from the inverse transform to the forward one; and the
  // product's loads stay behind the inverse transform.
  __builtin_amdgcn_sched_barrier(0);
  int tx = threadIdx.x;
  asm volatile("" : "+v"(tx));
  {
    const int team = tx / C::TT, t = tx % C::TT, q = t / C::T3, tid = t % C::T3;
    const size_t full = (size_t)M * M;
    const double2* r1 =
        reinterpret_cast<const double2*>(R) + (size_t)__builtin_amdgcn_readfirstlane(y0) * L;
    const double2* r2 = r1 + full / 2;
    const double2* r3 = r2 + full / 2;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const unsigned kb = team * L + t + boff3<L3>(b, q);
      double2 f1[3], f2[3], f3[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        f1[u] = load_stream<NT>(r1 + (kb + u * L3));
        f2[u] = load_stream<NT>(r2 + (kb + u * L3));
        f3[u] = load_stream<NT>(r3 + (kb + u * L3));
      }
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        double2& d = o[3 * b + u];
        d.x = (f1[u].x * inv_np) * (f2[u].x * inv_np) - (f3[u].x * inv_np) * (d.x * inv_np);
        d.y = (f1[u].y * inv_np) * (f2[u].y * inv_np) - (f3[u].y * inv_np) * (d.y * inv_np);
        // formed here: left to the compiler, the imaginary parts are computed where the exchange
        // below first uses them, and their 3 x 18 factors stay in registers until then
        asm volatile("" : "+v"(d.x), "+v"(d.y));
      }
    }
    // the product row, natural order -> the forward sub-transforms' decimated inputs
    double* buf = lds + team * C::PADL;
    double2 v[16];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      __syncthreads();
#pragma unroll
      for (int b = 0; b < 6; ++b)
        if (has3(b, q))
#pragma unroll
          for (int u = 0; u < 3; ++u)
            buf[padx(t + C::TT * b + u * L3)] = c ? o[3 * b + u].y : o[3 * b + u].x;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const double a = buf[padx(3 * (tid + C::T3 * r) + q)];
        if (c) v[r].y = a;
        else v[r].x = a;
      }
    }
    __syncthreads();  // the buffer's readers, before the sub-transforms' exchanges write it
    __builtin_amdgcn_sched_barrier(0);
    int tx2 = tx;
    asm volatile("" : "+v"(tx2));
    r2c_rows3<L3, XR>(v, Hout, M, mmax, y0, lds, tx2, tw3, twL, twN);
  }
}

// Rows per workgroup.  Measured at 6144^2 (4 steps of the 3/2-rule solver at 4096^2, rocprofv3):
// the inverse pass takes 200 us per array with 1, 2 or 4 rows; the forward pass 275 / 272 /
// 217 us -- its column segments are written, and 64-B pieces (4 rows) merge better.
#ifndef CFDJ_ROWS3_XR
#define CFDJ_ROWS3_XR 2
#endif
#ifndef CFDJ_ROWS3_FWD_XR
#define CFDJ_ROWS3_FWD_XR 4
#endif

template <int L3>
void launch_rows3(bool fwd, const Real2d3Args& a, const double* fin, double* fout, double2* H,
                  hipStream_t st, int batch = 1) {
  constexpr int XR = CFDJ_ROWS3_XR;
  // inverse: `batch` arrays, (mmax + 1) n complex / n n reals apart
  const dim3 grid(a.n / XR, batch), block(XR * Cfg3<L3>::TT);
  const size_t hs = (size_t)(a.mmax + 1) * a.n, fs = (size_t)a.n * a.n;
  if (fwd) {
    constexpr int XF = CFDJ_ROWS3_FWD_XR * Cfg3<L3>::TT <= 1024 ? CFDJ_ROWS3_FWD_XR : XR;
    const dim3 gridf(a.n / XF), blockf(XF * Cfg3<L3>::TT);
    if (a.stream)
      hipLaunchKernelGGL((rows3_fwd_kernel<L3, XF, true>), gridf, blockf, 0, st, fin, H, a.n,
                         a.mmax, a.tw3L, a.twL, a.twN);
    else
      hipLaunchKernelGGL((rows3_fwd_kernel<L3, XF, false>), gridf, blockf, 0, st, fin, H, a.n,
                         a.mmax, a.tw3L, a.twL, a.twN);
  } else {
    if (a.stream)
      hipLaunchKernelGGL((rows3_inv_kernel<L3, XR, true>), grid, block, 0, st, H, fout, a.n,
                         a.mmax, a.tw3L, a.twL, a.twN, hs, fs);
    else
      hipLaunchKernelGGL((rows3_inv_kernel<L3, XR, false>), grid, block, 0, st, H, fout, a.n,
                         a.mmax, a.tw3L, a.twL, a.twN, hs, fs);
  }
}

#ifndef CFDJ_ROWS3_JAC_XR
#define CFDJ_ROWS3_JAC_XR 4
#endif
template <int L3>
void launch_rows3_jac(const Real2d3Args& a, const double2* x4, const double* r, double2* xj,
                      double inv_np, hipStream_t st) {
  constexpr int XJ = CFDJ_ROWS3_JAC_XR * Cfg3<L3>::TT <= 1024 ? CFDJ_ROWS3_JAC_XR : CFDJ_ROWS3_XR;
  const dim3 grid(a.n / XJ), block(XJ * Cfg3<L3>::TT);
  if (a.stream)
    hipLaunchKernelGGL((rows3_jac_kernel<L3, XJ, true>), grid, block, 0, st, x4, r, xj, a.n, a.mmax,
                       inv_np, a.tw3L, a.twL, a.twN);
  else
    hipLaunchKernelGGL((rows3_jac_kernel<L3, XJ, false>), grid, block, 0, st, x4, r, xj, a.n,
                       a.mmax, inv_np, a.tw3L, a.twL, a.twN);
}

template <int M3>
void launch_cols3(bool fwd, const Real2d3Args& a, double2* x, int batch, hipStream_t st) {
  const int ncols = a.mmax + 1;
  const dim3 grid((unsigned)(ncols * batch)), block(Cfg3<M3>::TT);
  if (fwd) hipLaunchKernelGGL((cols3_kernel<M3, -1>), grid, block, 0, st, x, a.tw3M, a.twN);
  else hipLaunchKernelGGL((cols3_kernel<M3, 1>), grid, block, 0, st, x, a.tw3M, a.twN);
}

template <int M3>
void launch_cols3_ps32(bool fwd, const Real2d3Args& a, const Ps32HalfArgs& s, const double2* src,
                       double2* dst, hipStream_t st) {
  const dim3 block(Cfg3<M3>::TT);
  if (fwd)
    hipLaunchKernelGGL((cols3_ps32_out_kernel<M3>), dim3((unsigned)(M3 + 1)), block, 0, st, src,
                       dst, s.scale_out, a.tw3M, a.twN);
  else
    hipLaunchKernelGGL((cols3_ps32_in_kernel<M3>), dim3((unsigned)(4 * (M3 + 1))), block, 0, st,
                       src, dst, s.kx, s.scale_in, a.tw3M, a.twN);
}

void check3(const Real2d3Args& a) {
  if (!real2d3_supported(a.n) || a.mmax < 0 || a.mmax >= a.n / 2 || a.n % CFDJ_ROWS3_XR != 0 ||
      a.n % CFDJ_ROWS3_FWD_XR != 0 || a.n % CFDJ_ROWS3_JAC_XR != 0)
    throw Error{CFDJ_ERR_ARG, "3 * 2^k transform: unsupported size"};
}

}  // namespace

bool real2d3_supported(int n) { return n == 1536 || n == 3072 || n == 6144; }

void launch_c2r2d3(const Real2d3Args& a, double2* x, double* r, int batch, hipStream_t st) {
  check3(a);
  switch (a.n) {
    case 1536: launch_cols3<512>(false, a, x, batch, st); break;
    case 3072: launch_cols3<1024>(false, a, x, batch, st); break;
    default: launch_cols3<2048>(false, a, x, batch, st); break;
  }
  CFDJ_HIP(hipGetLastError());
  if (batch < 1) return;
  switch (a.n) {
    case 1536: launch_rows3<256>(false, a, nullptr, r, x, st, batch); break;
    case 3072: launch_rows3<512>(false, a, nullptr, r, x, st, batch); break;
    default: launch_rows3<1024>(false, a, nullptr, r, x, st, batch); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_r2c2d3(const Real2d3Args& a, const double* r, double2* x, hipStream_t st) {
  check3(a);
  switch (a.n) {
    case 1536:
      launch_rows3<256>(true, a, r, nullptr, x, st);
      launch_cols3<512>(true, a, x, 1, st);
      break;
    case 3072:
      launch_rows3<512>(true, a, r, nullptr, x, st);
      launch_cols3<1024>(true, a, x, 1, st);
      break;
    default:
      launch_rows3<1024>(true, a, r, nullptr, x, st);
      launch_cols3<2048>(true, a, x, 1, st);
      break;
  }
  CFDJ_HIP(hipGetLastError());
}

// The 3/2-rule solver's transforms between its half-spectrum state and the padded grid.
static void check_ps32(const Real2d3Args& a) {
  check3(a);
  if (a.mmax != a.n / 3) throw Error{CFDJ_ERR_ARG, "3/2-rule transform: mmax must be n / 3"};
}

void launch_ps32_c2r2d3(const Real2d3Args& a, const Ps32HalfArgs& s, const double2* hs, double2* x,
                        double* r, int nrow, hipStream_t st) {
  check_ps32(a);
  if (nrow < 0 || nrow > 4) throw Error{CFDJ_ERR_ARG, "3/2-rule transform: bad array count"};
  switch (a.n) {
    case 1536: launch_cols3_ps32<512>(false, a, s, hs, x, st); break;
    case 3072: launch_cols3_ps32<1024>(false, a, s, hs, x, st); break;
    default: launch_cols3_ps32<2048>(false, a, s, hs, x, st); break;
  }
  CFDJ_HIP(hipGetLastError());
  if (nrow < 1) return;
  switch (a.n) {
    case 1536: launch_rows3<256>(false, a, nullptr, r, x, st, nrow); break;
    case 3072: launch_rows3<512>(false, a, nullptr, r, x, st, nrow); break;
    default: launch_rows3<1024>(false, a, nullptr, r, x, st, nrow); break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_ps32_r2c2d3(const Real2d3Args& a, const Ps32HalfArgs& s, const double* r, double2* x,
                        double2* hs, hipStream_t st) {
  check_ps32(a);
  switch (a.n) {
    case 1536:
      launch_rows3<256>(true, a, r, nullptr, x, st);
      launch_cols3_ps32<512>(true, a, s, x, hs, st);
      break;
    case 3072:
      launch_rows3<512>(true, a, r, nullptr, x, st);
      launch_cols3_ps32<1024>(true, a, s, x, hs, st);
      break;
    default:
      launch_rows3<1024>(true, a, r, nullptr, x, st);
      launch_cols3_ps32<2048>(true, a, s, x, hs, st);
      break;
  }
  CFDJ_HIP(hipGetLastError());
}

void launch_ps32_product_r2c2d3(const Real2d3Args& a, const Ps32HalfArgs& s, const double2* x4,
                                const double* r, double2* xj, double2* hs, double inv_np,
                                hipStream_t st) {
  check_ps32(a);
  switch (a.n) {
    case 1536:
      launch_rows3_jac<256>(a, x4, r, xj, inv_np, st);
      launch_cols3_ps32<512>(true, a, s, xj, hs, st);
      break;
    case 3072:
      launch_rows3_jac<512>(a, x4, r, xj, inv_np, st);
      launch_cols3_ps32<1024>(true, a, s, xj, hs, st);
      break;
    default:
      launch_rows3_jac<1024>(a, x4, r, xj, inv_np, st);
      launch_cols3_ps32<2048>(true, a, s, xj, hs, st);
      break;
  }
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
