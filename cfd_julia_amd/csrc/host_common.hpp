// Host-side helpers shared by the libcfdj.so translation units: error guard, device
// allocation, the Poisson symbol tables, rocFFT plan bundles and the fused-FFT state.
#pragma once
#include <algorithm>

#include "cfdj_internal.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>

namespace cfdj {

template <class F>
inline int guard(F&& f) {
  try {
    f();
    return CFDJ_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host allocation failed");
    return CFDJ_ERR_HIP;
  } catch (const std::exception& e) {
    set_error(e.what());
    return CFDJ_ERR_STATE;
  } catch (...) {
    set_error("unknown C++ exception");
    return CFDJ_ERR_STATE;
  }
}

inline void fft_setup() {
  static std::once_flag once;
  static rocfft_status st = rocfft_status_success;
  std::call_once(once, [] { st = rocfft_setup(); });
  CFDJ_FFT(st);
}

inline void select_device(int device) {
  if (device >= 0) CFDJ_HIP(hipSetDevice(device));
}

template <class T>
inline T* dalloc(size_t n) {
  void* p = nullptr;
  CFDJ_HIP(hipMalloc(&p, n * sizeof(T) + 16));
  return static_cast<T*>(p);
}

template <class T>
inline void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

// Common.jl:106-113 wavenumber table (0-based): kx[0] = eps, kx[m] = hx*m for m < nx/2,
// kx[m] = hx*(m - nx) for m >= nx/2, hx = 2pi/nx.
inline std::vector<double> kx_table(int nx, double eps) {
  std::vector<double> kx(nx);
  const double hx = (2.0 * M_PI) / nx;
  const int h = nx / 2;
  for (int i = 1; i <= h; ++i) {
    kx[i - 1] = hx * (double)(i - 1);
    kx[i + h - 1] = hx * (double)(i - h - 1);
  }
  kx[0] = eps;
  return kx;
}

inline void check_grid(int nx, int ny, double dx, double dy) {
  CFDJ_REQUIRE(nx >= 4 && ny >= 4, "nx and ny must be >= 4");
  CFDJ_REQUIRE(nx % 2 == 0, "nx must be even (Common.jl:108 loops to nx/2)");
  CFDJ_REQUIRE(ny <= nx, "ny > nx: Common.jl:113 aliases ky = kx (BoundsError)");
  CFDJ_REQUIRE(dx > 0 && dy > 0 && std::isfinite(dx) && std::isfinite(dy),
               "dx, dy must be positive and finite");
}

// ---- spectral symbol tables + constants (Common.jl:101-103, 119-121) ----------------
// Internal symbol kind (not in the C header): the cavity's DST-I multiplier.
constexpr int kSymbolDirichletExt = 100;

struct Symbol {
  int nx = 0, ny = 0, nxh = 0, kind = CFDJ_SYMBOL_FD;
  double aa = 0, bb = 0, cc = 0, scale = 0;
  double* cx = nullptr;  // FD: cos(kx[m]); spectral: kx[m]^2   (m < nxh)
  double* cy = nullptr;  // FD: cos(ky[n]); spectral: -ky[n]^2  (n < ny)
  double* cy_mirror = nullptr;  // ny < nx: cy[(ny - n) % ny] (see DivideParams)
  // The divide evaluates (aa + bb*cx[m]) + cc*cy[n] without FMA.
  //  FD (Common.jl:101-103,119-121):  aa + bb cos kx + cc cos ky, kx = 2pi/nx * index.
  //  spectral (fft_s.jl:18-34):       (-kx^2) - ky^2 = (0 + (-1)*kx^2) + 1*(-ky^2)
  //    with kx = 2pi/(nx dx) * index -- every extra operation is exact, so the result is
  //    bit-identical to the reference expression.
  void init(int nx_, int ny_, double dx, double dy, double eps, int kind_ = CFDJ_SYMBOL_FD) {
    nx = nx_;
    ny = ny_;
    nxh = nx / 2 + 1;
    kind = kind_;
    scale = 1.0 / ((double)nx * (double)ny);  // ifft normalisation, folded into divide
    std::vector<double> hcx(nxh), hcy(ny);
    if (kind == CFDJ_SYMBOL_FD) {
      aa = -2.0 / (dx * dx) - 2.0 / (dy * dy);
      bb = 2.0 / (dx * dx);
      cc = 2.0 / (dy * dy);
      std::vector<double> kx = kx_table(nx, eps);
      for (int m = 0; m < nxh; ++m) hcx[m] = std::cos(kx[m]);
      for (int n = 0; n < ny; ++n) hcy[n] = std::cos(kx[n]);
    } else if (kind == kSymbolDirichletExt) {
      // Odd-odd extension of a (nx/2) x (ny/2)-cell Dirichlet box onto this nx x ny
      // periodic grid: d = tx + ty with tx[m] = (2/dx^2)(cos(pi m/(nx/2)) - 1) (the
      // reference's iden denominator, lid_driven_cavity.jl:64-69), applied as e * (1/d).
      aa = 0.0;
      bb = 1.0;
      cc = 1.0;
      const int cx_cells = nx / 2, cy_cells = ny / 2;
      auto t = [](int k, int cells, double h) {
        const int kk = k <= cells ? k : 2 * cells - k;  // exact even symmetry
        return (2.0 / (h * h)) * (std::cos((M_PI * kk) / cells) - 1.0);
      };
      for (int m = 0; m < nxh; ++m) hcx[m] = t(m, cx_cells, dx);
      for (int n = 0; n < ny; ++n) hcy[n] = t(n, cy_cells, dy);
    } else {
      aa = 0.0;
      bb = -1.0;
      cc = 1.0;
      // fft_s.jl:19-27: hx = 2pi/(nx dx); kx[i] = hx(i-1), kx[i+nx/2] = hx(i - nx/2 - 1.)
      std::vector<double> kx(nx);
      const double hx = (2.0 * M_PI) / ((double)nx * dx);
      const int h = nx / 2;
      for (int i = 1; i <= h; ++i) {
        kx[i - 1] = hx * (double)(i - 1);
        kx[i + h - 1] = hx * ((double)(i - h) - 1.0);
      }
      kx[0] = eps;
      for (int m = 0; m < nxh; ++m) hcx[m] = kx[m] * kx[m];
      for (int n = 0; n < ny; ++n) hcy[n] = -(kx[n] * kx[n]);
    }
    cx = dalloc<double>(nxh);
    cy = dalloc<double>(ny);
    CFDJ_HIP(hipMemcpy(cx, hcx.data(), nxh * sizeof(double), hipMemcpyHostToDevice));
    CFDJ_HIP(hipMemcpy(cy, hcy.data(), ny * sizeof(double), hipMemcpyHostToDevice));
    if (ny != nx && kind != kSymbolDirichletExt) {  // the Dirichlet symbol is even
      std::vector<double> hm(ny);
      for (int n = 0; n < ny; ++n) hm[n] = hcy[(ny - n) % ny];
      cy_mirror = dalloc<double>(ny);
      CFDJ_HIP(hipMemcpy(cy_mirror, hm.data(), ny * sizeof(double), hipMemcpyHostToDevice));
    }
  }
  void destroy() {
    dfree(cx);
    dfree(cy);
    dfree(cy_mirror);
  }
  DivideParams divide(double2* spec, int width, int rows, int pitch, int kx_off,
                      bool neg) const {
    DivideParams p;
    p.spec = spec;
    p.cx = cx;
    p.cy = cy;
    p.cy_mirror = cy_mirror;
    p.width = width;
    p.rows = rows;
    p.pitch = pitch;
    p.kx_off = kx_off;
    p.nxh = nxh;
    p.aa = aa;
    p.bb = bb;
    p.cc = cc;
    p.scale = scale;
    p.neg = neg;
    p.recip = kind == kSymbolDirichletExt;
    return p;
  }
};

// ---- rocFFT plan bundle --------------------------------------------------------------
struct Plans {
  std::vector<rocfft_plan> plans;
  rocfft_execution_info info = nullptr;
  void* work = nullptr;
  size_t work_bytes = 0;

  rocfft_plan add(rocfft_transform_type type, rocfft_result_placement place, size_t dim,
                  const size_t* lengths, size_t batch, rocfft_plan_description desc) {
    rocfft_plan p = nullptr;
    CFDJ_FFT(rocfft_plan_create(&p, place, type, rocfft_precision_double, dim, lengths, batch,
                                desc));
    plans.push_back(p);
    size_t wb = 0;
    CFDJ_FFT(rocfft_plan_get_work_buffer_size(p, &wb));
    if (wb > work_bytes) work_bytes = wb;
    return p;
  }
  void finalize(hipStream_t st) {
    CFDJ_FFT(rocfft_execution_info_create(&info));
    CFDJ_FFT(rocfft_execution_info_set_stream(info, st));
    if (work_bytes) {
      CFDJ_HIP(hipMalloc(&work, work_bytes));
      CFDJ_FFT(rocfft_execution_info_set_work_buffer(info, work, work_bytes));
    }
  }
  void exec(rocfft_plan p, const void* in, void* out) {
    void* ib[1] = {const_cast<void*>(in)};
    void* ob[1] = {out};
    CFDJ_FFT(rocfft_execute(p, ib, out ? ob : nullptr, info));
  }
  void destroy() {
    for (auto p : plans) rocfft_plan_destroy(p);
    plans.clear();
    if (info) rocfft_execution_info_destroy(info);
    info = nullptr;
    if (work) (void)hipFree(work);
    work = nullptr;
  }
};

// exp(-2 pi i k / n), k < n, rounded from long double (x86 80-bit) arithmetic.
inline double2* twiddle_table(int n) {
  const long double pi = 3.141592653589793238462643383279502884L;
  std::vector<double2> h(n);
  for (int k = 0; k < n; ++k) {
    const long double a = 2.0L * pi * (long double)k / (long double)n;
    h[k] = make_double2((double)cosl(a), (double)-sinl(a));
  }
  double2* d = dalloc<double2>(n);
  CFDJ_HIP(hipMemcpy(d, h.data(), n * sizeof(double2), hipMemcpyHostToDevice));
  return d;
}

// Hand-written 3-pass FFT Poisson (poisson_fft.hip) state: twiddle tables.
struct Fused {
  int nx = 0, ny = 0, ncu = 256;
  double2* twL = nullptr;
  double2* twN = nullptr;
  double2* twM = nullptr;  // == twN on square grids
  bool ready() const { return twN != nullptr; }
  void init(int nx_, int ny_) {
    nx = nx_;
    ny = ny_;
    int dev = 0;
    CFDJ_HIP(hipGetDevice(&dev));
    CFDJ_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    twL = twiddle_table(nx / 2);
    twN = twiddle_table(nx);
    twM = ny == nx ? twN : twiddle_table(ny);
  }
  void destroy() {
    if (twM != twN) dfree(twM);
    dfree(twL);
    dfree(twN);
    twL = twN = twM = nullptr;
  }
  // y-slab `rank` of `nranks` (rows = ny / nranks); one GPU: rank 0 of 1, C == H.
  FusedPoissonArgs args(const Symbol& sym, const double* f, double* s, double2* H, double2* C,
                        int rows, int rank, int nranks, bool neg) const {
    FusedPoissonArgs a;
    a.nx = nx;
    a.ny = ny;
    a.rows = rows;
    a.f = f;
    a.s = s;
    a.H = H;
    a.C = C;
    a.Cout = nullptr;
    a.tile8 = 0;
    a.kb = (nx / 2) / nranks;
    a.m0 = rank * a.kb;
    int lg = 0;
    while ((1 << lg) < rows) ++lg;
    a.rl_log2 = lg;
    a.seg = (unsigned)((size_t)a.kb * rows);
    a.twL = twL;
    a.twN = twN;
    a.twM = twM;
    a.cx = sym.cx;
    a.cy = sym.cy;
    a.cy_mirror = sym.cy_mirror;
    a.aa = sym.aa;
    a.bb = sym.bb;
    a.cc = sym.cc;
    a.scale = sym.scale;
    a.neg = neg;
    a.recip = sym.kind == kSymbolDirichletExt;
    a.ncu = ncu;
    a.mmax = 0;
    a.col0 = nullptr;
    a.fx = nullptr;
    a.Hx = nullptr;
    a.wrows = nullptr;
    a.cp = nullptr;
    a.ncp = 0;
    a.csout = nullptr;
    a.hx_H = nullptr;
    a.hx_lo = a.hx_hi = nullptr;
    a.hx_c0lo = a.hx_c0hi = nullptr;
    a.stream = a.stream_out = stream_loads_pay((size_t)nx * rows * sizeof(double));
    return a;
  }
  FusedPoissonArgs args(const Symbol& sym, const double* f, double* s, double2* H,
                        bool neg) const {
    return args(sym, f, s, H, H, ny, 0, 1, neg);
  }
};

// Tables of the substructured y-slab solve (schur.hip), built in long double.
struct SchurTables {
  static constexpr int kC = CFDJ_SCHUR_CHUNK;  // chunk rows of the interior solve (schur.hip)
  int rl = 0, L = 0, P = 0, K = 0;
  double inv_dy2 = 0, dy2 = 0;
  double *cinv = nullptr, *corr = nullptr, *g = nullptr;
  double *tip = nullptr, *tg = nullptr, *tA = nullptr, *tB = nullptr, *tiq = nullptr;
  double* tD = nullptr;  // [L] 2 + ep: minus the diagonal of the operator scaled by dy^2
  int* jt = nullptr;  // [L/8] trace rows above round-off per tile
  bool ready() const { return cinv != nullptr; }
  void init(int nx, int ny, double dx, double dy, double eps, int nranks) {
    typedef long double ld;
    const ld pi = 3.141592653589793238462643383279502884L;
    P = nranks;
    rl = ny / nranks;
    L = nx / 2;
    K = rl / kC;
    const double aa = -2.0 / (dx * dx) - 2.0 / (dy * dy);
    const double bb = 2.0 / (dx * dx);
    const double cc = 2.0 / (dy * dy);
    inv_dy2 = 1.0 / (dy * dy);  // the off-diagonal: cc == 2 inv_dy2 exactly
    dy2 = (double)(1.0L / (ld)inv_dy2);
    const std::vector<double> kx = kx_table(nx, eps);
    const double ce = std::cos(kx[0]);  // reference cos(ky[1]) = cos(eps)
    std::vector<double> hc((size_t)L * P, 0.0), hr(L, 0.0);
    std::vector<double> hg((size_t)L * (rl + 1), 0.0);
    std::vector<double> hip((size_t)L * kC, 0.0), htg((size_t)L * (kC + 1), 0.0), hA(L, 0.0), hB(L, 1.0),
        hiq((size_t)L * K, 0.0), hD(L, 0.0);
    std::vector<int> hjt(L / 8, 1);
    std::vector<ld> s2(rl), qk(rl + 1);
    for (int k = 0; k <= rl; ++k) {
      const ld sn = sinl(pi * (ld)k / (ld)(2 * rl));
      qk[k] = 2.0L * sn * sn;  // 1 - cos(pi k / rl) without cancellation
    }
    for (int k = 1; k < rl; ++k) {
      const ld sn = sinl(pi * (ld)k / (ld)rl);
      s2[k] = sn * sn;
    }
    const ld dy4 = ((ld)dy * (ld)dy) * ((ld)dy * (ld)dy);
    const ld o = (ld)inv_dy2;
    // homogeneous solution with h(0) = 1, h(n) = 0 of psi[j-1] + psi[j+1] - (2 + eps) psi[j]
    // = 0, cosh th = 1 + eps/2: e^{-j th} expm1(-2(n-j) th) / expm1(-2 n th)
    auto homog = [](ld th, int n, int j) {
      return expl(-(ld)j * th) * (expm1l(-2.0L * (ld)(n - j) * th) / expm1l(-2.0L * n * th));
    };
    for (int m = 1; m < L; ++m) {  // m = 0: packed DC / Nyquist column, gathered-column FFT
      const double dm = aa + bb * std::cos(kx[m]);  // Common.jl:120 order (no FMA)
      const ld em = (ld)dm + (ld)cc;                // constant-mode eigenvalue, exact sum
      ld a1 = 0.0L, an = 0.0L;
      for (int k = 1; k < rl; ++k) {
        const ld t = s2[k] / (em - (ld)cc * qk[k]);
        a1 += t;
        an += (k & 1) ? t : -t;
      }
      a1 *= 2.0L / (ld)rl;
      an *= 2.0L / (ld)rl;
      const ld diag = (ld)dm - 2.0L * a1 / dy4, off = -an / dy4;
      std::vector<ld> mu(P);
      for (int j = 0; j < P; ++j) mu[j] = diag + 2.0L * off * cosl(2.0L * pi * j / P);
      for (int d = 0; d < P; ++d) {
        ld c = 0.0L;
        for (int j = 0; j < P; ++j) c += cosl(2.0L * pi * (ld)j * d / P) / mu[j];
        hc[(size_t)m * P + d] = (double)(c / P);
      }
      const double dref = (aa + bb * std::cos(kx[m])) + cc * ce;  // reference D(m, 0)
      hr[m] = (double)(1.0L / (ld)dref - 1.0L / em);
      // the operator scaled by dy^2 (1/o): off-diagonal 1, diagonal -(2 + ep), ep = -e_m/o
      const ld ep = -em / o;
      const ld x = ep / 2.0L;
      const ld th = log1pl(x + sqrtl(x * (x + 2.0L)));
      // gL(j) <= e^{-j th}: below 2^-64 of gL(1) beyond j = 45 / th (+2 for safety)
      const ld jcut = 45.0L / th + 2.0L;
      const int jm = jcut >= (ld)rl ? rl : (int)jcut;
      hjt[m >> 3] = std::max(hjt[m >> 3], jm);
      for (int j = 0; j <= rl; ++j)  // trace pass: gL over the slab, 8-mode tiles
        hg[(((size_t)(m >> 3)) * (rl + 1) + j) * 8 + (m & 7)] = (double)homog(th, rl, j);
      // chunk Thomas pivots p_i = -(1 + s_i): s_1 = 1 + ep, s_i = (s(1 + ep) + ep)/(1 + s)
      ld sv = 1.0L + ep;
      for (int i = 1; i < kC; ++i) {
        if (i > 1) sv = (sv * (1.0L + ep) + ep) / (1.0L + sv);
        hip[(size_t)m * kC + (i - 1)] = (double)(-1.0L / (1.0L + sv));
      }
      std::vector<ld> gc(kC + 1);
      for (int i = 0; i <= kC; ++i) {
        gc[i] = homog(th, kC, i);
        htg[(size_t)m * (kC + 1) + i] = (double)gc[i];
      }
      // interface system A v_{k-1} + B v_k + A v_{k+1}: A = g(C-1), B = -(2 + ep) + 2 g(1)
      const ld A = gc[kC - 1], B = -(2.0L + ep) + 2.0L * gc[1];
      hA[m] = (double)A;
      hB[m] = (double)B;
      hD[m] = (double)(2.0L + ep);
      ld q = B;
      for (int k = 1; k < K; ++k) {
        if (k > 1) q = B - A * A / q;
        hiq[(size_t)m * K + (k - 1)] = (double)(1.0L / q);
      }
    }
    cinv = upload(hc);
    corr = upload(hr);
    g = upload(hg);
    tip = upload(hip);
    tg = upload(htg);
    tA = upload(hA);
    tB = upload(hB);
    tiq = upload(hiq);
    tD = upload(hD);
    jt = dalloc<int>(hjt.size());
    CFDJ_HIP(hipMemcpy(jt, hjt.data(), hjt.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  static double* upload(const std::vector<double>& h) {
    double* d = dalloc<double>(h.size());
    CFDJ_HIP(hipMemcpy(d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    return d;
  }
  void destroy() {
    for (double** p : {&cinv, &corr, &g, &tip, &tg, &tA, &tB, &tiq, &tD}) dfree(*p);
    dfree(jt);
  }
  SchurArgs args(double2* H, double2* T, int rank, double out_scale, int ny) const {
    SchurArgs a;
    a.H = H;
    a.T = T;
    a.tstride = (size_t)4 * L;
    a.cinv = cinv;
    a.corr = corr;
    a.g = g;
    a.tip = tip;
    a.tg = tg;
    a.tA = tA;
    a.tB = tB;
    a.jt = jt;
    a.cs = nullptr;
    a.tiq = tiq;
    a.tD = tD;
    a.halo8 = nullptr;
    a.tnum = 4;
    a.csT = nullptr;
    a.inv_dy2 = inv_dy2;
    a.dy2 = dy2;
    a.out_scale = out_scale;
    a.inv_ny = 1.0 / (double)ny;
    a.rl = rl;
    a.L = L;
    a.P = P;
    a.rank = rank;
    a.tile8 = 1;
    return a;
  }
};

// The substructured path: square power-of-two grids (the reference's ky = kx table is the
// periodic y-symbol only when ny == nx), power-of-two rank counts, slabs of 512..4096 rows.
inline bool schur_ok(int nx, int ny, int nranks) {
  if (nx != ny || nranks < 1 || (nranks & (nranks - 1)) != 0 || ny % nranks != 0) return false;
  return schur_supported(ny / nranks) && fused_rows_supported(nx, ny / nranks);
}

// The fused path on `nranks` y-slabs: power-of-two slabs whose column blocks split evenly.
inline bool fused_ok(int nx, int ny, int nranks) {
  if (nranks < 1 || (nranks & (nranks - 1)) != 0 || ny % nranks != 0) return false;
  if ((nx / 2) % nranks != 0) return false;
  return fused_poisson_supported(nx, ny, ny / nranks);
}

// Poisson path selection (cfdj_vm_set_poisson / cfdj_fps_set_poisson).
inline bool resolve_fused(int path, int nx, int ny, int nranks) {
  if (path == CFDJ_POISSON_ROCFFT) return false;
  const bool ok = fused_ok(nx, ny, nranks);
  if (path == CFDJ_POISSON_FUSED && !ok)
    throw Error{CFDJ_ERR_ARG, "fused Poisson needs power-of-two sides, nx 1024..16384, ny "
                              "1024..8192, a power-of-two rank count and >= 8 rows per rank"};
  return ok;
}

}  // namespace cfdj
