// Internal declarations shared by the libcfdj.so translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <string>
#include <vector>

#include "cfdj.h"

// rows per chunk of the Schur interior solve (schur.hip, host_common.hpp SchurTables)
#ifndef CFDJ_SCHUR_CHUNK
#define CFDJ_SCHUR_CHUNK 32
#endif

namespace cfdj {

// ---- errors ------------------------------------------------------------------------
void set_error(const std::string& msg);
const char* last_error();

struct Error {
  int code;
  std::string msg;
};

#define CFDJ_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      throw ::cfdj::Error{CFDJ_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
  } while (0)

#define CFDJ_FFT(expr)                                                                  \
  do {                                                                                  \
    rocfft_status s_ = (expr);                                                          \
    if (s_ != rocfft_status_success)                                                    \
      throw ::cfdj::Error{CFDJ_ERR_ROCFFT, std::string(#expr) + ": rocfft status " +     \
                                               std::to_string((int)s_)};                \
  } while (0)

#define CFDJ_NCCL(expr)                                                                 \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      throw ::cfdj::Error{CFDJ_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)}; \
  } while (0)

#define CFDJ_REQUIRE(cond, msg)                                                         \
  do {                                                                                  \
    if (!(cond)) throw ::cfdj::Error{CFDJ_ERR_ARG, (msg)};                              \
  } while (0)

// ---- streaming loads ------------------------------------------------------------------
// A load of data that is read once by one workgroup and not again soon (the forward row
// pass's input, omega^n in the stage kernels, the spectral solvers' elementwise inputs):
// with NT it is issued as a non-temporal load, so the line does not displace what the next
// kernel re-reads (the half spectrum, psi) from the caches.  At 4096^2: step 0.776 -> 0.744
// ms.  The host launches the NT instantiation of a kernel where the fields outgrow the 256 MB
// last-level cache (stream_loads_pay); on grids that live in that cache the plain loads are
// 3 % faster (and a run-time flag per load cost 1-2 % either way: a template flag).  Not
// for lines several workgroups share (halo rows of the stencil, the 32-B column pieces of the
// inverse row pass: 49 -> 84 us with it).  CFDJ_NT_LOADS=0 builds plain loads everywhere.
#ifndef CFDJ_NT_LOADS
#define CFDJ_NT_LOADS 1
#endif
template <bool NT>
__device__ __forceinline__ double2 load_stream(const double2* p) {
#if CFDJ_NT_LOADS
  if constexpr (NT) {
    typedef double cfdj_d2v __attribute__((ext_vector_type(2)));
    const cfdj_d2v t = __builtin_nontemporal_load(reinterpret_cast<const cfdj_d2v*>(p));
    return make_double2(t.x, t.y);
  }
#endif
  return *p;
}
template <bool NT>
__device__ __forceinline__ double load_stream(const double* p) {
#if CFDJ_NT_LOADS
  if constexpr (NT) return __builtin_nontemporal_load(p);
#endif
  return *p;
}
// The same for stores of data that is read back only after far more than the caches hold has
// gone by (the spectral solvers' scratch spectra: hybrid 4096^2 1.52 -> 1.45 ms/step).
template <bool NT>
__device__ __forceinline__ void store_stream(double2* p, double2 v) {
#if CFDJ_NT_LOADS
  if constexpr (NT) {
    typedef double cfdj_d2v __attribute__((ext_vector_type(2)));
    const cfdj_d2v t = {v.x, v.y};
    __builtin_nontemporal_store(t, reinterpret_cast<cfdj_d2v*>(p));
    return;
  }
#endif
  *p = v;
}
// One field of `bytes` bytes among the half dozen a step cycles through: beyond 64 MB they do
// not stay in the last-level cache from one kernel to the next anyway.
inline bool stream_loads_pay(size_t bytes) { return bytes >= ((size_t)64 << 20); }

// ---- XCD-aware block order ------------------------------------------------------------
// Workgroups are dealt round-robin over the 8 XCDs (blocks b and b+8 share an XCD and its
// L2; MI355X_MICROARCH.md, Workgroup dispatch).  xcd_remap gives each XCD a contiguous
// range of the logical work index so neighbouring tiles (which share cache lines: 64-B
// halves of a 128-B line, stencil edge columns and halo rows) meet in the same L2.
// Bijective for any n; speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int b, int n) {
  constexpr int X = 8;
  const int q = n / X, r = n % X;  // XCD x gets q + (x < r) consecutive logical indices
  const int x = b % X, slot = b / X;
  if (slot >= q + (x < r ? 1 : 0)) return b;  // cannot happen for b < n
  return x * q + (x < r ? x : r) + slot;
}

// ---- kernel parameter blocks --------------------------------------------------------
// Constants of Common.jl:149-152 plus the RK3 stage weights of vm.jl:28,43-47,62-66.
struct StageCoef {
  double aa, bb, gg, hh;  // 1/(re dx^2), 1/(re dy^2), 1/(4dx dy), 1/3
  double dt;              // stage 1: wn + dt*r
  double c25dt;           // stage 2: (.75wn + .25wt) + (.25dt)*r
  double c23, c23dt;      // stage 3: (wn/3 + (2/3)wt) + ((2/3)dt)*r
};

// One slab of rows [0, ny) (local), pitch nx, x contiguous.  Row -1 / row ny are read
// from the lo / hi ghost rows (on one GPU: the periodic wrap rows of the same array).
struct StageParams {
  bool stream = false;  // omega^n by streaming loads; marching kernel: the output by streaming stores
  const double* w;     // stencil input omega_s
  const double* w_lo;
  const double* w_hi;
  const double* s;     // streamfunction psi
  const double* s_lo;
  const double* s_hi;
  const double* wn;    // omega^n (pointwise; stages 2 and 3)
  double* out;         // stage output (stage 0: the bare RHS r)
  int nx, ny;
  int y0, ycount;      // rows [y0, y0 + ycount) of the slab are computed (halo split) ...
  int y0b = 0, ycount_b = 0;  // ... and, in the same launch, rows [y0b, y0b + ycount_b)
                       // (marching kernel only)
  int nblk_a = 0, nblk_b = 0;  // set by launch_stage: rows_per_wave blocks each window touches
  bool cp_accumulate = false;  // colpart: add to the stored partial instead of replacing it
  double* colpart;     // optional: column sums of `out` per block of rows_per_wave rows,
                       // [y / rows_per_wave][nx] (increasing row order, the slab's row 0 last)
  int rows_per_wave;
  bool march;          // true: always the marching kernel (rows_per_wave rows per wavefront)
  StageCoef k;
};

void launch_stage(int stage, const StageParams& p, hipStream_t st);
// Which kernel launch_stage picks for these parameters: the row-group one (true) or the
// marching one.
bool stage_runs_row_group(const StageParams& p);
// Column sums of a slab field in the stage kernel's partial layout (rows_per_wave blocks):
// colpart[b][x] = sum of f[y][x] over rows y of block b (fields not written by a stage).
void launch_colpart(const double* f, int nx, int rows, int rpw, double* colpart,
                    hipStream_t st);
// out8[0][x] = sum over the nb blocks of colpart[b][x]; rows 1..7 of out8 zeroed.
void launch_colsum_row(const double* colpart, int nb, int nx, double* out8, hipStream_t st);
// dst[i ds] = src[i ss], i < n (complex elements).
void launch_strided_copy(double2* dst, int ds, const double2* src, int ss, int n,
                         hipStream_t st);

// Spectral divide (Common.jl:118-121) on a (width x rows) block of the half spectrum
// stored with row pitch `pitch` (complex elements); column i of the block is the
// global x-wavenumber index kx_off + i, row j the global y index.  Elements with global
// kx >= nxh are padding and are zeroed.  neg folds the f = -w of Common.jl:134.
struct DivideParams {
  double2* spec;
  const double* cx;  // cos(kx[m]), m = 0..nxh-1
  const double* cy;  // cos(ky[n]), n = 0..ny-1
  // ny < nx only: cos(ky[(ny-n) mod ny]).  Common.jl:113 aliases ky = kx, so for ny < nx
  // the symbol is not Hermitian in y and the reference's real(ifft(e/d)) equals the
  // c2r of e * (1/d(m,n) + 1/d(-m,-n))/2; NULL when ny == nx (plain division).
  const double* cy_mirror;
  int width, rows, pitch, kx_off, nxh;
  double aa, bb, cc, scale;
  bool neg;
  bool recip;  // multiply by the rounded reciprocal (lid_driven_cavity.jl:17 e * iden)
};
void launch_divide(const DivideParams& p, hipStream_t st);

// Slab-FFT transposition helpers (multi-GPU / virtual ranks).
// pack:   X[jl*nxh + kx] -> S[(q*rows + jl)*kb + kl],  kx = q*kb + kl (zero padding)
// unpack: S[(q*rows + jl)*kb + kl] -> X[jl*nxh + kx]   (kx < nxh)
void launch_pack(const double2* X, double2* S, int nxh, int rows, int kb, int nranks,
                 hipStream_t st);
void launch_unpack(const double2* S, double2* X, int nxh, int rows, int kb, int nranks,
                   hipStream_t st);

// Hand-written fused FD-FFT Poisson for power-of-two grids (poisson_fft.hip):
// pass 0 = row r2c (f -> column-major packed half spectrum H[m][y], pitch `rows`),
// pass 1 = column FFT + divide + inverse FFT on C (in place), pass 2 = row c2r (H -> s).
// One GPU: C == H.  y-slabs: H is the all-to-all send buffer (columns [q kb, (q+1) kb) are
// the contiguous chunk for rank q), C the receive buffer, where column ml of this rank is
// stored as P segments of `rows` elements (one per source rank), kb * rows apart.
struct FusedPoissonArgs {
  int nx, ny, rows;     // row length, column length (global ny), rows of this GPU
  const double* f;      // input field (pitch nx, `rows` rows)
  double* s;            // output streamfunction (pitch nx)
  double2* H;           // (nx/2) x rows packed half spectrum, column-major
  double2* C;           // column-pass buffer (kb columns of ny)
  double2* Cout;        // column-pass output (nullptr: in place into C)
  int tile8;            // row passes: spectrum in 8-mode tiles (Schur y-slab path)
  int m0, kb;           // first global column and column count of C
  int rl_log2;          // log2(rows per column segment of C)
  unsigned seg;         // elements between the segments of one column of C
  const double2* twL;   // exp(-2 pi i k/(nx/2)), k < nx/2
  const double2* twN;   // exp(-2 pi i k/nx), k < nx
  const double2* twM;   // exp(-2 pi i k/ny), k < ny
  const double* cx;     // cos(kx[m]), m <= nx/2
  const double* cy;     // cos(ky[k]), k < ny
  const double* cy_mirror;  // cy[(ny-k) % ny] or nullptr (symbol even in ky)
  double aa, bb, cc, scale;
  bool neg;
  bool recip;           // see DivideParams::recip
  int ncu;              // compute units (persistent grid size)
  double2* col0;        // row passes, 8-mode tiles, where fused_rows_take_col0(): the packed
                        // column 0 as a dense array [rows] -- written (also) by pass 0, read
                        // (instead of H's column 0) by pass 2; null: H only
  const double* fx;     // pass 0 with col0: one more workgroup transforms the first rows of
  double2* Hx;          // this 8-row array into this 8-row tiled spectrum (null: none)
  double2* wrows;       // pass 0 with col0: the input's first and last rows, as they are, to
                        // wrows[0 .. nx/2) and wrows[nx/2 .. nx) (null: none)
  const double* cp;     // pass 0 with col0: nx/64 more workgroups add the ncp partial rows
  int ncp;              // cp[b][x] (a field's column sums per block of rows) up into
  double* csout;        // csout[x] -- the launch that would do it otherwise (null: none)
  int mmax;             // pass 2, > 0: H is zero in the columns above mmax, which are not read
  // pass 2 with col0 (8-mode tiles): two more rows -- rows 0 and 1 of the 8-row tiled spectrum
  // hx_H (SchurArgs::halo8) -- go to the slab's halo rows hx_lo / hx_hi, their packed column 0
  // from *hx_c0lo / *hx_c0hi (null: none)
  const double2* hx_H;
  double* hx_lo;
  double* hx_hi;
  const double2* hx_c0lo;
  const double2* hx_c0hi;
  bool stream;          // pass 0: the input rows by streaming loads (load_stream)
  bool stream_out;      // pass 2 (small-item kernel): the output rows by streaming stores
};
bool fused_poisson_supported(int nx, int ny, int rows);
bool fused_rows_take_col0(int nx, int rows);
bool fused_rows_supported(int nx, int rows);  // the row passes alone (y-slab Schur path)
void launch_fused_poisson_pass(int pass, const FusedPoissonArgs& a, hipStream_t st);
// The 2/3-rule solver's product rows in one kernel (poisson_fft.hip, rows_jac_np_kernel):
// inverse row pass of the scratch spectrum a.H (columns 0..a.mmax), product with the three
// real fields at a.f, forward row pass into the scratch spectrum a.C; rows of up to 4096 reals.
bool rows_jac_supported(int nx, int rows);
void launch_rows_jac(const FusedPoissonArgs& a, double inv_np, hipStream_t st);

// DST-I Poisson solve of the cavity on its own interior (dst_poisson.hip): pass 0 = x-DST of
// the rows of w (sign folded in) -> T, pass 1 = y-DST, iden multiply, y-DST on T in place,
// pass 2 = x-DST of the rows of T -> interior of s.  T holds (nx/2) mode pairs x JT row
// slots (row j in slot j - 1, JT >= ny); tx / ty are the Dirichlet symbol tables of the
// (2nx) x (2ny) extension grid (tx[k], k <= nx; ty[p], p < 2ny, even about ny).
struct DstPoissonArgs {
  int nx, ny, P, JT;   // cavity cells, node-array pitch, row slots per mode pair
  const double* w;     // (nx+1) x (ny+1) node array, right-hand side = (neg ? -w : w)
  double* s;           // node array receiving the interior solution
  double2* T;
  const double* tx;
  const double* ty;
  double scale;        // 1 / ((2nx)(2ny))
  bool neg;
  const double2* twX;  // exp(-2 pi i k / (2nx))
  const double2* twY;  // exp(-2 pi i k / (2ny))
  int ncu;
  // optional (pass 2): per-workgroup sums of (s - sprev)^2 over the interior into part[0 ..
  // dst_rows_grid(nx, ny, ncu, half))
  const double* sprev;
  double* part;
  // passes on the half-length transform (bit p = pass p) instead of the odd extension's:
  // dst_half_passes(nx, ny)
  int half;
};
bool dst_poisson_supported(int nx, int ny);
// Which passes run the half-length DST kernels: they halve the arithmetic and the threads per
// transform, which pays where a pass still fills the chip (row passes from nx = 4096, column
// pass from ny = 2048); CFDJ_DST_HALF=0 / 1 (read at the call) forces none / all.
int dst_half_passes(int nx, int ny);
int dst_rows_grid(int nx, int ny, int ncu, int half);
void launch_dst_poisson_pass(int pass, const DstPoissonArgs& a, hipStream_t st);

// In-place 2-D complex FFT of `batch` nx-by-ny arrays (x contiguous) in two passes,
// unnormalised both ways (fft2d_c2c.hip).  dir < 0 forward, > 0 inverse; twX / twY:
// exp(-2 pi i k / n) device tables for n = nx, ny.
bool c2c2d_supported(int nx, int ny);
void launch_c2c2d(double2* a, int nx, int ny, int batch, int dir, const double2* twX,
                  const double2* twY, hipStream_t st);
// real(ifft2(a)) (unnormalised) -> r, `a` overwritten; fft2(complex(r, 0)) -> a.
void launch_c2r2d(double2* a, double* r, int nx, int ny, int batch, const double2* twX,
                  const double2* twY, hipStream_t st);
void launch_r2c2d(const double* r, double2* a, int nx, int ny, int batch, const double2* twX,
                  const double2* twY, hipStream_t st);
// r[0] = real(ifft2(wf)), r[1] = real(ifft2(wf / (kx[i]^2 + kx[j]^2))), x = 2 scratch arrays.
void launch_hybrid_c2r2d(const double2* wf, const double* kx, double2* x, double* r, int nx,
                         int ny, const double2* twX, const double2* twY, hipStream_t st);

// 2-D transforms of REAL n-by-n fields on the half spectrum (fft2d_r2c.hip): modes kx index
// m = 0..n/2, all ky; element (m, k) at m n + k (ky contiguous), column n/2 = the kx Nyquist
// column.  Unnormalised both ways.
struct HalfSpecArgs {
  int n;                // nx = ny
  const double2* twL;   // exp(-2 pi i k/(n/2))
  const double2* twN;   // exp(-2 pi i k/n)
  int ncu;              // compute units (persistent row pass)
  const double* kx;     // wavenumbers (Common.jl:190-199), n entries; ky = kx
  int tx0, ty0, ty1;    // 2/3 rule: indices tx0 <= i < n - tx0, ty0 <= k < ty1 are zeroed
  bool stream;          // once-read inputs by streaming loads (load_stream)
};
// Inverse modes: which arrays the column pass forms from the one spectrum w_f it reads.
//   kHalfPlain  1 array : w_f
//   kHalfHybrid 2 arrays: w_f, w_f / k2                          (hybrid.jl:103,115)
//   kHalfPs23   4 arrays: i kx w_f / k2, i ky w_f, i ky w_f / k2, i kx w_f, 2/3-rule modes
//                         zeroed                      (pseudospectral_23_rule.jl:109-133)
enum { kHalfPlain = 1, kHalfHybrid = 2, kHalfPs23 = 3 };
bool half2d_supported(int nx, int ny);
// hs = fft2(r) (half); scratch: n/2 x n complex.
void launch_half_r2c2d(const HalfSpecArgs& a, const double* r, double2* scratch, double2* hs,
                       hipStream_t st);
// r[b] = real(ifft2(factor_b(hs))) n n, b < arrays of `mode`; x: arrays x (n/2 x n) complex
// scratch.  hs is left intact.
void launch_half_c2r2d(const HalfSpecArgs& a, int mode, const double2* hs, double2* x, double* r,
                       hipStream_t st);
// hs_out = fft2 (half) of the 2/3 rule's product r[0] r[1] - r[2] r[3], r[b] = real(ifft2(
// factor_b(hs))) / n^2 as launch_half_c2r2d(kHalfPs23) forms them: the fourth field's rows, the
// product and its row transform in one kernel (r: three n x n arrays are written).  Grids of
// up to 4096^2 (half_ps23_jacobian_supported).
bool half_ps23_jacobian_supported(int n);
void launch_half_ps23_jacobian(const HalfSpecArgs& a, const double2* hs, double2* x, double* r,
                               double2* hs_out, hipStream_t st);

// 2-D transforms of REAL n-by-n fields with n = 3 * 2^k (1536, 3072, 6144: the 3/2 rule's
// product grids) on the columns m = 0..mmax of the half spectrum (fft2d_r2c3.hip): element
// (m, k) at m n + k (ky contiguous); the spectrum is zero / not wanted beyond column mmax
// (mmax < n/2), slot (0, .) holds the DC column alone.  Unnormalised both ways.
struct Real2d3Args {
  int n;                 // grid size
  int mmax;              // last kx column held
  const double2* tw3L;   // exp(-2 pi i k/(n/6)): the row transforms' power-of-two thirds
  const double2* twL;    // exp(-2 pi i k/(n/2))
  const double2* twN;    // exp(-2 pi i k/n)
  const double2* tw3M;   // exp(-2 pi i k/(n/3)): the column transforms' thirds
  bool stream;           // once-read / once-written real fields by streaming loads / stores
};
bool real2d3_supported(int n);
// r[b] = real(ifft2(x[b])) n n for b < batch; x: batch x (mmax + 1) x n complex, transformed
// in place along y on the way.
void launch_c2r2d3(const Real2d3Args& a, double2* x, double* r, int batch, hipStream_t st);
// x = columns 0..mmax of fft2(r).
void launch_r2c2d3(const Real2d3Args& a, const double* r, double2* x, hipStream_t st);
// The same transforms for the 3/2-rule solver on the half spectrum hs of its UNPADDED grid
// (columns m = 0..N/2 of N = 2n/3 elements, ky contiguous, then the N/2 + 1 elements
// w_f(-m, N/2), m = 0..N/2, which that solver's spectra do not share with their other half;
// a.mmax = N/2): the padding and the derivative factors of pseudospectral_32_rule.jl:109-154
// are applied where the inverse column pass loads a column, the unpadding of :171-178 where the
// forward one stores it.
struct Ps32HalfArgs {
  const double* kx;   // the reference's wavenumber table of the unpadded grid (kx[0] = eps)
  double scale_in;    // (nxe nye) / (nx ny)
  double scale_out;   // (nx ny) / (nxe nye)
};
// x[b] = the padded derivative spectrum b of hs, b < 4, transformed along y (4 x (mmax + 1) x n);
// r[b] = real(ifft2(.)) of the first `nrow` of them (the inverse row pass).
void launch_ps32_c2r2d3(const Real2d3Args& a, const Ps32HalfArgs& s, const double2* hs, double2* x,
                        double* r, int nrow, hipStream_t st);
// hs = unpadded fft2((r[0] r[1] - r[2] real(ifft_x(x4))) inv_np^2): the fourth field's inverse row
// pass, the product (pseudospectral_32_rule.jl:156-169) and its forward transform, the rows in
// one kernel.  x4: that field's (mmax + 1) x n array from launch_ps32_c2r2d3; r: three n x n
// real arrays; xj: (mmax + 1) x n scratch.
void launch_ps32_product_r2c2d3(const Real2d3Args& a, const Ps32HalfArgs& s, const double2* x4,
                                const double* r, double2* xj, double2* hs, double inv_np,
                                hipStream_t st);
// hs = unpadded fft2(r) (columns 0..N/2); x: (mmax + 1) x n scratch.
void launch_ps32_r2c2d3(const Real2d3Args& a, const Ps32HalfArgs& s, const double* r, double2* x,
                        double2* hs, hipStream_t st);

// Substructured y-solve of the y-slab Poisson path (schur.hip): per x-mode
// m = 1..L-1, the periodic y-tridiagonal of the reference symbol split at one separator row
// per rank (row 0 of each slab); interior blocks by DST-I (odd-extension FFT of length
// 2 rl in LDS), separators by a P x P circulant system from the gathered traces.
struct SchurArgs {
  double2* H;           // this rank's half spectrum in 8-mode tiles, rl rows (in place)
  double2* T;           // traces of every rank: rank q's [L][4] block (f_sep, t_1, t_n,
                        // column sum) starts at T + q * tstride
  size_t tstride;       // complex elements between two ranks' blocks (>= 4 L)
  const double* cinv;   // [L][P] first row of the inverse circulant separator system
  const double* corr;   // [L] 1/D_ref(m, 0) - 1/e_m (the reference's ky[1] = eps)
  const double* g;      // trace Green's function gL(j), j = 0..rl, in 8-mode tiles
  const double2* cs;    // spectrum of the slab's column sum (row 0 of an 8-row tile
                        // spectrum): the trace's column sum per mode
  const int* jt;        // [L/8] rows of a tile's traces above round-off (gL decay)
  const double* tip;    // [L][32] inverse pivots of a 31-row chunk (system scaled by dy^2)
  const double* tg;     // [L][33] chunk homogeneous solution g(i), g(0) = 1, g(32) = 0
  const double* tA;     // [L] interface off-diagonal g(31)
  const double* tB;     // [L] interface diagonal -(2 + eps) + 2 g(1)
  const double* tiq;    // [L][K] inverse pivots of the K-1 interface system
  const double* tD;     // [L] 2 + ep = -dy^2 d_m: the scaled operator's diagonal, negated
  int tnum;             // numbers per mode in T: 4, or 3 (no column sum: csT has the total's)
  const double2* csT;   // [L] spectrum of the column sum over ALL ranks' rows, or null: then
                        // the solve adds up the ranks' fourth trace numbers
  double2* halo8;       // optional: 8-row tiled spectrum receiving psi-hat of the rows just
                        // outside the slab -- row 0: the row before the slab's first (from the
                        // operator's equation at the separator row), row 1: the next slab's
                        // separator row -- so psi's halo rows need no exchange
  double inv_dy2, dy2, out_scale, inv_ny;
  int rl, L, P, rank;
  int tile8;            // H in 8-mode tiles (sidx in poisson_fft.hip); required
};
bool schur_supported(int rl);
void launch_schur_pass(int pass, const SchurArgs& a, hipStream_t st);  // 0 traces, 1 solve

// The packed DC / Nyquist column (x-modes 0 and nx/2 as Re / Im of one complex column of
// length ny), already FFT'd along y: split with Z[-k], divide each half by the reference
// symbol of its x-mode (e[1,1] = 0), re-pack; in place.
struct PackedDivParams {
  double2* Z;
  const double* cx;     // cos(kx[m]), m <= L
  const double* cy;     // cos(ky[k]), k < ny
  double aa, bb, cc, scale;
  int L, ny;
  bool neg;
};
void launch_packed_divide(const PackedDivParams& p, hipStream_t st);

// The packed DC / Nyquist column of the y-slab path solved whole, everything in LDS (one
// workgroup, or one per real column): the column's ny elements are read from P rank segments
// of `rows` elements (segment q at src + q * seg_stride: the all-gather's receive layout),
// transformed along y, split into the DC and the Nyquist column, each divided by its
// reference symbol (e[1,1] = 0), re-packed, transformed back and written to the dense column
// `dst`.  ny = 1024..8192 (a power of two); `a` supplies the symbol tables, the twiddles and
// `neg`.  With cs_src (square grids, the two-workgroup form): one more workgroup adds up the P
// ranks' column-sum rows (rank q's nx reals at cs_src + q * seg_stride) and writes the sum's
// half spectrum, modes 1 .. nx/2 - 1, to csT.
bool col0_solve_supported(int ny);
bool col0_solve_takes_colsum(int nx, int ny, int rows);
void launch_col0_solve(const FusedPoissonArgs& a, const double2* src, size_t seg_stride,
                       int rows, double2* dst, hipStream_t st, const double2* cs_src = nullptr,
                       int nranks = 0, double2* csT = nullptr);
// Whether the forward row pass of the 8-mode-tile layout takes FusedPoissonArgs::cp.
bool fused_rows_take_colsum(int nx, int rows);

// Finiteness check: sets *flag = 1 if any element is not finite.
void launch_check_finite(const double* a, size_t n, int* flag, hipStream_t st);

}  // namespace cfdj
