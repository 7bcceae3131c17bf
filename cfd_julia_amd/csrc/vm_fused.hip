// FFT-fused stage kernel of the single-GPU vortex-merger step.
//
// One RK3 stage of vm.jl (vm_rhs, Common.jl:132-182, + the stage update, vm.jl:28,43-47,
// 62-66) is normally five HBM passes: row r2c, column FFT/divide/iFFT, row c2r (psi to
// HBM), the Arakawa stage kernel (psi back from HBM), and next stage's row r2c re-reading
// its output.  This kernel fuses everything on the row side of the column pass:
//
//   HA (column-pass output, psi-hat along x per row)  --row c2r in LDS-->  psi rows
//   psi rows + omega rows (HBM) + omega^n          --Arakawa + RK stage-->  omega_out (HBM)
//   omega_out rows                                 --row r2c in LDS-->      HB (HBM)
//
// so psi never touches HBM and omega_out is transformed while it is still on chip: per
// stage HBM sees HA 8 + omega 8 (+ omega^n 8) + omega_out 8 + HB 8 B per cell (32 / 40)
// plus the column pass 16, instead of 24/32 + 48.
//
// A workgroup owns a band of `band` consecutive rows and marches through it XR rows at a
// time.  LDS holds XR + 2 row slots (L complex = one real row each, padded): the psi rows
// s-1 .. s+XR of the current stencil rows s .. s+XR-1.  After the stencil the slots of
// psi rows s-1 .. s+XR-2 are dead; the XR output rows go there, are forward-transformed
// in place and written out as the next stage's spectrum; then the same slots receive
// psi rows s+XR+1 .. s+2XR (inverse transforms of the prefetched HA rows).  Row y of the
// band lives in slot (y - s0 + 1) mod (XR + 2).
//
// Spectrum layouts (both column-major, m-th column = x-mode m, packed DC/Nyquist in m = 0
// as in poisson_fft.hip): HB is natural (row y at y); HA is rotated by one (row y at
// (y - 1) mod M, written so by the column pass), so the XR psi rows s+XR+1 .. s+2XR a
// step reads are one aligned XR*16-B segment per column, like the XR output rows it
// writes to HB.
//
// The stencil arithmetic is stencil.hpp's (contraction off, the reference's order); the
// FFT code may contract (tolerance 1e-12 relative on psi, as poisson_fft.hip).
#pragma clang fp contract(fast)
#include "fft_lds.hpp"
#include "stencil.hpp"

namespace cfdj {

namespace {

template <int L>
struct FCfg {
  using P = Plan<L>;
  static constexpr int T = P::T;                       // threads per row transform
  static constexpr int XR = L >= 2048 ? 2 : (L >= 1024 ? 4 : 8);
  static constexpr int NSLOT = XR + 2;
  static constexpr int SLOT = P::ROWSTRIDE;            // complex elements per slot
  static constexpr int THREADS = XR * T;
  static constexpr int PAIRS = (L / 2) * XR / THREADS;  // (m, L-m) pairs per thread
  static_assert(THREADS == 256, "one 256-thread workgroup per CU");
  static_assert(NSLOT * SLOT * 16 <= 140 * 1024, "slots must leave room for twiddles");
};

// Pair slot e of a round: row qq, columns m and L-m; 16 lanes take 16 consecutive m of one
// row, the XR rows of one m are XR*16 contiguous bytes of a column.
template <int L>
__device__ __forceinline__ void fpair(int e, int& qq, int& m) {
  constexpr int XR = FCfg<L>::XR;
  qq = (e >> 4) % XR;
  m = ((e >> 4) / XR) * 16 + (e & 15);
}

template <int L>
struct HLoads {
  double2 xm[FCfg<L>::PAIRS], xp[FCfg<L>::PAIRS];
  double2 xh;  // X[L/2] for the lanes with m = 0
};

// Spectrum rows qq < nrows of the rotated layout at positions pos + qq (pos + nrows <= M).
template <int L>
__device__ __forceinline__ void load_h(HLoads<L>& ld, const double2* __restrict__ HA, int M,
                                       int pos, int nrows) {
  using C = FCfg<L>;
  const double2* base = HA + __builtin_amdgcn_readfirstlane(pos);
#pragma unroll
  for (int i = 0; i < C::PAIRS; ++i) {
    int qq, m;
    fpair<L>(threadIdx.x + i * C::THREADS, qq, m);
    if (qq < nrows) {
      ld.xm[i] = base[(unsigned)(m * M + qq)];
      ld.xp[i] = base[(unsigned)(((L - m) & (L - 1)) * M + qq)];  // m = 0: unused
      if (m == 0) ld.xh = base[(unsigned)((L / 2) * M + qq)];
    }
  }
}

// c2r pre-processing of the loaded rows into their slots (rows_inv_kernel's algebra).
template <int L>
__device__ __forceinline__ void pre_inv(const HLoads<L>& ld, double2* slots, int sf,
                                        int nrows, const TwLds<2 * L>& twN) {
  using C = FCfg<L>;
#pragma unroll
  for (int i = 0; i < C::PAIRS; ++i) {
    int qq, m;
    fpair<L>(threadIdx.x + i * C::THREADS, qq, m);
    if (qq >= nrows) continue;
    double2* bq = slots + ((sf + qq) % C::NSLOT) * C::SLOT;
    const double2 Xm = ld.xm[i];
    if (m == 0) {  // slot 0 = (X[0], X[L]), both real; Z[L/2] = 2 conj(X[L/2])
      bq[padx(0)] = make_double2(Xm.x + Xm.y, Xm.x - Xm.y);
      bq[padx(L / 2)] = make_double2(2.0 * ld.xh.x, -2.0 * ld.xh.y);
    } else {
      const double2 Xp = cconj(ld.xp[i]);
      const double2 S = cadd(Xm, Xp);
      const double2 D = cmul(cconj(twN.w(m)), csub(Xm, Xp));
      bq[padx(m)] = make_double2(S.x - D.y, S.y + D.x);
      bq[padx(L - m)] = make_double2(S.x + D.y, D.x - S.y);
    }
  }
}

// r2c post-processing of the transformed output rows into HB rows s + qq (natural layout;
// rows_fwd_kernel's algebra).
template <int L>
__device__ __forceinline__ void post_fwd(const double2* slots, int sf, double2* __restrict__ HB,
                                         int M, int s, const TwLds<2 * L>& twN) {
  using C = FCfg<L>;
  double2* base = HB + __builtin_amdgcn_readfirstlane(s);
#pragma unroll
  for (int i = 0; i < C::PAIRS; ++i) {
    int qq, m;
    fpair<L>(threadIdx.x + i * C::THREADS, qq, m);
    const double2* bq = slots + ((sf + qq) % C::NSLOT) * C::SLOT;
    const double2 Zm = bq[padx(m)];
    if (m == 0) {
      base[(unsigned)qq] = make_double2(Zm.x + Zm.y, Zm.x - Zm.y);
      const double2 Zh = bq[padx(L / 2)];
      base[(unsigned)((L / 2) * M + qq)] = make_double2(Zh.x, -Zh.y);
    } else {
      const double2 Zc = cconj(bq[padx(L - m)]);
      const double2 E = make_double2(0.5 * (Zm.x + Zc.x), 0.5 * (Zm.y + Zc.y));
      const double2 D = csub(Zm, Zc);
      const double2 O = make_double2(0.5 * D.y, -0.5 * D.x);
      const double2 WO = cmul(twN.w(m), O);
      base[(unsigned)(m * M + qq)] = cadd(E, WO);
      base[(unsigned)((L - m) * M + qq)] = cconj(csub(E, WO));
    }
  }
}

// psi at a lane's pair (x, x+1) of a slot row, with x-1 and x+2 (periodic in x).
template <int L>
__device__ __forceinline__ Win psi_win(const double2* row, int pp) {
  const double2 z = row[padx(pp)];
  Win w;
  w.a = z.x;
  w.b = z.y;
  w.l = row[padx((pp - 1) & (L - 1))].y;
  w.r = row[padx((pp + 1) & (L - 1))].x;
  return w;
}

// omega inputs of one stencil step, loaded in one batch (no branches, so the loads issue
// back to back and the wait is one vmcnt): wave w owns the contiguous x-pairs
// [w L/4, (w+1) L/4), chunk c of it pairs w L/4 + 64 c + lane, so x-neighbours across
// chunks come from the adjacent chunk's registers and only the wave range's two edge
// values per row are extra (wave-uniform) loads.
template <int L>
struct WIn {
  static constexpr int XR = FCfg<L>::XR, CH = L / 4 / kWave;
  double2 w[CH][XR + 2];
  double el[XR + 2], er[XR + 2];
};

// Rows s-1+j, j = J0 .. XR+1, of a stencil step (J0 = 2: the step's first two rows are the
// previous step's last two, carried by shift_w).
template <int L, int J0 = 0>
__device__ __forceinline__ void load_w(WIn<L>& in, const double* __restrict__ w, int M, int s,
                                       int wave, int lane) {
  constexpr int XR = FCfg<L>::XR, CH = WIn<L>::CH, NX = 2 * L;
  const int x0 = wave * (NX / 4);
  const int xl = x0 == 0 ? NX - 1 : x0 - 1;
  const int xr = x0 + NX / 4 == NX ? 0 : x0 + NX / 4;
#pragma unroll
  for (int j = J0; j < XR + 2; ++j) {
    const double* row = w + (size_t)((s - 1 + j) & (M - 1)) * NX;
    in.el[j] = row[xl];
    in.er[j] = row[xr];
#pragma unroll
    for (int c = 0; c < CH; ++c)
      in.w[c][j] = *reinterpret_cast<const double2*>(row + x0 + 2 * (c * kWave + lane));
  }
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Rows s+XR-1, s+XR of a step are rows s'-1, s' of the next (s' = s + XR): keep them.
template <int L>
__device__ __forceinline__ void shift_w(WIn<L>& in) {
  constexpr int XR = FCfg<L>::XR, CH = WIn<L>::CH;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    in.el[j] = in.el[XR + j];
    in.er[j] = in.er[XR + j];
#pragma unroll
    for (int c = 0; c < CH; ++c) in.w[c][j] = in.w[c][XR + j];
  }
}

// The Win of chunk c, row j: x-1 / x+2 from the neighbouring lanes, across chunk edges
// from the adjacent chunk (readlane), at the wave range's ends from the edge loads.
template <int L>
__device__ __forceinline__ Win w_win(const WIn<L>& in, int c, int j, int lane) {
  constexpr int CH = WIn<L>::CH;
  const double2 d = in.w[c][j];
  Win o;
  o.a = d.x;
  o.b = d.y;
  const double up = __shfl_up(d.y, 1, kWave);
  const double dn = __shfl_down(d.x, 1, kWave);
  const double lo = c == 0 ? in.el[j] : readlane_d(in.w[c > 0 ? c - 1 : 0][j].y, kWave - 1);
  const double hi = c == CH - 1 ? in.er[j] : readlane_d(in.w[c < CH - 1 ? c + 1 : 0][j].x, 0);
  o.l = lane == 0 ? lo : up;
  o.r = lane == kWave - 1 ? hi : dn;
  return o;
}

template <int L, int STAGE>
__global__ __launch_bounds__(256) void vm_fused_stage_kernel(const FusedStageParams p) {
  using P = Plan<L>;
  using C = FCfg<L>;
  constexpr int XR = C::XR;
  constexpr int NX = 2 * L;
  constexpr int CH = WIn<L>::CH;
  __shared__ double2 slots[C::NSLOT * C::SLOT];
  __shared__ TwLds<L> twL;
  __shared__ TwLds<2 * L> twN;
  const int M = p.ny;
  const int g = threadIdx.x / P::T;  // row group of the transforms
  const int tid = threadIdx.x % P::T;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int s0 = xcd_remap(blockIdx.x, gridDim.x) * p.band;
  const int iters = p.band / XR;
  const StageCoef k = p.k;

  twL.fill(p.twL);
  twN.fill(p.twN);
  // priming: psi rows s0-1, s0 (slots 0, 1; rotated positions s0-2, s0-1), then
  // s0+1 .. s0+XR (slots 2 .. XR+1; positions s0 .. s0+XR-1); the first stencil step's
  // omega loads go out behind them
  WIn<L> in;
  {
    HLoads<L> ld;
    load_h<L>(ld, p.HA, M, (s0 - 2) & (M - 1), 2);
    HLoads<L> ld2;
    load_h<L>(ld2, p.HA, M, s0, XR);
    load_w<L>(in, p.w, M, s0, wave, lane);
    __syncthreads();  // twiddle tables
    pre_inv<L>(ld, slots, 0, 2, twN);
    __syncthreads();
    double2 v[16];
    run_stages_if<L, 0, 1, true>(slots + (g % C::NSLOT) * C::SLOT, v, tid, twL, g < 2);
    pre_inv<L>(ld2, slots, 2, XR, twN);
    __syncthreads();
    run_stages_if<L, 0, 1, true>(slots + ((2 + g) % C::NSLOT) * C::SLOT, v, tid, twL, true);
  }

  for (int it = 0; it < iters; ++it) {
    const int s = s0 + it * XR;
    const int sf = (it * XR) % C::NSLOT;  // slot of psi row s-1 (and of output row s)
    const bool more = it + 1 < iters;

    // ---- stencil rows s .. s+XR-1 -> HBM and registers --------------------------------
    double2 wnv[CH][XR];
    if constexpr (STAGE >= 2) {
#pragma unroll
      for (int j = 0; j < XR; ++j)
#pragma unroll
        for (int c = 0; c < CH; ++c)
          wnv[c][j] = *reinterpret_cast<const double2*>(
              p.wn + (size_t)(s + j) * NX + wave * (NX / 4) + 2 * (c * kWave + lane));
    }
    double2 res[CH][XR];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int pp = wave * (L / 4) + c * kWave + lane;  // x-pair: x = 2 pp
      Win w[XR + 2], sv[XR + 2];
#pragma unroll
      for (int j = 0; j < XR + 2; ++j) {
        w[j] = w_win<L>(in, c, j, lane);
        sv[j] = psi_win<L>(slots + ((sf + j) % C::NSLOT) * C::SLOT, pp);
      }
#pragma unroll
      for (int j = 0; j < XR; ++j) {
        double r0, r1;
        pair_rhs(w[j], w[j + 1], w[j + 2], sv[j], sv[j + 1], sv[j + 2], k, r0, r1);
        const double2 wv = STAGE >= 2 ? wnv[c][j] : make_double2(0.0, 0.0);
        double2 out;
        out.x = stage_update<STAGE>(r0, w[j + 1].a, wv.x, k);
        out.y = stage_update<STAGE>(r1, w[j + 1].b, wv.y, k);
        *reinterpret_cast<double2*>(p.out + (size_t)(s + j) * NX + 2 * pp) = out;
        res[c][j] = out;
      }
    }
    // prefetch: the next psi rows' spectrum and the next step's omega rows (consumed after
    // the transforms)
    HLoads<L> ld;
    if (more) {
      load_h<L>(ld, p.HA, M, s + XR, XR);
      shift_w<L>(in);
      load_w<L, 2>(in, p.w, M, s + XR, wave, lane);
    }
    __syncthreads();  // every psi read of the dead slots is done

    // ---- output rows -> next stage's spectrum -----------------------------------------
    double2 v[16];
    if (p.write_spec) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int pp = wave * (L / 4) + c * kWave + lane;
#pragma unroll
        for (int j = 0; j < XR; ++j) slots[((sf + j) % C::NSLOT) * C::SLOT + padx(pp)] = res[c][j];
      }
      __syncthreads();
      run_stages<L, 0, -1, true>(slots + ((sf + g) % C::NSLOT) * C::SLOT, v, tid, twL);
      post_fwd<L>(slots, sf, p.HB, M, s, twN);
      __syncthreads();  // the slots are rewritten by the inverse transforms
    }

    // ---- psi rows s+XR+1 .. s+2XR into the same slots ---------------------------------
    if (more) {
      pre_inv<L>(ld, slots, sf, XR, twN);
      __syncthreads();
      run_stages<L, 0, 1, true>(slots + ((sf + g) % C::NSLOT) * C::SLOT, v, tid, twL);
    }
  }
}

template <int L>
void launch_l(int stage, const FusedStageParams& p, hipStream_t st) {
  const dim3 grid(p.ny / p.band), block(256);
  switch (stage) {
    case 1: hipLaunchKernelGGL((vm_fused_stage_kernel<L, 1>), grid, block, 0, st, p); break;
    case 2: hipLaunchKernelGGL((vm_fused_stage_kernel<L, 2>), grid, block, 0, st, p); break;
    default: hipLaunchKernelGGL((vm_fused_stage_kernel<L, 3>), grid, block, 0, st, p); break;
  }
}

}  // namespace

bool fused_stage_supported(int nx, int ny) {
  const bool p2 = nx > 0 && (nx & (nx - 1)) == 0 && ny > 0 && (ny & (ny - 1)) == 0;
  return p2 && nx >= 1024 && nx <= 4096 && ny >= 1024 && ny <= 8192;
}

int fused_stage_band(int nx, int ny, int ncu) {
  const int xr = nx >= 4096 ? 2 : (nx >= 2048 ? 4 : 8);
  int band = xr;
  while (band * 2 <= ny && ny / (band * 2) >= ncu) band *= 2;
  return band;
}

void launch_fused_stage(int stage, const FusedStageParams& p, hipStream_t st) {
  const int xr = p.nx >= 4096 ? 2 : (p.nx >= 2048 ? 4 : 8);
  if (!fused_stage_supported(p.nx, p.ny) || stage < 1 || stage > 3 || p.band < xr ||
      p.band % xr != 0 || p.ny % p.band != 0)
    throw Error{CFDJ_ERR_ARG, "fused stage kernel: unsupported size"};
  switch (p.nx) {
    case 1024: launch_l<512>(stage, p, st); break;
    case 2048: launch_l<1024>(stage, p, st); break;
    default: launch_l<2048>(stage, p, st); break;
  }
  CFDJ_HIP(hipGetLastError());
}

}  // namespace cfdj
