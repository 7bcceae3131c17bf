// libcfdj.so host side: handles, rocFFT plans, RCCL communicator, the RK3 step driver and
// the extern "C" ABI declared in include/cfdj.h.
//
// Device data layout: every field is a dense nx-by-rows fp64 block, x
// contiguous (the reference's column-major first index), pitch nx.  No ghost layers are
// stored: the periodic wrap in x is modular indexing inside the stage kernel, the wrap /
// halo in y is a pair of row pointers (on one GPU: the slab's own last / first row; on
// y-slabs: receive buffers filled by RCCL or, for virtual ranks, by device copies).
#include "host_common.hpp"

namespace cfdj {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* last_error() { return g_err.c_str(); }

}  // namespace cfdj

using namespace cfdj;

// =====================================================================================
// Static spectrum scratch of cfdj_fps_solve_device_noalloc
// =====================================================================================
// The half spectrum of the hand-written FFT Poisson passes, for callers that cannot
// allocate: (nx/2) * ny complex elements, at most kNoAllocMaxSpectrum (16 MiB).  Every GPU
// the library runs on holds its own copy of the array at its own address until the process
// ends.  In host code the array's name is only a stand-in: the device address comes from
// hipGetSymbolAddress, once per device with that device current (noalloc_scratch_init, at
// plan creation), and that pointer is what the kernels receive.
namespace {

constexpr size_t kNoAllocMaxSpectrum = (size_t)1 << 20;  // complex elements
static __device__ __align__(256) double2 g_noalloc_scratch[kNoAllocMaxSpectrum];

constexpr int kMaxDevices = 64;
std::mutex g_noalloc_mu;
double2* g_noalloc_ptr[kMaxDevices] = {};

// Resolve (once) and return the scratch array's address on the current device.
double2* noalloc_scratch_init() {
  int dev = -1;
  CFDJ_HIP(hipGetDevice(&dev));
  CFDJ_REQUIRE(dev >= 0 && dev < kMaxDevices, "device ordinal out of range");
  std::lock_guard<std::mutex> lk(g_noalloc_mu);
  if (g_noalloc_ptr[dev] == nullptr) {
    void* p = nullptr;
    CFDJ_HIP(hipGetSymbolAddress(&p, HIP_SYMBOL(g_noalloc_scratch)));
    CFDJ_REQUIRE(p != nullptr, "hipGetSymbolAddress returned a null scratch address");
    g_noalloc_ptr[dev] = static_cast<double2*>(p);
  }
  return g_noalloc_ptr[dev];
}

}  // namespace

// =====================================================================================
// Poisson handle (Common.jl:97-125 / fft_p.jl:8-42)
// =====================================================================================
struct cfdj_fps_plan {
  int device = -1;
  double dx = 0, dy = 0, eps = 0;
  hipStream_t stream = nullptr;
  Symbol sym;
  Plans plans;
  rocfft_plan fwd = nullptr, inv = nullptr;
  double2* spec = nullptr;
  double *f_dev = nullptr, *s_dev = nullptr;
  Fused fused;
  bool use_fused = false;
  double2* static_spec = nullptr;  // this device's g_noalloc_scratch (set at creation)

  void solve_device(const double* f, double* s) { solve_device(f, s, spec); }
  void solve_device(const double* f, double* s, double2* H) {
    if (use_fused) {
      const FusedPoissonArgs a = fused.args(sym, f, s, H, false);
      for (int pass = 0; pass < 3; ++pass) launch_fused_poisson_pass(pass, a, stream);
      return;
    }
    plans.exec(fwd, f, spec);
    launch_divide(sym.divide(spec, sym.nxh, sym.ny, sym.nxh, 0, false), stream);
    plans.exec(inv, spec, s);
  }
  ~cfdj_fps_plan() {
    fused.destroy();
    plans.destroy();
    sym.destroy();
    dfree(spec);
    dfree(f_dev);
    dfree(s_dev);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// =====================================================================================
// Vortex-merger handle (vm.jl:12-90 + Common.jl:132-182)
// =====================================================================================
namespace cfdj {

enum class Mode { Single, Virtual, Rccl };

struct Slab {
  int rank = 0, row0 = 0, rows = 0;
  double *wn = nullptr, *wa = nullptr, *wb = nullptr, *psi = nullptr;
  double* ghost = nullptr;  // 4 rows: w_lo, w_hi, s_lo, s_hi (slab mode only)
  double2 *X = nullptr, *S = nullptr, *Y = nullptr;  // slab-FFT buffers
  // Schur path: column-sum partials of wn / wa / wb as the stage kernel writes them
  // ([rows / rows_per_wave][nx], valid once a stage kernel or colpart wrote them), the
  // column-sum row padded to 8 rows (cs8) and its tiled row spectrum (cs)
  double* colpart[4] = {nullptr, nullptr, nullptr, nullptr};  // [3]: other inputs
  bool cp_valid[3] = {false, false, false};
  double* cs8 = nullptr;
  double2* cs = nullptr;
  // ... and psi-hat of the two rows just outside the slab (8-row tiled spectrum, rows 0 / 1),
  // which the solve kernel leaves for the inverse row pass to turn into psi's halo rows
  double2* hx8 = nullptr;
  void destroy() {
    dfree(wn);
    dfree(wa);
    dfree(wb);
    dfree(psi);
    dfree(ghost);
    dfree(X);
    dfree(S);
    dfree(Y);
    for (auto& c : colpart) dfree(c);
    dfree(cs8);
    dfree(cs);
    dfree(hx8);
  }
};

}  // namespace cfdj

struct cfdj_vm {
  Mode mode = Mode::Single;
  int nx = 0, ny = 0, nranks = 1, rank = 0, rows = 0, nxh = 0, kb = 0;
  double dx = 0, dy = 0, re = 0, eps = 0;
  int device = -1;
  int rows_per_wave = 16;
  bool stage_march = false;  // set by cfdj_vm_set_rows_per_wave: marching stage kernel only
  hipStream_t stream = nullptr;
  std::vector<Slab> slabs;
  Symbol sym;
  Plans plans;
  rocfft_plan fwd2d = nullptr, inv2d = nullptr;                  // Single
  rocfft_plan row_fwd = nullptr, row_inv = nullptr, col_fwd = nullptr, col_inv = nullptr;
  double2* spec = nullptr;                                       // Single
  Fused fused;                                                   // Single, 2^k grids
  bool use_fused = false;
  // substructured y-slab solve (schur.hip): traces of all ranks T, gathered column G
  SchurTables schur;
  bool use_schur = false;
  double2* csT = nullptr;  // [nx/2] spectrum of the column sum over all ranks' rows
  bool late_cs_on = true;  // CFDJ_SLAB_LATE_CS=0: a transform of the slab's own sums per rank
  // gather buffer of the substructured solve: per rank [4 L trace numbers][rows elements of
  // the packed column]; G: the solved packed column, dense
  double2* TG = nullptr;
  int ncp = 0;  // column-sum partial rows (blocks of rows_per_wave rows)
  double2* G = nullptr;
  // (and the rank's first and last input rows, nx / 2 complex each: the neighbours' halo rows)
  size_t tg_block() const { return (size_t)6 * (nx / 2) + (size_t)rows; }
  size_t tg_rows_off() const { return (size_t)4 * (nx / 2) + (size_t)rows; }
  rocfft_plan g_fwd = nullptr, g_inv = nullptr;
  ncclComm_t comm = nullptr;
  // y-slabs: halo exchanges on a side stream, overlapped with the Poisson passes (omega
  // halo) and the interior rows of the stage kernel (psi halo).  Collectives stay strictly
  // ordered: the main stream waits for the omega halo before its first collective.
  hipStream_t side = nullptr;
  hipEvent_t ev_src = nullptr, ev_whalo = nullptr, ev_psi = nullptr, ev_shalo = nullptr;
  bool whalo_pending = false;
  double* gather = nullptr;                                      // Rccl download buffer
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev;
  std::vector<int> ev_cat;
  size_t ev_used = 0;
  double ms[CFDJ_K_COUNT] = {};
  long launches[CFDJ_K_COUNT] = {};
  std::vector<int> ev_stage;  // RK3 stage (1..3) of a CFDJ_K_STAGE interval, else 0
  double stage_ms[3] = {};
  long stage_launches[3] = {};
  // finiteness check
  bool check_finite = false;
  int* d_flag = nullptr;
  // HIP graph of `nsteps` whole RK3 steps (single-GPU fused-Poisson handles), re-captured
  // when dt / nsteps / tuning change.
  bool use_graph = true;
  hipGraphExec_t gexec = nullptr;
  double g_dt = 0.0;
  int g_steps = -1;

  bool slab_mode() const { return mode != Mode::Single; }
  // Substructured path: psi's halo rows come out of the slab's own solve (the next slab's
  // separator value and the operator's equation at this slab's separator row), so psi is not
  // exchanged and the stage kernel runs as one launch.  CFDJ_SLAB_PSI_HALO=exchange at handle
  // creation keeps the exchange.
  bool local_psi = [] {
    const char* e = std::getenv("CFDJ_SLAB_PSI_HALO");
    return !(e && e[0] == 'e');
  }();
  bool psi_local() const {
    return slab_mode() && use_schur && local_psi && fused_rows_take_col0(nx, rows);
  }
  // ... and omega's halo rows travel in the solve's all-gather: every rank's first and last
  // input rows are part of its block, the stage kernel reads its neighbours' straight from the
  // gather buffer.  With both, a stage has one collective and no exchange of its own, no side
  // stream and no event.  CFDJ_SLAB_W_HALO=exchange keeps the omega exchange.
  bool gather_w = [] {
    const char* e = std::getenv("CFDJ_SLAB_W_HALO");
    return !(e && e[0] == 'e');
  }();
  bool w_in_gather() const { return psi_local() && gather_w; }
  // the slab's column sums ride in the gather untransformed (see poisson_schur)
  bool late_colsum() const {
    return slab_mode() && use_schur && late_cs_on && fused_rows_take_colsum(nx, rows) &&
           col0_solve_takes_colsum(nx, ny, rows);
  }
  // the slab whose block holds slab s's lower / upper halo row (a solo rehearsal has no
  // neighbours: its own)
  const double* gathered_row(const Slab& s, bool upper) const {
    const int P = nranks;
    int q = upper ? (s.rank + 1) % P : (s.rank + P - 1) % P;
    if (slabs.size() == 1 && P > 1 && mode == Mode::Virtual) q = s.rank;
    const double2* blk = TG + (size_t)q * tg_block() + tg_rows_off();
    return reinterpret_cast<const double*>(upper ? blk : blk + nx / 2);
  }

  // ---- timing -----------------------------------------------------------------------
  void reserve_events(size_t n) {
    while (ev.size() < n) {
      hipEvent_t e;
      CFDJ_HIP(hipEventCreate(&e));
      ev.push_back(e);
    }
  }
  void tbegin(int cat, int rk_stage = 0) {
    if (!timing) return;
    if (ev_used + 2 > ev.size()) reserve_events(ev.size() + 64);
    CFDJ_HIP(hipEventRecord(ev[ev_used], stream));
    ev_cat.push_back(cat);
    ev_stage.push_back(rk_stage);
  }
  void tend() {
    if (!timing) return;
    CFDJ_HIP(hipEventRecord(ev[ev_used + 1], stream));
    ev_used += 2;
  }
  void harvest() {  // after a stream sync
    if (!timing) return;
    for (size_t i = 0; i < ev_used / 2; ++i) {
      float t = 0.f;
      CFDJ_HIP(hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
      ms[ev_cat[i]] += t;
      launches[ev_cat[i]] += 1;
      if (ev_stage[i] >= 1 && ev_stage[i] <= 3) {
        stage_ms[ev_stage[i] - 1] += t;
        stage_launches[ev_stage[i] - 1] += 1;
      }
    }
    ev_used = 0;
    ev_cat.clear();
    ev_stage.clear();
  }

  // Column-sum partial buffers of the Schur path, one block per rows_per_wave rows (the
  // stage kernel's wave row ranges); re-sized and invalidated when rows_per_wave changes.
  void alloc_colparts() {
    ncp = (rows + rows_per_wave - 1) / rows_per_wave;
    for (auto& s : slabs) {
      for (auto& c : s.colpart) {
        dfree(c);
        c = dalloc<double>((size_t)ncp * nx);
      }
      for (bool& v : s.cp_valid) v = false;
    }
  }

  // ---- communication (slab mode) ------------------------------------------------------
  // Before a collective on the main stream: the side stream's omega halo (same
  // communicator) must have completed, so at most one RCCL operation is ever in flight.
  void comm_order() {
    if (whalo_pending) {
      CFDJ_HIP(hipStreamWaitEvent(stream, ev_whalo, 0));
      whalo_pending = false;
    }
  }

  // All-to-all of `count` complex elements per peer: send chunk q of slab p -> recv chunk
  // p of slab q.  pick(slab, send?) selects the buffers.
  template <class Pick>
  void alltoall(Pick pick, size_t count) {
    tbegin(CFDJ_K_COMM);
    comm_order();
    if (mode == Mode::Rccl) {
      Slab& s = slabs[0];
      CFDJ_NCCL(ncclAllToAll(pick(s, true), pick(s, false), 2 * count, ncclDouble, comm,
                             stream));
    } else {
      const size_t bytes = count * sizeof(double2);
      for (auto& sp : slabs)
        for (auto& sq : slabs)
          CFDJ_HIP(hipMemcpyAsync(pick(sq, false) + (size_t)sp.rank * count,
                                  pick(sp, true) + (size_t)sq.rank * count, bytes,
                                  hipMemcpyDeviceToDevice, stream));
    }
    tend();
  }

  // Fill the lo/hi ghost rows (offset 0/1 for w, 2/3 for psi) of every slab from the
  // neighbouring slabs' last/first rows.
  void halo(bool psi_field, const std::vector<const double*>& src) { halo(psi_field, src, stream); }
  void halo(bool psi_field, const std::vector<const double*>& src, hipStream_t hs) {
    const int off = psi_field ? 2 : 0;
    const size_t bytes = (size_t)nx * sizeof(double);
    tbegin(CFDJ_K_COMM);
    if (mode == Mode::Rccl) {
      Slab& s = slabs[0];
      const int prev = (rank + nranks - 1) % nranks, next = (rank + 1) % nranks;
      const double* first = src[0];
      const double* last = src[0] + (size_t)(rows - 1) * nx;
      double* lo = s.ghost + (size_t)(off + 0) * nx;
      double* hi = s.ghost + (size_t)(off + 1) * nx;
      // Order matters when prev == next (2 ranks): sends [to prev, to next], receives
      // [from next, from prev] so the k-th message between a pair matches by role.
      CFDJ_NCCL(ncclGroupStart());
      CFDJ_NCCL(ncclSend(first, nx, ncclDouble, prev, comm, hs));
      CFDJ_NCCL(ncclSend(last, nx, ncclDouble, next, comm, hs));
      CFDJ_NCCL(ncclRecv(hi, nx, ncclDouble, next, comm, hs));
      CFDJ_NCCL(ncclRecv(lo, nx, ncclDouble, prev, comm, hs));
      CFDJ_NCCL(ncclGroupEnd());
    } else {
      const int P = (int)slabs.size();
      for (int p = 0; p < P; ++p) {
        const int prev = (p + P - 1) % P, next = (p + 1) % P;
        double* lo = slabs[p].ghost + (size_t)(off + 0) * nx;
        double* hi = slabs[p].ghost + (size_t)(off + 1) * nx;
        CFDJ_HIP(hipMemcpyAsync(lo, src[prev] + (size_t)(slabs[prev].rows - 1) * nx, bytes,
                                hipMemcpyDeviceToDevice, hs));
        CFDJ_HIP(hipMemcpyAsync(hi, src[next], bytes, hipMemcpyDeviceToDevice, hs));
      }
    }
    tend();
  }

  // ---- Poisson: psi = fps(-w)  (Common.jl:134-136) ------------------------------------
  void poisson(const std::vector<const double*>& src, bool neg) {
    if (use_schur) {
      poisson_schur(src, neg);
      return;
    }
    if (!slab_mode() && use_fused) {
      const FusedPoissonArgs a = fused.args(sym, src[0], slabs[0].psi, spec, neg);
      static const int cat[3] = {CFDJ_K_FFT_FWD, CFDJ_K_DIVIDE, CFDJ_K_FFT_INV};
      for (int pass = 0; pass < 3; ++pass) {
        tbegin(cat[pass]);
        launch_fused_poisson_pass(pass, a, stream);
        tend();
      }
      return;
    }
    if (use_fused) {
      // y-slabs, hand-written passes: row r2c writes the column-major half spectrum X,
      // whose column blocks ARE the all-to-all chunks (no pack); the receive buffer Y holds
      // this rank's columns as P row segments, which the column pass addresses directly.
      const size_t cnt = (size_t)(nx / 2 / nranks) * rows;
      std::vector<FusedPoissonArgs> a;
      for (size_t i = 0; i < slabs.size(); ++i)
        a.push_back(fused.args(sym, src[i], slabs[i].psi, slabs[i].X, slabs[i].Y, rows,
                               slabs[i].rank, nranks, neg));
      for (auto& ai : a) {
        tbegin(CFDJ_K_FFT_FWD);
        launch_fused_poisson_pass(0, ai, stream);
        tend();
      }
      alltoall([](Slab& s, bool send) { return send ? s.X : s.Y; }, cnt);
      for (auto& ai : a) {
        tbegin(CFDJ_K_DIVIDE);
        launch_fused_poisson_pass(1, ai, stream);
        tend();
      }
      alltoall([](Slab& s, bool send) { return send ? s.Y : s.X; }, cnt);
      for (auto& ai : a) {
        tbegin(CFDJ_K_FFT_INV);
        launch_fused_poisson_pass(2, ai, stream);
        tend();
      }
      return;
    }
    if (!slab_mode()) {
      Slab& s = slabs[0];
      tbegin(CFDJ_K_FFT_FWD);
      plans.exec(fwd2d, src[0], spec);
      tend();
      tbegin(CFDJ_K_DIVIDE);
      launch_divide(sym.divide(spec, nxh, ny, nxh, 0, neg), stream);
      tend();
      tbegin(CFDJ_K_FFT_INV);
      plans.exec(inv2d, spec, s.psi);
      tend();
      return;
    }
    const size_t cnt = (size_t)rows * kb;
    for (size_t i = 0; i < slabs.size(); ++i) {
      Slab& s = slabs[i];
      tbegin(CFDJ_K_FFT_FWD);
      plans.exec(row_fwd, src[i], s.X);
      tend();
      tbegin(CFDJ_K_COMM);
      launch_pack(s.X, s.S, nxh, rows, kb, nranks, stream);
      tend();
    }
    alltoall([](Slab& s, bool send) { return send ? s.S : s.Y; }, cnt);
    for (auto& s : slabs) {
      tbegin(CFDJ_K_FFT_FWD);
      plans.exec(col_fwd, s.Y, nullptr);
      tend();
      tbegin(CFDJ_K_DIVIDE);
      launch_divide(sym.divide(s.Y, kb, ny, kb, s.rank * kb, neg), stream);
      tend();
      tbegin(CFDJ_K_FFT_INV);
      plans.exec(col_inv, s.Y, nullptr);
      tend();
    }
    alltoall([](Slab& s, bool send) { return send ? s.Y : s.S; }, cnt);
    for (size_t i = 0; i < slabs.size(); ++i) {
      Slab& s = slabs[i];
      tbegin(CFDJ_K_COMM);
      launch_unpack(s.S, s.X, nxh, rows, kb, nranks, stream);
      tend();
      tbegin(CFDJ_K_FFT_INV);
      plans.exec(row_inv, s.X, s.psi);
      tend();
    }
  }

  // y-slabs without a transpose (schur.hip): row r2c -> interior traces -> ONE all-gather of
  // every rank's traces, its piece of the packed DC / Nyquist column and (where the row pass
  // supplies them) its column sums and its first and last input rows -> that column's solve
  // -> separator + interior solve -> row c2r.  The gather buffer TG holds one block per rank,
  // [4 L: 4 trace numbers per x-mode, or 3 and then the L column sums][rows column elements]
  // [L first row][L last row]; a rank's own block is where its kernels write (in-place
  // all-gather).  The packed column is solved with the reference symbol: columns of up to
  // 8192 by launch_col0_solve straight from the blocks, longer ones by library transforms on
  // the dense copy G.
  void poisson_schur(const std::vector<const double*>& src, bool neg) {
    const int L = nx / 2;
    const double out_scale = (neg ? -1.0 : 1.0) / (double)nx;
    const bool col0_direct = fused_rows_take_col0(nx, rows);
    // the slab's column sums (the constant-mode correction's input) travel untransformed: the
    // forward row pass's extra workgroups add the partial rows up into the gather block, the
    // packed column's solve adds the ranks' rows and transforms the total -- instead of a
    // summing launch before the row pass and a transform per rank
    const bool late_cs = late_colsum();
    const size_t blk = tg_block();
    auto col_piece = [&](const Slab& s) { return TG + (size_t)s.rank * blk + (size_t)4 * L; };
    auto cs_piece = [&](const Slab& s) { return TG + (size_t)s.rank * blk + (size_t)3 * L; };
    auto schur_args = [&](const Slab& s) {
      SchurArgs sa = schur.args(s.X, TG, s.rank, out_scale, ny);
      sa.tstride = blk;
      sa.tile8 = 1;
      sa.cs = s.cs;
      sa.halo8 = psi_local() ? s.hx8 : nullptr;
      if (late_cs) {
        sa.tnum = 3;
        sa.csT = csT;
      }
      return sa;
    };
    // the slab's column sum per mode: the stage kernel's partials of this input (or a
    // colpart pass for other inputs), summed to one row, row r2c -> cs (8-mode tiles)
    std::vector<int> cp_idx(slabs.size());
    for (size_t i = 0; i < slabs.size(); ++i) {
      Slab& s = slabs[i];
      const int idx = src[i] == s.wn ? 0 : src[i] == s.wa ? 1 : src[i] == s.wb ? 2 : 3;
      cp_idx[i] = idx;
      const bool fresh = idx == 3 || !s.cp_valid[idx];
      if (late_cs && !fresh) continue;
      tbegin(CFDJ_K_FFT_FWD);
      if (fresh) {
        launch_colpart(src[i], nx, rows, rows_per_wave, s.colpart[idx], stream);
        if (idx < 3) s.cp_valid[idx] = true;
      }
      if (!late_cs) {
        launch_colsum_row(s.colpart[idx], ncp, nx, s.cs8, stream);
        if (!col0_direct) {  // (else: a workgroup of the slab's own row pass below)
          FusedPoissonArgs ca = fused.args(sym, s.cs8, nullptr, s.cs, s.cs, 8, 0, 1, neg);
          ca.tile8 = 1;
          launch_fused_poisson_pass(0, ca, stream);
        }
      }
      tend();
    }
    std::vector<FusedPoissonArgs> a;
    for (size_t i = 0; i < slabs.size(); ++i) {
      a.push_back(fused.args(sym, src[i], slabs[i].psi, slabs[i].X, slabs[i].X, rows,
                             slabs[i].rank, nranks, neg));
      a.back().tile8 = 1;  // 8-mode tiles: whole-line row writes, shared column reads
      if (col0_direct) {
        // column m = 0 (packed DC / Nyquist): written straight into the rank's block of the
        // gather buffer by pass 0, read from the solved dense column G by pass 2
        a.back().col0 = G + slabs[i].row0;
        if (!late_cs) {
          a.back().fx = slabs[i].cs8;
          a.back().Hx = slabs[i].cs;
        }
        if (w_in_gather())
          a.back().wrows = TG + (size_t)slabs[i].rank * blk + tg_rows_off();
        if (psi_local()) {  // pass 2 also writes psi's two halo rows
          const Slab& sl = slabs[i];
          a.back().hx_H = sl.hx8;
          a.back().hx_lo = sl.ghost + 2 * (size_t)nx;
          a.back().hx_hi = sl.ghost + 3 * (size_t)nx;
          a.back().hx_c0lo = G + (sl.row0 + ny - 1) % ny;
          a.back().hx_c0hi = G + (sl.row0 + sl.rows) % ny;
        }
      }
    }
    for (size_t i = 0; i < a.size(); ++i) {
      FusedPoissonArgs a0 = a[i];
      if (col0_direct) a0.col0 = col_piece(slabs[i]);
      if (late_cs) {
        a0.cp = slabs[i].colpart[cp_idx[i]];
        a0.ncp = ncp;
        a0.csout = reinterpret_cast<double*>(cs_piece(slabs[i]));
      }
      tbegin(CFDJ_K_FFT_FWD);
      launch_fused_poisson_pass(0, a0, stream);
      tend();
    }
    if (!col0_direct) {  // column 0 of the tiled spectrum: element j at 8 j
      tbegin(CFDJ_K_COMM);
      for (auto& s : slabs) launch_strided_copy(col_piece(s), 1, s.X, 8, rows, stream);
      tend();
    }
    for (auto& s : slabs) {
      tbegin(CFDJ_K_DIVIDE);
      launch_schur_pass(0, schur_args(s), stream);
      tend();
    }
    if (mode == Mode::Rccl) {
      // on the main stream: both solves below wait for it anyway, and a hop to another stream
      // and back costs more than the exchange hides
      tbegin(CFDJ_K_COMM);
      comm_order();
      CFDJ_NCCL(ncclAllGather(reinterpret_cast<double*>(TG + (size_t)rank * blk), TG, 2 * blk,
                              ncclDouble, comm, stream));
      tend();
    }
    tbegin(CFDJ_K_DIVIDE);
    FusedPoissonArgs ga = fused.args(sym, nullptr, nullptr, G, G, ny, 0, 1, neg);
    if (col0_solve_supported(ny)) {
      if (late_cs)
        launch_col0_solve(ga, TG + (size_t)4 * L, blk, rows, G, stream, TG + (size_t)3 * L, nranks,
                          csT);
      else
        launch_col0_solve(ga, TG + (size_t)4 * L, blk, rows, G, stream);
    } else {
      for (int q = 0; q < nranks; ++q)
        launch_strided_copy(G + (size_t)q * rows, 1, TG + (size_t)q * blk + (size_t)4 * L, 1, rows,
                            stream);
      plans.exec(g_fwd, G, nullptr);
      PackedDivParams pd;
      pd.Z = G;
      pd.cx = sym.cx;
      pd.cy = sym.cy;
      pd.aa = sym.aa;
      pd.bb = sym.bb;
      pd.cc = sym.cc;
      pd.scale = sym.scale;
      pd.L = L;
      pd.ny = ny;
      pd.neg = neg;
      launch_packed_divide(pd, stream);
      plans.exec(g_inv, G, nullptr);
    }
    tend();
    for (auto& s : slabs) {
      tbegin(CFDJ_K_DIVIDE);
      launch_schur_pass(1, schur_args(s), stream);
      tend();
    }
    if (!col0_direct) {
      tbegin(CFDJ_K_COMM);
      for (auto& s : slabs) launch_strided_copy(s.X, 8, G + s.row0, 1, rows, stream);
      tend();
    }
    for (auto& ai : a) {
      tbegin(CFDJ_K_FFT_INV);
      launch_fused_poisson_pass(2, ai, stream);
      tend();
    }
  }

  StageParams stage_params(const Slab& s, const double* w, const double* wn, double* out,
                           double dt) const {
    StageParams p;
    p.w = w;
    p.s = s.psi;
    if (slab_mode()) {
      p.w_lo = s.ghost;
      p.w_hi = s.ghost + nx;
      p.s_lo = s.ghost + 2 * (size_t)nx;
      p.s_hi = s.ghost + 3 * (size_t)nx;
    } else {
      p.w_lo = w + (size_t)(rows - 1) * nx;
      p.w_hi = w;
      p.s_lo = s.psi + (size_t)(rows - 1) * nx;
      p.s_hi = s.psi;
    }
    p.wn = wn;
    p.out = out;
    p.nx = nx;
    p.ny = rows;
    p.y0 = 0;
    p.ycount = rows;
    p.colpart = nullptr;
    p.rows_per_wave = rows_per_wave;
    p.march = stage_march;
    p.stream = stream_loads_pay((size_t)nx * rows * sizeof(double));
    const double dx2 = dx * dx, dy2 = dy * dy;
    p.k.aa = 1.0 / (re * dx2);
    p.k.bb = 1.0 / (re * dy2);
    p.k.gg = 1.0 / ((4.0 * dx) * dy);
    p.k.hh = 1.0 / 3.0;
    p.k.dt = dt;
    p.k.c25dt = 0.25 * dt;
    p.k.c23 = 2.0 / 3.0;
    p.k.c23dt = (2.0 / 3.0) * dt;
    return p;
  }

  // One RHS evaluation on the stage input + the fused stage update.
  // stage 1: wn -> wa;  stage 2: (wa, wn) -> wb;  stage 3: (wb, wn) -> wn;  0: w -> out = r
  void stage(int st, double dt) {
    std::vector<const double*> src(slabs.size());
    for (size_t i = 0; i < slabs.size(); ++i)
      src[i] = st == 1 ? slabs[i].wn : st == 2 ? slabs[i].wa : slabs[i].wb;
    if (psi_local()) {
      stage_local_psi(st, dt, src);
      return;
    }
    if (slab_mode() && side && !timing && rows >= 3) {
      stage_overlapped(st, dt, src);
      return;
    }
    poisson(src, true);
    if (slab_mode()) {
      halo(false, src);
      std::vector<const double*> ps(slabs.size());
      for (size_t i = 0; i < slabs.size(); ++i) ps[i] = slabs[i].psi;
      halo(true, ps);
    }
    for (size_t i = 0; i < slabs.size(); ++i) {
      Slab& s = slabs[i];
      double* out = st == 1 ? s.wa : st == 2 ? s.wb : s.wn;
      tbegin(CFDJ_K_STAGE, st);
      StageParams p = stage_params(s, src[i], s.wn, out, dt);
      if (use_schur) {  // column-sum partials of the output for the next stage's Poisson
        const int oi = st == 1 ? 1 : st == 2 ? 2 : 0;
        p.colpart = s.colpart[oi];
        s.cp_valid[oi] = true;
      }
      launch_stage(st, p, stream);
      tend();
    }
  }

  // The y-slab stage of the substructured path: the omega halo exchange (on the side stream,
  // during the Poisson passes, where there is one), the solve -- which leaves psi AND its two
  // halo rows --, and the stage kernel over all rows in one launch.
  void stage_local_psi(int st, double dt, const std::vector<const double*>& src) {
    if (w_in_gather()) {
      // (nothing: the rows ride in the solve's gather)
    } else if (side && !timing) {
      CFDJ_HIP(hipEventRecord(ev_src, stream));
      CFDJ_HIP(hipStreamWaitEvent(side, ev_src, 0));
      halo(false, src, side);
      CFDJ_HIP(hipEventRecord(ev_whalo, side));
      whalo_pending = true;
    } else {
      halo(false, src);
    }
    poisson(src, true);
    comm_order();  // (a no-op where the Poisson path had a collective on the main stream)
    for (size_t i = 0; i < slabs.size(); ++i) {
      Slab& s = slabs[i];
      double* out = st == 1 ? s.wa : st == 2 ? s.wb : s.wn;
      tbegin(CFDJ_K_STAGE, st);
      StageParams p = stage_params(s, src[i], s.wn, out, dt);
      if (w_in_gather()) {
        p.w_lo = gathered_row(s, false);
        p.w_hi = gathered_row(s, true);
      }
      const int oi = st == 1 ? 1 : st == 2 ? 2 : 0;
      p.colpart = s.colpart[oi];
      s.cp_valid[oi] = true;
      launch_stage(st, p, stream);
      tend();
    }
  }

  // The y-slab stage with the exchanges on the side stream: omega halo during the Poisson
  // passes, psi halo during the interior rows of the stage kernel; the first and last rows
  // (which read the halo rows) run after it.  RCCL ranks (one slab), and virtual slabs created
  // with CFDJ_VIRTUAL_OVERLAP=1, which run the identical event schedule with device copies in
  // place of the collectives.
  void stage_overlapped(int st, double dt, const std::vector<const double*>& src) {
    CFDJ_HIP(hipEventRecord(ev_src, stream));
    CFDJ_HIP(hipStreamWaitEvent(side, ev_src, 0));
    halo(false, src, side);
    CFDJ_HIP(hipEventRecord(ev_whalo, side));
    whalo_pending = true;
    poisson(src, true);
    comm_order();  // (a no-op where the Poisson path had a collective on the main stream)
    CFDJ_HIP(hipEventRecord(ev_psi, stream));
    CFDJ_HIP(hipStreamWaitEvent(side, ev_psi, 0));
    std::vector<const double*> ps(slabs.size());
    for (size_t i = 0; i < slabs.size(); ++i) ps[i] = slabs[i].psi;
    halo(true, ps, side);
    CFDJ_HIP(hipEventRecord(ev_shalo, side));
    // interior rows first, then -- in one launch -- the first and the last row (which read
    // the halo rows) adding their values to their blocks' column partials: the stage kernel
    // sums a block in that order in a one-launch stage as well
    std::vector<StageParams> sp;
    for (size_t i = 0; i < slabs.size(); ++i) {
      Slab& s = slabs[i];
      double* out = st == 1 ? s.wa : st == 2 ? s.wb : s.wn;
      StageParams p = stage_params(s, src[i], s.wn, out, dt);
      if (use_schur) {
        const int oi = st == 1 ? 1 : st == 2 ? 2 : 0;
        p.colpart = s.colpart[oi];
        s.cp_valid[oi] = true;
      }
      p.y0 = 1;
      p.ycount = rows - 2;
      launch_stage(st, p, stream);
      sp.push_back(p);
    }
    CFDJ_HIP(hipStreamWaitEvent(stream, ev_shalo, 0));
    for (StageParams& p : sp) {
      p.y0 = 0;
      p.ycount = 1;
      p.y0b = rows - 1;
      p.ycount_b = 1;
      p.cp_accumulate = true;
      launch_stage(st, p, stream);
    }
  }

  // `n` back-to-back launches of ONE kernel of the step between two events on the handle's
  // stream: the per-launch device time the roofline is priced on (bench.py).  kernel =
  // CFDJ_KB_*; single-GPU fused handles only.  Clobbers the stage / spectrum buffers and
  // (stage 3) advances wn -- run it after the timed regions.
  double kernel_bench(int kernel, double dt, int n) {
    CFDJ_REQUIRE(mode == Mode::Single && use_fused,
                 "kernel bench needs a single-GPU handle on the fused Poisson path");
    CFDJ_REQUIRE(kernel >= CFDJ_KB_STAGE1 && kernel <= CFDJ_KB_ROWS_INV, "bad kernel id");
    CFDJ_REQUIRE(n >= 1, "launches must be >= 1");
    Slab& s = slabs[0];
    const FusedPoissonArgs a = fused.args(sym, s.wn, s.psi, spec, true);
    hipEvent_t e[2];
    CFDJ_HIP(hipEventCreate(&e[0]));
    CFDJ_HIP(hipEventCreate(&e[1]));
    float t = 0.f;
    try {
      CFDJ_HIP(hipEventRecord(e[0], stream));
      for (int i = 0; i < n; ++i) {
        switch (kernel) {
          case CFDJ_KB_STAGE1: launch_stage(1, stage_params(s, s.wn, s.wn, s.wa, dt), stream); break;
          case CFDJ_KB_STAGE2: launch_stage(2, stage_params(s, s.wa, s.wn, s.wb, dt), stream); break;
          case CFDJ_KB_STAGE3: launch_stage(3, stage_params(s, s.wb, s.wn, s.wn, dt), stream); break;
          default: launch_fused_poisson_pass(kernel - CFDJ_KB_ROWS_FWD, a, stream); break;
        }
      }
      CFDJ_HIP(hipEventRecord(e[1], stream));
      CFDJ_HIP(hipEventSynchronize(e[1]));
      CFDJ_HIP(hipEventElapsedTime(&t, e[0], e[1]));
    } catch (...) {
      (void)hipEventDestroy(e[0]);
      (void)hipEventDestroy(e[1]);
      throw;
    }
    (void)hipEventDestroy(e[0]);
    (void)hipEventDestroy(e[1]);
    return (double)t / n;
  }

  void steps_eager(double dt, int nsteps) {
    for (int n = 0; n < nsteps; ++n) {
      stage(1, dt);
      stage(2, dt);
      stage(3, dt);
    }
  }

  void invalidate_graph() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    gexec = nullptr;
    g_steps = -1;
  }

  void step_async(double dt, int nsteps) {
    if (nsteps == 0) return;
    // omega^n may have changed since the last step (upload, cfdj_vm_field_device users)
    for (auto& s : slabs) s.cp_valid[0] = false;
    // Graphs only around our own kernels (rocFFT calls are not captured), and never with
    // timing on: event-record nodes captured from hipEventRecord are not recorded on this
    // ROCm (hipEventElapsedTime -> invalid resource handle), so timed runs launch eagerly.
    if (!use_graph || timing || mode != Mode::Single || !use_fused) {
      steps_eager(dt, nsteps);
      return;
    }
    if (!gexec || g_dt != dt || g_steps != nsteps) {
      invalidate_graph();
      hipGraph_t g = nullptr;
      CFDJ_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
      try {
        steps_eager(dt, nsteps);
      } catch (...) {
        (void)hipStreamEndCapture(stream, &g);
        if (g) (void)hipGraphDestroy(g);
        throw;
      }
      CFDJ_HIP(hipStreamEndCapture(stream, &g));
      const hipError_t e = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      CFDJ_HIP(e);
      g_dt = dt;
      g_steps = nsteps;
    }
    CFDJ_HIP(hipGraphLaunch(gexec, stream));
  }

  void sync() {
    if (side) CFDJ_HIP(hipStreamSynchronize(side));
    CFDJ_HIP(hipStreamSynchronize(stream));
    harvest();
    if (check_finite) {
      CFDJ_HIP(hipMemsetAsync(d_flag, 0, sizeof(int), stream));
      for (auto& s : slabs) launch_check_finite(s.wn, (size_t)nx * s.rows, d_flag, stream);
      int flag = 0;
      CFDJ_HIP(hipMemcpyAsync(&flag, d_flag, sizeof(int), hipMemcpyDeviceToHost, stream));
      CFDJ_HIP(hipStreamSynchronize(stream));
      if (flag) throw Error{CFDJ_ERR_NONFINITE, "non-finite vorticity after step"};
    }
  }

  // side stream (default priority) and the events that order it against the main stream
  void create_side() {
    CFDJ_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    for (hipEvent_t* e : {&ev_src, &ev_whalo, &ev_psi, &ev_shalo})
      CFDJ_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }

  void init_buffers() {
    nxh = nx / 2 + 1;
    const int P = nranks;
    kb = (nxh + P - 1) / P;
    rows = ny / P;
    const size_t n = (size_t)nx * rows;
    for (auto& s : slabs) {
      s.rows = rows;
      s.row0 = s.rank * rows;
      s.wn = dalloc<double>(n);
      s.wa = dalloc<double>(n);
      s.wb = dalloc<double>(n);
      s.psi = dalloc<double>(n);
      if (slab_mode()) {
        s.ghost = dalloc<double>(4 * (size_t)nx);
        s.X = dalloc<double2>((size_t)nxh * rows);
        s.S = dalloc<double2>((size_t)P * kb * rows);
        s.Y = dalloc<double2>((size_t)ny * kb);
      }
    }
    if (slab_mode()) {
      size_t len_x = (size_t)nx, len_y = (size_t)ny;
      row_fwd = plans.add(rocfft_transform_type_real_forward, rocfft_placement_notinplace, 1,
                          &len_x, rows, nullptr);
      row_inv = plans.add(rocfft_transform_type_real_inverse, rocfft_placement_notinplace, 1,
                          &len_x, rows, nullptr);
      rocfft_plan_description desc = nullptr;
      CFDJ_FFT(rocfft_plan_description_create(&desc));
      size_t stride = (size_t)kb;
      CFDJ_FFT(rocfft_plan_description_set_data_layout(
          desc, rocfft_array_type_complex_interleaved, rocfft_array_type_complex_interleaved,
          nullptr, nullptr, 1, &stride, 1, 1, &stride, 1));
      col_fwd = plans.add(rocfft_transform_type_complex_forward, rocfft_placement_inplace, 1,
                          &len_y, kb, desc);
      col_inv = plans.add(rocfft_transform_type_complex_inverse, rocfft_placement_inplace, 1,
                          &len_y, kb, desc);
      rocfft_plan_description_destroy(desc);
      if (schur_ok(nx, ny, nranks)) {
        schur.init(nx, ny, dx, dy, eps, nranks);
        TG = dalloc<double2>((size_t)nranks * ((size_t)6 * (nx / 2) + (size_t)(ny / nranks)));
        G = dalloc<double2>((size_t)ny);
        csT = dalloc<double2>((size_t)nx / 2);
        CFDJ_HIP(hipMemset(csT, 0, (size_t)(nx / 2) * sizeof(double2)));
        if (const char* e = std::getenv("CFDJ_SLAB_LATE_CS")) late_cs_on = e[0] != '0';
        g_fwd = plans.add(rocfft_transform_type_complex_forward, rocfft_placement_inplace, 1,
                          &len_y, 1, nullptr);
        g_inv = plans.add(rocfft_transform_type_complex_inverse, rocfft_placement_inplace, 1,
                          &len_y, 1, nullptr);
        use_schur = true;
      }
    } else {
      size_t lens[2] = {(size_t)nx, (size_t)ny};
      fwd2d = plans.add(rocfft_transform_type_real_forward, rocfft_placement_notinplace, 2,
                        lens, 1, nullptr);
      inv2d = plans.add(rocfft_transform_type_real_inverse, rocfft_placement_notinplace, 2,
                        lens, 1, nullptr);
      spec = dalloc<double2>((size_t)nxh * ny);
    }
    plans.finalize(stream);
    d_flag = dalloc<int>(1);
    if (fused_ok(nx, ny, nranks)) {
      fused.init(nx, ny);
      use_fused = true;
    }
    if (use_schur && !fused.ready()) fused.init(nx, ny);  // row-pass twiddles
    if (use_schur) {
      for (auto& s : slabs) {
        s.cs8 = dalloc<double>((size_t)8 * nx);
        s.cs = dalloc<double2>((size_t)8 * (nx / 2));
        s.hx8 = dalloc<double2>((size_t)8 * (nx / 2));
        CFDJ_HIP(hipMemset(s.hx8, 0, (size_t)8 * (nx / 2) * sizeof(double2)));
      }
      alloc_colparts();
    }
  }

  ~cfdj_vm() {
    if (stream) (void)hipStreamSynchronize(stream);
    invalidate_graph();
    for (auto& s : slabs) s.destroy();
    plans.destroy();
    sym.destroy();
    fused.destroy();
    schur.destroy();
    dfree(TG);
    dfree(G);
    dfree(csT);
    dfree(spec);
    dfree(gather);
    dfree(d_flag);
    for (auto e : ev) (void)hipEventDestroy(e);
    if (side) (void)hipStreamSynchronize(side);
    for (hipEvent_t e : {ev_src, ev_whalo, ev_psi, ev_shalo})
      if (e) (void)hipEventDestroy(e);
    if (side) (void)hipStreamDestroy(side);
    if (comm) ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// =====================================================================================
// C ABI
// =====================================================================================
namespace {

cfdj_vm* new_vm(int nx, int ny, double dx, double dy, double re, double eps, int device,
                Mode mode, int nranks, int rank, int solo_rank = -1) {
  check_grid(nx, ny, dx, dy);
  CFDJ_REQUIRE(std::isfinite(re) && re != 0.0, "re must be finite and non-zero");
  CFDJ_REQUIRE(nranks >= 1 && ny % nranks == 0, "ny must be divisible by the rank count");
  CFDJ_REQUIRE(ny / nranks >= 2, "each slab needs at least 2 rows");
  CFDJ_REQUIRE(rank >= 0 && rank < nranks, "rank out of range");
  fft_setup();
  select_device(device);
  std::unique_ptr<cfdj_vm> h(new cfdj_vm);
  CFDJ_HIP(hipGetDevice(&h->device));
  h->mode = mode;
  h->nx = nx;
  h->ny = ny;
  h->dx = dx;
  h->dy = dy;
  h->re = re;
  h->eps = eps;
  h->nranks = nranks;
  h->rank = rank;
  // rows per wavefront of the marching stage kernel, from sweeps of the whole step: one GPU
  // (grids the row-group kernel does not take) 32 from 2048 rows on, else 8; a y-slab of 8 M
  // cells and more 16 -- the tall-tile kernel's block, which the substructured path's slabs
  // then run (8192^2 / 8: 45 us per launch against 50 for the marching kernel at its best
  // setting) -- and 8 below (4096^2 / 4 and / 8: the marching kernel is 2 % ahead on the step)
  if (nranks == 1) h->rows_per_wave = ny >= 2048 ? 32 : 8;
  else h->rows_per_wave = (long long)nx * (ny / nranks) >= (1LL << 23) ? 16 : 8;
  if (const char* e = std::getenv("CFDJ_SLAB_ROWS_PER_WAVE")) {  // (tests, A/B runs)
    const int v = std::atoi(e);
    if (nranks > 1 && v >= 1) h->rows_per_wave = v;
  }
  CFDJ_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  if (mode == Mode::Virtual && solo_rank >= 0) {
    // one rank's share of the nranks-rank step, alone on this GPU: its slab only, every
    // exchange a copy from itself (timing rehearsal: the field is not the global solution)
    h->slabs.resize(1);
    h->slabs[0].rank = solo_rank;
  } else if (mode == Mode::Virtual) {
    h->slabs.resize(nranks);
    for (int p = 0; p < nranks; ++p) h->slabs[p].rank = p;
  } else {
    h->slabs.resize(1);
    h->slabs[0].rank = rank;
  }
  h->sym.init(nx, ny, dx, dy, eps);
  h->init_buffers();
  return h.release();
}

void check_ld(long ld, long need, const char* what) {
  if (ld < need) throw Error{CFDJ_ERR_ARG, std::string(what) + ": leading dimension too small"};
}

// Reference ghost fill of a ghosted (nx+2)x(ny+2) column-major array, vm.jl:68-76 /
// Common.jl:138-146 order: row nx+2 <- 2, col ny+2 <- 2, row 1 <- nx+1, col 1 <- ny+1.
void ghost_fill(double* g, long ld, int nx, int ny) {
  auto at = [&](int i, int j) -> double& { return g[(size_t)(i - 1) + (size_t)(j - 1) * ld]; };
  for (int j = 1; j <= ny + 2; ++j) at(nx + 2, j) = at(2, j);
  for (int i = 1; i <= nx + 2; ++i) at(i, ny + 2) = at(i, 2);
  for (int j = 1; j <= ny + 2; ++j) at(1, j) = at(nx + 1, j);
  for (int i = 1; i <= nx + 2; ++i) at(i, 1) = at(i, ny + 1);
}

}  // namespace

extern "C" {

const char* cfdj_last_error(void) { return g_err.c_str(); }

// 01_Heat_Equation_FTCS/ftcs.jl:34-41 -- host code (BASELINE config 1 is CPU plumbing only).
int cfdj_ftcs(int nx, int nt, double beta, const double* u0, double* un, long ldu) {
  return guard([&] {
    CFDJ_REQUIRE(nx >= 2 && nt >= 0 && u0 && un && ldu >= nx + 1, "bad arguments");
    for (int i = 0; i <= nx; ++i) un[i] = u0[i];
    for (int k = 1; k <= nt; ++k) {
      const double* a = un + (size_t)(k - 1) * ldu;
      double* b = un + (size_t)k * ldu;
      for (int i = 1; i < nx; ++i) b[i] = a[i] + beta * (a[i + 1] - 2.0 * a[i] + a[i - 1]);
      b[0] = 0.0;   // boundary condition at x = -1 (ftcs.jl:39)
      b[nx] = 0.0;  // boundary condition at x = 1 (ftcs.jl:40)
    }
  });
}

const char* cfdj_version(void) { return "cfdj 0.1.0 (gfx950)"; }

int cfdj_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ---- Poisson ---------------------------------------------------------------------------
int cfdj_fps_create(int nx, int ny, double dx, double dy, double eps, int device,
                    cfdj_fps_plan** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr, "out is NULL");
    *out = nullptr;
    check_grid(nx, ny, dx, dy);
    fft_setup();
    select_device(device);
    std::unique_ptr<cfdj_fps_plan> h(new cfdj_fps_plan);
    CFDJ_HIP(hipGetDevice(&h->device));
    CFDJ_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->sym.init(nx, ny, dx, dy, eps);
    h->dx = dx;
    h->dy = dy;
    h->eps = eps;
    size_t lens[2] = {(size_t)nx, (size_t)ny};
    h->fwd = h->plans.add(rocfft_transform_type_real_forward, rocfft_placement_notinplace, 2,
                          lens, 1, nullptr);
    h->inv = h->plans.add(rocfft_transform_type_real_inverse, rocfft_placement_notinplace, 2,
                          lens, 1, nullptr);
    h->plans.finalize(h->stream);
    h->spec = dalloc<double2>((size_t)h->sym.nxh * ny);
    h->f_dev = dalloc<double>((size_t)nx * ny);
    h->s_dev = dalloc<double>((size_t)nx * ny);
    if (fused_ok(nx, ny, 1)) {
      h->fused.init(nx, ny);
      h->use_fused = true;
    }
    // set-up, the plan's device current: only plans that can use the static scratch look its
    // address up (a failing lookup must not break plans on the library-FFT path)
    if (h->use_fused) h->static_spec = noalloc_scratch_init();
    *out = h.release();
  });
}

int cfdj_fps_solve(cfdj_fps_plan* h, const double* f, long ldf, double* s, long lds) {
  return guard([&] {
    CFDJ_REQUIRE(h && f && s, "NULL argument");
    const int nx = h->sym.nx, ny = h->sym.ny;
    check_ld(ldf, nx, "ldf");
    check_ld(lds, nx, "lds");
    select_device(h->device);
    CFDJ_HIP(hipMemcpy2DAsync(h->f_dev, nx * sizeof(double), f, ldf * sizeof(double),
                              nx * sizeof(double), ny, hipMemcpyHostToDevice, h->stream));
    h->solve_device(h->f_dev, h->s_dev);
    CFDJ_HIP(hipMemcpy2DAsync(s, lds * sizeof(double), h->s_dev, nx * sizeof(double),
                              nx * sizeof(double), ny, hipMemcpyDeviceToHost, h->stream));
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_fps_solve_device(cfdj_fps_plan* h, const double* f_dev, double* s_dev) {
  return guard([&] {
    CFDJ_REQUIRE(h && f_dev && s_dev, "NULL argument");
    select_device(h->device);
    h->solve_device(f_dev, s_dev);
  });
}

// The same solve with the half spectrum in the library's static device array: no
// hipMalloc / hipFree / rocFFT call on this path (only the three hand-written passes).
int cfdj_fps_solve_device_noalloc(cfdj_fps_plan* h, const double* f_dev, double* s_dev) {
  return guard([&] {
    CFDJ_REQUIRE(h && f_dev && s_dev, "NULL argument");
    CFDJ_REQUIRE(h->use_fused,
                 "cfdj_fps_solve_device_noalloc needs a plan on the hand-written FFT path "
                 "(power-of-two nx, ny >= 1024, ny <= nx): rocFFT may allocate");
    const size_t need = (size_t)(h->sym.nx / 2) * (size_t)h->sym.ny;
    if (need > kNoAllocMaxSpectrum)
      throw Error{CFDJ_ERR_ARG, "cfdj_fps_solve_device_noalloc: (nx/2)*ny = " +
                                    std::to_string(need) + " complex elements exceed the static "
                                    "scratch of " + std::to_string(kNoAllocMaxSpectrum) +
                                    " (e.g. 2048 x 1024); use cfdj_fps_solve_device"};
    CFDJ_REQUIRE(h->static_spec != nullptr, "static scratch not initialised");
    select_device(h->device);
    // nothing in the scratch has to start at zero: the row pass writes every element of
    // the (nx/2) x ny spectrum before the column pass reads it
    h->solve_device(f_dev, s_dev, h->static_spec);
  });
}

int cfdj_fps_stream(cfdj_fps_plan* h, void** hip_stream) {
  return guard([&] {
    CFDJ_REQUIRE(h && hip_stream, "NULL argument");
    *hip_stream = static_cast<void*>(h->stream);
  });
}

void cfdj_fps_destroy(cfdj_fps_plan* h) {
  if (!h) return;
  (void)guard([&] {
    select_device(h->device);
    delete h;
  });
}

int cfdj_fps(int nx, int ny, double dx, double dy, double eps, const double* f, long ldf,
             double* s, long lds) {
  cfdj_fps_plan* h = nullptr;
  int rc = cfdj_fps_create(nx, ny, dx, dy, eps, -1, &h);
  if (rc != CFDJ_OK) return rc;
  rc = cfdj_fps_solve(h, f, ldf, s, lds);
  cfdj_fps_destroy(h);
  return rc;
}

// ---- vortex merger -------------------------------------------------------------------
int cfdj_vm_create(int nx, int ny, double dx, double dy, double re, double eps, int device,
                   cfdj_vm** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr, "out is NULL");
    *out = nullptr;
    *out = new_vm(nx, ny, dx, dy, re, eps, device, Mode::Single, 1, 0);
  });
}

int cfdj_vm_create_virtual(int nx, int ny, double dx, double dy, double re, double eps,
                           int device, int nranks, cfdj_vm** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr, "out is NULL");
    *out = nullptr;
    // CFDJ_VIRTUAL_SOLO_RANK=r: only rank r's slab (a timing rehearsal of one rank's compute)
    int solo = -1;
    if (const char* sr = std::getenv("CFDJ_VIRTUAL_SOLO_RANK")) {
      solo = std::atoi(sr);
      CFDJ_REQUIRE(solo >= 0 && solo < nranks, "CFDJ_VIRTUAL_SOLO_RANK out of range");
    }
    std::unique_ptr<cfdj_vm> h(
        new_vm(nx, ny, dx, dy, re, eps, device, Mode::Virtual, nranks, 0, solo));
    // CFDJ_VIRTUAL_OVERLAP=1: the RCCL ranks' side-stream schedule (halo exchanges behind
    // events, interior / edge split of the stage kernel) with device copies standing in for
    // the exchanges -- the event graph of the multi-GPU step on one GPU
    const char* ov = std::getenv("CFDJ_VIRTUAL_OVERLAP");
    if (ov && ov[0] == '1') h->create_side();
    if (solo >= 0) {
      // what the absent ranks would have delivered: zeros (finite, so the step stays sane)
      auto zero = [](void* p, size_t bytes) {
        if (p) CFDJ_HIP(hipMemset(p, 0, bytes));
      };
      zero(h->TG, (size_t)nranks * h->tg_block() * sizeof(double2));
      zero(h->G, (size_t)ny * sizeof(double2));
      Slab& sl = h->slabs[0];
      zero(sl.X, (size_t)h->nxh * h->rows * sizeof(double2));
      zero(sl.S, (size_t)nranks * h->kb * h->rows * sizeof(double2));
      zero(sl.Y, (size_t)ny * h->kb * sizeof(double2));
    }
    *out = h.release();
  });
}

int cfdj_comm_unique_id(void* out128) {
  return guard([&] {
    CFDJ_REQUIRE(out128 != nullptr, "out is NULL");
    ncclUniqueId id;
    CFDJ_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out128, &id, sizeof(id));
  });
}

int cfdj_vm_create_dist(int nx, int ny, double dx, double dy, double re, double eps,
                        int device, int rank, int nranks, const void* nccl_id,
                        cfdj_vm** out) {
  return guard([&] {
    CFDJ_REQUIRE(out != nullptr && nccl_id != nullptr, "NULL argument");
    *out = nullptr;
    // One rank: the single-GPU path, unless CFDJ_FORCE_SLAB=1 asks for the RCCL slab code
    // with a one-rank communicator (self send/recv + all-to-all) -- the only way to run
    // the RCCL path on a one-GPU machine (RCCL refuses two ranks on one device).
    const char* force = std::getenv("CFDJ_FORCE_SLAB");
    if (nranks == 1 && !(force && force[0] == '1')) {
      *out = new_vm(nx, ny, dx, dy, re, eps, device, Mode::Single, 1, 0);
      return;
    }
    std::unique_ptr<cfdj_vm> h(new_vm(nx, ny, dx, dy, re, eps, device, Mode::Rccl, nranks,
                                      rank));
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof(id));
    CFDJ_NCCL(ncclCommInitRank(&h->comm, nranks, id, rank));
    // halo overlap (CFDJ_NO_OVERLAP=1: everything on one stream, for A/B runs)
    const char* no_ov = std::getenv("CFDJ_NO_OVERLAP");
    if (!(no_ov && no_ov[0] == '1')) h->create_side();
    *out = h.release();
  });
}

int cfdj_vm_comm_ranks(cfdj_vm* h, int* ranks) {
  return guard([&] {
    CFDJ_REQUIRE(h && ranks, "NULL argument");
    *ranks = 0;
    if (h->comm) CFDJ_NCCL(ncclCommCount(h->comm, ranks));
  });
}

int cfdj_vm_upload(cfdj_vm* h, const double* w, long ldw) {
  return guard([&] {
    CFDJ_REQUIRE(h && w, "NULL argument");
    check_ld(ldw, (long)h->nx + 2, "ldw");
    select_device(h->device);
    const int nx = h->nx;
    for (auto& s : h->slabs) {
      const double* src = w + 1 + (size_t)(1 + s.row0) * ldw;  // &w[2, 2 + row0]
      CFDJ_HIP(hipMemcpy2DAsync(s.wn, nx * sizeof(double), src, ldw * sizeof(double),
                                nx * sizeof(double), s.rows, hipMemcpyHostToDevice,
                                h->stream));
    }
    CFDJ_HIP(hipStreamSynchronize(h->stream));
  });
}

int cfdj_vm_download(cfdj_vm* h, double* w, long ldw) {
  return guard([&] {
    CFDJ_REQUIRE(h && w, "NULL argument");
    check_ld(ldw, (long)h->nx + 2, "ldw");
    select_device(h->device);
    const int nx = h->nx;
    double* dst = w + 1 + ldw;  // &w[2,2]
    if (h->mode == Mode::Rccl) {
      if (!h->gather) h->gather = dalloc<double>((size_t)nx * h->ny);
      CFDJ_NCCL(ncclAllGather(h->slabs[0].wn, h->gather, (size_t)nx * h->rows, ncclDouble,
                              h->comm, h->stream));
      CFDJ_HIP(hipMemcpy2DAsync(dst, ldw * sizeof(double), h->gather, nx * sizeof(double),
                                nx * sizeof(double), h->ny, hipMemcpyDeviceToHost,
                                h->stream));
    } else {
      for (auto& s : h->slabs)
        CFDJ_HIP(hipMemcpy2DAsync(dst + (size_t)s.row0 * ldw, ldw * sizeof(double), s.wn,
                                  nx * sizeof(double), nx * sizeof(double), s.rows,
                                  hipMemcpyDeviceToHost, h->stream));
    }
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    ghost_fill(w, ldw, nx, h->ny);
  });
}

int cfdj_vm_step_async(cfdj_vm* h, double dt, int nsteps) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(nsteps >= 0, "nsteps must be >= 0");
    CFDJ_REQUIRE(std::isfinite(dt), "dt must be finite");
    select_device(h->device);
    h->step_async(dt, nsteps);
  });
}

int cfdj_vm_sync(cfdj_vm* h) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    select_device(h->device);
    h->sync();
  });
}

int cfdj_vm_step(cfdj_vm* h, double dt, int nsteps) {
  int rc = cfdj_vm_step_async(h, dt, nsteps);
  if (rc != CFDJ_OK) return rc;
  return cfdj_vm_sync(h);
}

int cfdj_vm_rhs(cfdj_vm* h, const double* w, long ldw, double* r, long ldr, double* s,
                long lds) {
  return guard([&] {
    CFDJ_REQUIRE(h && w && r && s, "NULL argument");
    CFDJ_REQUIRE(h->mode != Mode::Rccl, "cfdj_vm_rhs needs a single-GPU or virtual-slab handle");
    check_ld(ldw, (long)h->nx + 2, "ldw");
    check_ld(ldr, (long)h->nx + 2, "ldr");
    check_ld(lds, (long)h->nx + 2, "lds");
    select_device(h->device);
    const int nx = h->nx, ny = h->ny;
    const size_t rowb = nx * sizeof(double);
    std::vector<const double*> src;
    for (auto& sl : h->slabs) {
      sl.cp_valid[1] = sl.cp_valid[2] = false;  // wa / wb are scratch here
      CFDJ_HIP(hipMemcpy2DAsync(sl.wa, rowb, w + 1 + (size_t)(1 + sl.row0) * ldw,
                                ldw * sizeof(double), rowb, sl.rows, hipMemcpyHostToDevice,
                                h->stream));
      src.push_back(sl.wa);
    }
    h->poisson(src, true);
    if (h->slab_mode()) {
      h->halo(false, src);
      std::vector<const double*> ps;
      for (auto& sl : h->slabs) ps.push_back(sl.psi);
      h->halo(true, ps);
    }
    for (auto& sl : h->slabs) {
      h->tbegin(CFDJ_K_STAGE);
      launch_stage(0, h->stage_params(sl, sl.wa, sl.wa, sl.wb, 0.0), h->stream);
      h->tend();
      CFDJ_HIP(hipMemcpy2DAsync(r + 1 + (size_t)(1 + sl.row0) * ldr, ldr * sizeof(double), sl.wb,
                                rowb, rowb, sl.rows, hipMemcpyDeviceToHost, h->stream));
      CFDJ_HIP(hipMemcpy2DAsync(s + 1 + (size_t)(1 + sl.row0) * lds, lds * sizeof(double),
                                sl.psi, rowb, rowb, sl.rows, hipMemcpyDeviceToHost, h->stream));
    }
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    h->harvest();
    ghost_fill(s, lds, nx, ny);
  });
}

int cfdj_vm_set_timing(cfdj_vm* h, int enable) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    h->harvest();
    h->timing = enable != 0;
    for (int k = 0; k < CFDJ_K_COUNT; ++k) {
      h->ms[k] = 0.0;
      h->launches[k] = 0;
    }
    for (int k = 0; k < 3; ++k) {
      h->stage_ms[k] = 0.0;
      h->stage_launches[k] = 0;
    }
  });
}

int cfdj_vm_stage_timing(cfdj_vm* h, double* ms3, long* launches3) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    for (int k = 0; k < 3; ++k) {
      if (ms3) ms3[k] = h->stage_ms[k];
      if (launches3) launches3[k] = h->stage_launches[k];
    }
  });
}

int cfdj_vm_timing(cfdj_vm* h, double* ms, long* launches) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    for (int k = 0; k < CFDJ_K_COUNT; ++k) {
      if (ms) ms[k] = h->ms[k];
      if (launches) launches[k] = h->launches[k];
    }
  });
}

int cfdj_vm_kernel_bench(cfdj_vm* h, int kernel, double dt, int launches,
                         double* ms_per_launch) {
  return guard([&] {
    CFDJ_REQUIRE(h && ms_per_launch, "NULL argument");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    *ms_per_launch = h->kernel_bench(kernel, dt, launches);
  });
}

int cfdj_vm_set_check_finite(cfdj_vm* h, int enable) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    h->check_finite = enable != 0;
  });
}

int cfdj_vm_field_device(cfdj_vm* h, double** w_dev) {
  return guard([&] {
    CFDJ_REQUIRE(h && w_dev, "NULL argument");
    CFDJ_REQUIRE(h->mode != Mode::Virtual, "virtual-rank handles hold several slabs");
    *w_dev = h->slabs[0].wn;
  });
}

int cfdj_vm_slab(cfdj_vm* h, int* row0, int* rows) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    // virtual handles hold every slab (the whole grid), except the one-rank rehearsal
    const bool all = h->mode == Mode::Virtual && (int)h->slabs.size() == h->nranks;
    if (row0) *row0 = all ? 0 : h->slabs[0].row0;
    if (rows) *rows = all ? h->ny : h->rows;
  });
}

int cfdj_vm_set_rows_per_wave(cfdj_vm* h, int rows) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(rows >= 1, "rows must be >= 1");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    h->rows_per_wave = rows;
    h->stage_march = true;
    if (h->use_schur) h->alloc_colparts();  // partial blocks follow the wave row ranges
    h->invalidate_graph();
  });
}

int cfdj_vm_stage_kernel(cfdj_vm* h, int* row_group) {
  return guard([&] {
    CFDJ_REQUIRE(h && row_group, "NULL argument");
    Slab& s = h->slabs[0];
    StageParams p = h->stage_params(s, s.wn, s.wn, s.wa, 0.0);
    if (h->use_schur) p.colpart = s.colpart[1];
    *row_group = stage_runs_row_group(p) ? 1 : 0;
  });
}

int cfdj_vm_set_poisson(cfdj_vm* h, int path) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(path >= CFDJ_POISSON_AUTO && path <= CFDJ_POISSON_SCHUR, "bad path");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    const bool can_schur = h->slab_mode() && h->schur.ready();
    if (path == CFDJ_POISSON_SCHUR && !can_schur)
      throw Error{CFDJ_ERR_ARG, "substructured Poisson needs y-slabs of a square power-of-two "
                                "grid with 512..4096 rows per rank"};
    const bool sc = path == CFDJ_POISSON_SCHUR || (path == CFDJ_POISSON_AUTO && can_schur);
    const bool f = sc ? h->use_fused : resolve_fused(path, h->nx, h->ny, h->nranks);
    if (f && !h->fused.ready()) h->fused.init(h->nx, h->ny);
    h->use_fused = f;
    h->use_schur = sc;
    h->invalidate_graph();
  });
}

int cfdj_vm_set_graph(cfdj_vm* h, int enable) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    h->use_graph = enable != 0;
    h->invalidate_graph();
  });
}

int cfdj_vm_get_poisson(cfdj_vm* h) {
  if (!h) return CFDJ_ERR_ARG;
  if (h->use_schur) return CFDJ_POISSON_SCHUR;
  return h->use_fused ? CFDJ_POISSON_FUSED : CFDJ_POISSON_ROCFFT;
}

int cfdj_fps_get_poisson(cfdj_fps_plan* h) {
  if (!h) return CFDJ_ERR_ARG;
  return h->use_fused ? CFDJ_POISSON_FUSED : CFDJ_POISSON_ROCFFT;
}

int cfdj_fps_set_symbol(cfdj_fps_plan* h, int kind) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(kind == CFDJ_SYMBOL_FD || kind == CFDJ_SYMBOL_SPECTRAL, "bad symbol kind");
    select_device(h->device);
    CFDJ_HIP(hipStreamSynchronize(h->stream));
    const int nx = h->sym.nx, ny = h->sym.ny;
    h->sym.destroy();
    h->sym.init(nx, ny, h->dx, h->dy, h->eps, kind);
  });
}

int cfdj_fps_set_poisson(cfdj_fps_plan* h, int path) {
  return guard([&] {
    CFDJ_REQUIRE(h != nullptr, "NULL handle");
    CFDJ_REQUIRE(path >= CFDJ_POISSON_AUTO && path <= CFDJ_POISSON_FUSED, "bad path");
    select_device(h->device);
    const bool f = resolve_fused(path, h->sym.nx, h->sym.ny, 1);
    if (f && !h->fused.ready()) h->fused.init(h->sym.nx, h->sym.ny);
    if (f && !h->static_spec) h->static_spec = noalloc_scratch_init();
    h->use_fused = f;
  });
}

void cfdj_vm_destroy(cfdj_vm* h) {
  if (!h) return;
  (void)guard([&] {
    select_device(h->device);
    delete h;
  });
}

}  // extern "C"
