/*
 * cfdj.h -- C ABI of libcfdj.so, the MI355X (gfx950) implementation of the
 * t-bltg/CFD_Julia 2D vorticity-streamfunction Navier-Stokes hot path.
 *
 * The reference has no FFI: its "boundary" is a plain Julia call.  Each entry point
 * below replaces one reference function (cited file:line, relative to the reference
 * repository root) and keeps that function's argument meaning:
 *
 *   - arrays are caller-owned, column-major (x = Julia's first index is contiguous),
 *     passed as (pointer, leading dimension in elements); a pointer may address any
 *     element, e.g. &s[2,2] of a ghosted array, exactly as a Julia `pointer(s, k)`;
 *   - host arrays are touched only during the call; every call that moves data
 *     synchronises the handle's HIP stream before returning;
 *   - device memory, rocFFT plans, HIP streams/events and RCCL communicators are owned
 *     by the opaque handle;
 *   - all functions return CFDJ_OK (0) or a negative CFDJ_ERR_* code; no C++ exception
 *     crosses the ABI; cfdj_last_error() returns a thread-local message;
 *   - one host thread per handle at a time.
 *
 * Julia binding: julia/CFDJ.jl.  Python binding: cfd_julia_amd/_lib.py (ctypes).
 */
#ifndef CFDJ_H_
#define CFDJ_H_

#ifdef __cplusplus
extern "C" {
#endif

#define CFDJ_OK 0
#define CFDJ_ERR_ARG -1       /* bad size/pointer/argument (Julia: BoundsError, DivideError) */
#define CFDJ_ERR_HIP -2       /* HIP runtime failure (out of memory, launch failure, ...) */
#define CFDJ_ERR_ROCFFT -3    /* rocFFT plan/execute failure */
#define CFDJ_ERR_RCCL -4      /* RCCL communicator / collective failure */
#define CFDJ_ERR_NONFINITE -5 /* non-finite vorticity detected (optional check) */
#define CFDJ_ERR_STATE -6     /* call not valid in the handle's current state */

/* Kernel-category indices for cfdj_vm_timing(). */
#define CFDJ_K_STAGE 0    /* fused Arakawa Jacobian + 5-pt Laplacian + RK3 stage kernel */
#define CFDJ_K_FFT_FWD 1  /* forward transforms: hand-written row r2c pass, or rocFFT D2Z */
#define CFDJ_K_DIVIDE 2   /* column pass (FFT + divide by the FD symbol, Common.jl:119-121, +
                             inverse FFT), the substructured y-solve, or the divide kernel */
#define CFDJ_K_FFT_INV 3  /* inverse transforms: hand-written row c2r pass, or rocFFT Z2D */
#define CFDJ_K_COMM 4     /* collectives and halo exchanges (multi-GPU only) */
#define CFDJ_K_COUNT 5

/* Poisson implementation (cfdj_vm_set_poisson / cfdj_fps_set_poisson). */
#define CFDJ_POISSON_AUTO 0   /* fused where supported, rocFFT otherwise (default) */
#define CFDJ_POISSON_ROCFFT 1 /* rocFFT D2Z + divide kernel + rocFFT Z2D */
#define CFDJ_POISSON_FUSED 2  /* hand-written 3-pass FFT: power-of-two nx 1024..16384,
                                 ny 1024..8192, power-of-two rank counts (on y-slabs:
                                 all-to-all transposes of the half spectrum) */
#define CFDJ_POISSON_SCHUR 3  /* y-slabs only: hand-written row FFTs + substructured y-solve
                                 (chunked tridiagonal interiors, P x P separator system; one
                                 all-gather of 48 B per x-mode and three rows per rank instead
                                 of transposes -- it also carries the stencil's halo rows);
                                 square power-of-two grids up to 16384^2, 512..4096 rows per
                                 rank.  AUTO on y-slabs picks it where supported. */

/* Poisson symbol (cfdj_fps_set_symbol). */
#define CFDJ_SYMBOL_FD 0       /* Common.jl:119-121 / fft_p.jl:37-39: aa + bb cos kx + cc cos ky */
#define CFDJ_SYMBOL_SPECTRAL 1 /* 13_Poisson_Solver_FFT_Spectral/fft_s.jl:32-34: -kx^2 - ky^2 */

typedef struct cfdj_vm cfdj_vm;   /* periodic vortex-merger solver state */
typedef struct cfdj_fps_plan cfdj_fps_plan; /* periodic FD-FFT Poisson solver */

/* ---- library ------------------------------------------------------------------ */
const char* cfdj_last_error(void);
const char* cfdj_version(void);
/* Number of visible HIP devices (0 without a GPU; never fails). */
int cfdj_device_count(void);

/* ---- periodic FD-FFT Poisson: Common.jl:97-125 `fps`, fft_p.jl:8-42 `ps_fft` ------
 * Solves  (u[i+1,j]-2u[i,j]+u[i-1,j])/dx^2 + (u[i,j+1]-2u[i,j]+u[i,j-1])/dy^2 = f
 * on the periodic nx-by-ny grid with the reference's symbol
 *   aa + bb*cos(kx_i) + cc*cos(ky_j),  kx[1] = eps,  ky = kx,  e[1,1] = 0.
 * Requires nx even and ny <= nx (Common.jl:108,113).  The plan is built once per
 * handle (the reference re-plans on every call). */
int cfdj_fps_create(int nx, int ny, double dx, double dy, double eps, int device,
                    cfdj_fps_plan** out);
/* f: nx-by-ny host array (ldf >= nx) -> s: nx-by-ny host block (lds >= nx).
 * Common.jl:97 writes s[2:nx+1, 2:ny+1]: pass &s[2,2] and lds = nx+2. */
int cfdj_fps_solve(cfdj_fps_plan* h, const double* f, long ldf, double* s, long lds);
/* Same, on device pointers (contiguous, pitch nx) on the handle's stream; no sync. */
int cfdj_fps_solve_device(cfdj_fps_plan* h, const double* f_dev, double* s_dev);
/* No counterpart in the reference: cfdj_fps_solve_device for callers that cannot allocate
 * device memory (tight serving loops, harnesses that forbid hipMalloc, code that captures
 * the plan's stream -- cfdj_fps_stream -- into a HIP graph).  The half spectrum lives in a
 * static device array of the library instead of the plan's buffer; the call itself runs only
 * the three hand-written FFT passes on the plan's stream (no hipMalloc / hipFree / rocFFT),
 * no sync.  Limits: a plan on the
 * CFDJ_POISSON_FUSED path and (nx/2)*ny <= 1048576 complex elements (16 MiB, e.g.
 * 2048 x 1024 or 1024 x 1024); larger or rocFFT-path plans return CFDJ_ERR_ARG.  All calls
 * on one GPU share that GPU's array (any plan, any stream): calls that overlap on one GPU
 * race; nothing in it needs clearing between calls. */
int cfdj_fps_solve_device_noalloc(cfdj_fps_plan* h, const double* f_dev, double* s_dev);
/* The plan's HIP stream (a hipStream_t, created hipStreamNonBlocking) on which
 * cfdj_fps_solve_device and cfdj_fps_solve_device_noalloc enqueue their kernels: for callers
 * that order their own work against the solve (events, hipStreamSynchronize) or capture it. */
int cfdj_fps_stream(cfdj_fps_plan* h, void** hip_stream);
/* Select the Poisson implementation (CFDJ_POISSON_*); ARG error if unsupported. */
int cfdj_fps_set_poisson(cfdj_fps_plan* h, int path);
/* The implementation in use (CFDJ_POISSON_ROCFFT or CFDJ_POISSON_FUSED; ARG on NULL). */
int cfdj_fps_get_poisson(cfdj_fps_plan* h);
/* Select the symbol: CFDJ_SYMBOL_FD (default, fps/ps_fft) or CFDJ_SYMBOL_SPECTRAL
 * (fft_s.jl:8-37 ps_spectral: kx = 2pi/(nx dx) * index, kx[1] = eps, ky = kx). */
int cfdj_fps_set_symbol(cfdj_fps_plan* h, int kind);
void cfdj_fps_destroy(cfdj_fps_plan* h);
/* One-shot convenience with the reference's per-call semantics. */
int cfdj_fps(int nx, int ny, double dx, double dy, double eps, const double* f, long ldf,
             double* s, long lds);

/* ---- periodic vortex merger: vm.jl:12-90 `numerical`, Common.jl:132-182 `vm_rhs` --
 * nx-by-ny periodic grid; re = Reynolds number; eps = the fps wavenumber guard (1e-6).
 * device = HIP device ordinal (-1: current device). */
int cfdj_vm_create(int nx, int ny, double dx, double dy, double re, double eps,
                   int device, cfdj_vm** out);
/* Multi-GPU y-slab variant (one process per GPU).  rank/nranks: this process's slot;
 * nccl_id: 128-byte RCCL unique id from cfdj_comm_unique_id() on rank 0, broadcast by
 * the host.  Rank p owns global rows [p*ny/nranks, (p+1)*ny/nranks).  ny % nranks == 0. */
int cfdj_vm_create_dist(int nx, int ny, double dx, double dy, double re, double eps,
                        int device, int rank, int nranks, const void* nccl_id,
                        cfdj_vm** out);
int cfdj_comm_unique_id(void* out128);
/* Number of ranks of the handle's RCCL communicator as RCCL itself reports it
 * (ncclCommCount); 0 for handles without a communicator (single-GPU, virtual slabs). */
int cfdj_vm_comm_ranks(cfdj_vm* h, int* ranks);
/* Virtual-rank variant for testing the slab decomposition on ONE GPU: nranks slabs,
 * halo exchange and FFT transposes by device copies in one process. */
int cfdj_vm_create_virtual(int nx, int ny, double dx, double dy, double re, double eps,
                           int device, int nranks, cfdj_vm** out);

/* Load the vorticity from a reference-layout ghosted (nx+2)-by-(ny+2) host array
 * (vm.jl:117; ldw >= nx+2).  The interior w[2:nx+1, 2:ny+1] is authoritative; ghosts
 * are periodic copies in every reference caller (vm.jl:121-128, tgv.jl:119-123).
 * Distributed handles take the FULL global array on every rank and keep their slab. */
int cfdj_vm_upload(cfdj_vm* h, const double* w, long ldw);
/* Store the vorticity into a ghosted (nx+2)-by-(ny+2) host array, ghosts filled in the
 * order of vm.jl:68-76.  Distributed handles: every rank receives the global field. */
int cfdj_vm_download(cfdj_vm* h, double* w, long ldw);
/* nsteps SSP-RK3 steps of size dt (vm.jl:24-87, without the text snapshots), fully
 * device-resident; returns after the stream has drained. */
int cfdj_vm_step(cfdj_vm* h, double dt, int nsteps);
/* Enqueue nsteps steps without waiting (pair with cfdj_vm_sync). */
int cfdj_vm_step_async(cfdj_vm* h, double dt, int nsteps);
int cfdj_vm_sync(cfdj_vm* h);
/* One vm_rhs (Common.jl:132-182) on a ghosted host array w: writes r[2:nx+1,2:ny+1]
 * (ldr >= nx+2) and the whole ghosted s (lds >= nx+2, ghost order Common.jl:138-146).
 * Single-GPU and virtual-slab handles (not RCCL ranks). */
int cfdj_vm_rhs(cfdj_vm* h, const double* w, long ldw, double* r, long ldr, double* s,
                long lds);
/* Per-kernel-category device time (HIP events on the handle's stream).  enable != 0
 * starts recording (and clears the counters); ms[CFDJ_K_COUNT] / launches[CFDJ_K_COUNT]
 * receive the accumulated totals (either may be NULL). */
int cfdj_vm_set_timing(cfdj_vm* h, int enable);
int cfdj_vm_timing(cfdj_vm* h, double* ms, long* launches);
/* The CFDJ_K_STAGE time split by RK3 stage (vm.jl:28 / 43-47 / 62-66): ms3[3], launches3[3]
 * for stages 1..3, accumulated over the same recording as cfdj_vm_timing. */
int cfdj_vm_stage_timing(cfdj_vm* h, double* ms3, long* launches3);
/* Kernel microbenchmark (no reference equivalent; bench.py's roofline): `launches`
 * back-to-back launches of one kernel of the step between two HIP events on the handle's
 * stream; *ms_per_launch = elapsed / launches.  Single-GPU handles on the fused Poisson
 * path.  Overwrites the stage and spectrum buffers and (stage 3) advances the vorticity:
 * call it after the runs whose results matter. */
#define CFDJ_KB_STAGE1 1   /* vm_stage_kernel<1>: wn -> w1 (vm.jl:28) */
#define CFDJ_KB_STAGE2 2   /* vm_stage_kernel<2>: (w1, wn) -> w2 (vm.jl:43-47) */
#define CFDJ_KB_STAGE3 3   /* vm_stage_kernel<3>: (w2, wn) -> wn (vm.jl:62-66) */
#define CFDJ_KB_ROWS_FWD 4 /* fused Poisson pass 1: row r2c FFT */
#define CFDJ_KB_COLS 5     /* fused Poisson pass 2: column FFT + divide + inverse FFT */
#define CFDJ_KB_ROWS_INV 6 /* fused Poisson pass 3: row c2r FFT */
int cfdj_vm_kernel_bench(cfdj_vm* h, int kernel, double dt, int launches,
                         double* ms_per_launch);
/* Optional finiteness check of the vorticity after each cfdj_vm_step call. */
int cfdj_vm_set_check_finite(cfdj_vm* h, int enable);
/* Device pointer of this rank's nx-by-(ny/nranks) vorticity slab (pitch nx). */
int cfdj_vm_field_device(cfdj_vm* h, double** w_dev);
/* Shape of this rank's slab: global row offset and row count. */
int cfdj_vm_slab(cfdj_vm* h, int* row0, int* rows);
/* Tuning: select the marching stage kernel (one wavefront walks `rows` rows of a
 * 128-column strip).  Without this call the row-group stage kernel runs wherever it applies
 * (nx a multiple of 512, even row count, no column partial sums) and the marching kernel,
 * with a rows-per-wavefront default chosen per size, elsewhere.  Results are bit-identical. */
int cfdj_vm_set_rows_per_wave(cfdj_vm* h, int rows);
/* The stage kernel a step of this handle launches: 1 = row-group kernel, 0 = marching. */
int cfdj_vm_stage_kernel(cfdj_vm* h, int* row_group);
/* Replay cfdj_vm_step's kernel sequence from a captured HIP graph (default on; used on
 * single-GPU handles with the fused Poisson path, others launch eagerly). */
int cfdj_vm_set_graph(cfdj_vm* h, int enable);
/* Select / query the Poisson implementation (CFDJ_POISSON_*; single-GPU and slab handles). */
int cfdj_vm_set_poisson(cfdj_vm* h, int path);
int cfdj_vm_get_poisson(cfdj_vm* h);
void cfdj_vm_destroy(cfdj_vm* h);

/* ---- lid-driven cavity: 18_NS2D_Lid_Driven_Cavity/lid_driven_cavity.jl ---------------
 * (nx+1)-by-(ny+1) node arrays wn, sn (column-major, ld >= nx+1) on the unit box with
 * dx = 1/nx, dy = 1/ny.  One step = the RK3 loop body of lid_driven_cavity.jl:75-114:
 * three (rhs, stage update, bc2 Jensen wall vorticity, fps_sine DST-I Poisson) rounds and
 * the RMS of the streamfunction change. */
typedef struct cfdj_cavity cfdj_cavity;
#define CFDJ_CAVITY_DST 0 /* fps_sine (lid_driven_cavity.jl:11-21), the reference's solver */
#define CFDJ_CAVITY_MG 1  /* V-cycle multigrid (mg_N.jl), red-black GS, warm-started */
int cfdj_cavity_create(int nx, int ny, double dx, double dy, double re, int device,
                       cfdj_cavity** out);
/* Poisson solver for the streamfunction; n_level/v1/v2/v3/tol/max_iter as mg_N.jl:7
 * (ignored for CFDJ_CAVITY_DST). */
int cfdj_cavity_set_poisson(cfdj_cavity* h, int solver, int n_level, int v1, int v2, int v3,
                            double tol, int max_iter);
int cfdj_cavity_upload(cfdj_cavity* h, const double* wn, long ldw, const double* sn, long lds);
int cfdj_cavity_download(cfdj_cavity* h, double* wn, long ldw, double* sn, long lds);
/* nsteps RK3 steps; rms[k] (may be NULL) = lid_driven_cavity.jl:112-114 of step k. */
int cfdj_cavity_step(cfdj_cavity* h, double dt, int nsteps, double* rms);
/* lid_driven_cavity.jl:124-159 `rhs`: r interior from w, s (r boundary left 0).  A function
 * of its arguments: the handle's vorticity and streamfunction are not touched (only stage
 * scratch is), so it may be called between cfdj_cavity_upload and cfdj_cavity_step. */
int cfdj_cavity_rhs(cfdj_cavity* h, const double* w, long ldw, const double* s, long lds,
                    double* r, long ldr);
/* Total V-cycles run by the multigrid Poisson solves so far. */
long cfdj_cavity_mg_iterations(cfdj_cavity* h);
void cfdj_cavity_destroy(cfdj_cavity* h);
/* lid_driven_cavity.jl:11-21 `fps_sine`: s[2:nx,2:ny] solving the 5-point Dirichlet
 * Poisson problem with right-hand side f[2:nx,2:ny] (one-shot). */
int cfdj_fps_sine(int nx, int ny, double dx, double dy, const double* f, long ldf, double* s,
                  long lds);

/* ---- multigrid: 17_Poisson_Solver_Multigrid/mg_N.jl:7-114 -------------------------------
 * n_level-level V-cycle on the (nx+1)x(ny+1) Dirichlet problem lap(u) = f; u carries the
 * boundary values in and the solution out.  Smoother: red-black ordering of the
 * Common.jl:78-92 Gauss-Seidel update (the reference sweeps lexicographically; converged
 * solutions agree to the tolerance).  rms_hist (may be NULL) receives iterations+1
 * residual norms (Common.jl:229-232), the first being the initial residual.
 * The two-level solver of 17_Poisson_Solver_Multigrid/mg.jl:7-85 is n_level = 2 with the
 * roles of v2 and v3 exchanged: mg.jl relaxes the coarse grid v3 times (mg.jl:66) and the
 * corrected fine grid v2 times (mg.jl:77), mg_N.jl the other way round (mg_N.jl:91,103);
 * pass (v1, v3, v2) for mg.jl's (v1, v2, v3). */
typedef struct cfdj_mg cfdj_mg;
int cfdj_mg_create(int nx, int ny, double dx, double dy, int n_level, int v1, int v2, int v3,
                   int device, cfdj_mg** out);
int cfdj_mg_solve(cfdj_mg* h, const double* f, long ldf, double* u, long ldu, double tol,
                  int max_iter, int* iterations, double* rms_hist);
/* The fine-grid residual r = f - lap(u) of the last cfdj_mg_solve's final convergence
 * check (mg_N.jl:59 / mg.jl:47 leave it in the caller's `r`; boundary entries are 0):
 * (nx+1) x (ny+1), ldr >= nx+1. */
int cfdj_mg_residual(cfdj_mg* h, double* r, long ldr);
void cfdj_mg_destroy(cfdj_mg* h);

/* ---- 15_Poisson_Solver_Gauss_Seidel/gauss_seidel.jl:8-54 ----------------------------------
 * The reference's "Gauss-Seidel" is a Jacobi sweep (residual of the old iterate everywhere,
 * then u += r / (-2/dx^2 - 2/dy^2)); up to 5*max_iter sweeps, convergence checked every
 * freq sweeps against tol * the initial residual norm.  u in/out (boundary = data). */
int cfdj_jacobi_solve(int nx, int ny, double dx, double dy, const double* f, long ldf,
                      double* u, long ldu, long max_iter, double tol, long freq,
                      long* iterations, double* rms);

/* ---- spectral NS2D: 20_NS2D_Hybrid_Solver/hybrid.jl, 21/22 pseudospectral -------------
 * The vorticity spectrum w_f (complex nx x ny, as the reference's Array{ComplexF64}) is
 * advanced by the low-storage RK3 / Crank-Nicolson loop of hybrid.jl:41-67 (identical in
 * pseudospectral_32_rule.jl and pseudospectral_23_rule.jl); `kind` selects `jacobian`:
 * hybrid.jl:92-152 (Arakawa in physical space), pseudospectral_23_rule.jl:95-144 (2/3-rule
 * truncation) or pseudospectral_32_rule.jl:94-186 (3/2-rule padding).  Square even grids
 * (the reference aliases ky = kx, Common.jl:198). */
typedef struct cfdj_spec cfdj_spec;
#define CFDJ_SPEC_HYBRID 0
#define CFDJ_SPEC_PS23 1
#define CFDJ_SPEC_PS32 2
int cfdj_spec_create(int nx, int ny, double dx, double dy, double re, double eps, int kind,
                     int device, cfdj_spec** out);
/* hybrid.jl:24-28: w_f = fft(wn[2:nx+1, 2:ny+1]), w_f[1,1] = 0 (wn ghosted, ld >= nx+2). */
int cfdj_spec_upload(cfdj_spec* h, const double* wn, long ldw);
/* nsteps iterations of hybrid.jl:41-67. */
int cfdj_spec_step(cfdj_spec* h, double dt, int nsteps);
/* hybrid.jl:71-76: ut = real(ifft(w_f)) on (nx+1) x (ny+1) nodes (ld >= nx+1). */
int cfdj_spec_download(cfdj_spec* h, double* ut, long ldu);
/* w_f itself, complex nx x ny column-major as interleaved (re, im) doubles.  w_f is the
 * spectrum of a real field (the only kind the reference's loop produces).  The hybrid solver's
 * set_spectrum and jacobian keep the Hermitian part (w_f(k) + conj(w_f(-k))) / 2 of their
 * input -- all that hybrid.jl's jacobian() sees of it through real(ifft(.)), so
 * cfdj_spec_jacobian matches it for any input.  The pseudospectral rules require the spectrum
 * of a real field: where the solver keeps half of it (square power-of-two grids of
 * 1024..8192, 2/3 rule) they read the modes kx index 0..nx/2 and take the others to be their
 * conjugate mirror.  get_spectrum returns the state with its conjugate mirror. */
int cfdj_spec_get_spectrum(cfdj_spec* h, double* wf);
int cfdj_spec_set_spectrum(cfdj_spec* h, const double* wf);
/* One `jacobian(nx, ny, dx, dy, wf, k2)` call: jf = fft(-J(w, psi)) (complex, as above). */
int cfdj_spec_jacobian(cfdj_spec* h, const double* wf, double* jf);
void cfdj_spec_destroy(cfdj_spec* h);

/* ---- 01_Heat_Equation_FTCS/ftcs.jl:34-41 (host code: BASELINE config 1 is CPU-only) -------
 * un is (nx+1) x (nt+1) column-major (ld >= nx+1): column 0 is u0, column k the FTCS step
 * u_i <- u_i + beta (u_{i+1} - 2 u_i + u_{i-1}) with u_0 = u_nx = 0. */
int cfdj_ftcs(int nx, int nt, double beta, const double* u0, double* un, long ldu);

#ifdef __cplusplus
}
#endif
#endif /* CFDJ_H_ */
