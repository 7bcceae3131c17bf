# CFDJ.jl -- thin ccall shim over libcfdj.so (include/cfdj.h) so the reference's scripts
# can swap their hot path for the MI355X implementation:
#
#   include("../julia/CFDJ.jl"); using .CFDJ
#   vm.jl:139        un = CFDJ.numerical(nx, ny, nt, Δx, Δy, Δt, re, x, y, wn, ns)
#   Common.jl:136    CFDJ.fps(nx, ny, Δx, Δy, u, e, data, data1, f, s)
#   vm.jl:26         CFDJ.vm_rhs(nx, ny, Δx, Δy, re, w, u, e, data, data1, r, s, f)
#   lid_driven_cavity.jl:197  CFDJ.cavity_numerical(nx, ny, nt, Δx, Δy, Δt, re, wn, sn, rms)
#   lid_driven_cavity.jl:84   CFDJ.fps_sine(nx, ny, Δx, Δy, f, u, e, data, data1, iden, sn)
#   lid_driven_cavity.jl:78   CFDJ.cavity_rhs(nx, ny, Δx, Δy, re, w, s, r)
#   fft_d.jl:73      un[2:nx, 2:ny] = CFDJ.ps_fst(nx, ny, Δx, Δy, f)
#   mg_N.jl:180      CFDJ.mg_N(Δx, Δy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out, n_level)
#   mg.jl:146        CFDJ.mg(Δx, Δy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out)
#
# Same positional arguments and in-place semantics as the Julia originals; FFT scratch
# arguments are accepted and ignored (the GPU handle owns its buffers).  Errors from the
# library are raised as ErrorException (argument errors as BoundsError, like the reference).
# Device handles are cached per parameter set (a vm.jl run calls vm_rhs 3 x 2000 times):
# Julia's GC does not see device memory, so handles are never left to finalizers alone;
# `CFDJ.release!()` destroys every cached handle.
# Untested in CI: the build image has no `julia`.
module CFDJ

const libcfdj = get(ENV, "CFDJ_LIB", joinpath(@__DIR__, "..", "cfd_julia_amd", "libcfdj.so"))

function check(rc::Cint, where::String)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:cfdj_last_error, libcfdj), Cstring, ()))
    rc == -1 && throw(BoundsError("$where: $msg"))
    error("$where failed ($rc): $msg")
end

mutable struct VM
    h::Ptr{Cvoid}
    nx::Int
    ny::Int
end

function VM(nx, ny, Δx, Δy, re; ε=1e-6, device=-1)
    out = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:cfdj_vm_create, libcfdj), Cint,
                (Cint, Cint, Cdouble, Cdouble, Cdouble, Cdouble, Cint, Ref{Ptr{Cvoid}}),
                nx, ny, Δx, Δy, re, ε, device, out), "cfdj_vm_create")
    vm = VM(out[], nx, ny)
    finalizer(destroy!, vm)
    return vm
end

function destroy!(vm::VM)
    vm.h == C_NULL && return nothing
    ccall((:cfdj_vm_destroy, libcfdj), Cvoid, (Ptr{Cvoid},), vm.h)
    vm.h = C_NULL
    return nothing
end

# One handle per (nx, ny, Δx, Δy, re, ε, device): device buffers, FFT tables and the HIP
# stream are created once and reused by every vm_rhs / numerical call with those parameters.
const VM_CACHE = Dict{Tuple, VM}()

function cached_vm(nx, ny, Δx, Δy, re; ε=1e-6, device=-1)
    key = (Int(nx), Int(ny), Float64(Δx), Float64(Δy), Float64(re), Float64(ε), Int(device))
    get!(() -> VM(nx, ny, Δx, Δy, re; ε=ε, device=device), VM_CACHE, key)
end

upload!(vm::VM, w::Matrix{Float64}) =
    check(ccall((:cfdj_vm_upload, libcfdj), Cint, (Ptr{Cvoid}, Ptr{Cdouble}, Clong),
                vm.h, w, size(w, 1)), "cfdj_vm_upload")
download!(vm::VM, w::Matrix{Float64}) =
    check(ccall((:cfdj_vm_download, libcfdj), Cint, (Ptr{Cvoid}, Ptr{Cdouble}, Clong),
                vm.h, w, size(w, 1)), "cfdj_vm_download")
step!(vm::VM, Δt, n) =
    check(ccall((:cfdj_vm_step, libcfdj), Cint, (Ptr{Cvoid}, Cdouble, Cint), vm.h, Δt, n),
          "cfdj_vm_step")

"vm.jl:12-90 on the GPU; snapshots every nt÷ns steps as in the reference."
function numerical(nx, ny, nt, Δx, Δy, Δt, re, x, y, wn, ns)
    vm = cached_vm(nx, ny, Δx, Δy, re)
    upload!(vm, wn)
    freq = nt ÷ ns
    m = 1
    k = 0
    while k < nt
        chunk = min(freq - mod(k, freq), nt - k)
        step!(vm, Δt, chunk)
        k += chunk
        if mod(k, freq) == 0
            @show k
            download!(vm, wn)
            ut = wn[2:nx+2, 2:ny+2]
            open("vm$m.txt", "w") do io
                for j ∈ 1:ny + 1, i ∈ 1:nx + 1
                    write(io, "$(x[i]) $(y[j]) $(ut[i, j])\n")
                end
            end
        end
    end
    download!(vm, wn)
    return wn[2:nx+2, 2:ny+2]
end

"Common.jl:132-182: r (interior) and s (with ghosts) from w."
function vm_rhs(nx, ny, Δx, Δy, re, w, u, e, data, data1, r, s, f)
    vm = cached_vm(nx, ny, Δx, Δy, re)
    check(ccall((:cfdj_vm_rhs, libcfdj), Cint,
                (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                vm.h, w, size(w, 1), r, size(r, 1), s, size(s, 1)), "cfdj_vm_rhs")
    f[1:nx, 1:ny] .= .-w[2:nx+1, 2:ny+1]
    return nothing
end

# Poisson plans (cfdj_fps_plan), cached like the VM handles.
const FPS_CACHE = Dict{Tuple, Ptr{Cvoid}}()

function cached_fps(nx, ny, Δx, Δy, ε; device=-1)
    key = (Int(nx), Int(ny), Float64(Δx), Float64(Δy), Float64(ε), Int(device))
    get!(FPS_CACHE, key) do
        out = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:cfdj_fps_create, libcfdj), Cint,
                    (Cint, Cint, Cdouble, Cdouble, Cdouble, Cint, Ref{Ptr{Cvoid}}),
                    nx, ny, Δx, Δy, ε, device, out), "cfdj_fps_create")
        out[]
    end
end

"Common.jl:97-125: s[2:nx+1, 2:ny+1] = FD-FFT Poisson solution of ∇²s = f."
function fps(nx, ny, Δx, Δy, u, e, data, data1, f, s, ε=1e-6)
    h = cached_fps(nx, ny, Δx, Δy, ε)
    check(ccall((:cfdj_fps_solve, libcfdj), Cint,
                (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                h, f, size(f, 1), pointer(s, 2 + size(s, 1)), size(s, 1)), "cfdj_fps_solve")
    return nothing
end

# ---- 18_NS2D_Lid_Driven_Cavity/lid_driven_cavity.jl --------------------------------------
const CAVITY_CACHE = Dict{Tuple, Ptr{Cvoid}}()

"Cavity handle for (nx, ny, Δx, Δy, re); poisson = :dst (fps_sine) or :mg (V-cycle, mg_N.jl)."
function cached_cavity(nx, ny, Δx, Δy, re; device=-1, poisson=:dst, n_level=0, v1=2, v2=2,
                       v3=2, tol=1e-9, max_iter=100_000)
    key = (Int(nx), Int(ny), Float64(Δx), Float64(Δy), Float64(re), Int(device), poisson,
           Int(n_level), Int(v1), Int(v2), Int(v3), Float64(tol), Int(max_iter))
    get!(CAVITY_CACHE, key) do
        out = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:cfdj_cavity_create, libcfdj), Cint,
                    (Cint, Cint, Cdouble, Cdouble, Cdouble, Cint, Ref{Ptr{Cvoid}}),
                    nx, ny, Δx, Δy, re, device, out), "cfdj_cavity_create")
        if poisson == :mg
            nl = n_level > 0 ? n_level : Int(floor(log2(min(nx, ny))))
            check(ccall((:cfdj_cavity_set_poisson, libcfdj), Cint,
                        (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Cint, Cdouble, Cint),
                        out[], 1, nl, v1, v2, v3, tol, max_iter), "cfdj_cavity_set_poisson")
        end
        out[]
    end
end

"lid_driven_cavity.jl:58-118: advances wn, sn in place for nt steps and fills rms[1:nt]."
function cavity_numerical(nx, ny, nt, Δx, Δy, Δt, re, wn, sn, rms; kw...)
    length(rms) >= nt || throw(BoundsError(rms, nt))
    h = cached_cavity(nx, ny, Δx, Δy, re; kw...)
    check(ccall((:cfdj_cavity_upload, libcfdj), Cint,
                (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                h, wn, size(wn, 1), sn, size(sn, 1)), "cfdj_cavity_upload")
    # in chunks of 100 steps, printing like lid_driven_cavity.jl:116
    k = 0
    while k < nt
        chunk = min(100 - mod(k, 100), nt - k)
        check(ccall((:cfdj_cavity_step, libcfdj), Cint, (Ptr{Cvoid}, Cdouble, Cint, Ptr{Cdouble}),
                    h, Δt, chunk, pointer(rms, k + 1)), "cfdj_cavity_step")
        k += chunk
        if mod(k, 100) == 0 println(k, " ", rms[k]) end
    end
    check(ccall((:cfdj_cavity_download, libcfdj), Cint,
                (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                h, wn, size(wn, 1), sn, size(sn, 1)), "cfdj_cavity_download")
    return nothing
end

"lid_driven_cavity.jl:124-159: r[2:nx, 2:ny] from w and s."
function cavity_rhs(nx, ny, Δx, Δy, re, w, s, r)
    h = cached_cavity(nx, ny, Δx, Δy, re)
    check(ccall((:cfdj_cavity_rhs, libcfdj), Cint,
                (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                h, w, size(w, 1), s, size(s, 1), r, size(r, 1)), "cfdj_cavity_rhs")
    return nothing
end

"lid_driven_cavity.jl:11-21: sn[2:nx, 2:ny] from f[2:nx, 2:ny] (u, e, data, data1, iden ignored)."
function fps_sine(nx, ny, Δx, Δy, f, u, e, data, data1, iden, sn)
    check(ccall((:cfdj_fps_sine, libcfdj), Cint,
                (Cint, Cint, Cdouble, Cdouble, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                nx, ny, Δx, Δy, f, size(f, 1), sn, size(sn, 1)), "cfdj_fps_sine")
    return nothing
end

"14_Poisson_Solver_FST/fft_d.jl:7-23: the (nx-1) x (ny-1) interior solution for f[2:nx, 2:ny]."
function ps_fst(nx, ny, Δx, Δy, f)
    sn = zeros(Float64, nx + 1, ny + 1)
    check(ccall((:cfdj_fps_sine, libcfdj), Cint,
                (Cint, Cint, Cdouble, Cdouble, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                nx, ny, Δx, Δy, f, size(f, 1), sn, size(sn, 1)), "cfdj_fps_sine")
    return sn[2:nx, 2:ny]
end

# ---- 17_Poisson_Solver_Multigrid/mg_N.jl and mg.jl ------------------------------------------
# One V-cycle solve on the GPU (red-black ordering of the Common.jl:78-92 update); fills u_n
# and r (the final fine residual) in place and writes the reference's residual history and
# the three `out` lines.
function mg_run(Δx, Δy, nx, ny, r, f, u_n, sweeps, max_iter, tol, out, n_level, freq, resfile)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:cfdj_mg_create, libcfdj), Cint,
                (Cint, Cint, Cdouble, Cdouble, Cint, Cint, Cint, Cint, Cint, Ref{Ptr{Cvoid}}),
                nx, ny, Δx, Δy, n_level, sweeps[1], sweeps[2], sweeps[3], -1, h),
          "cfdj_mg_create")
    it = Ref{Cint}(0)
    hist = zeros(Float64, max_iter + 1)
    try
        check(ccall((:cfdj_mg_solve, libcfdj), Cint,
                    (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong, Cdouble, Cint,
                     Ref{Cint}, Ptr{Cdouble}),
                    h[], f, size(f, 1), u_n, size(u_n, 1), tol, max_iter, it, hist),
              "cfdj_mg_solve")
        check(ccall((:cfdj_mg_residual, libcfdj), Cint, (Ptr{Cvoid}, Ptr{Cdouble}, Clong),
                    h[], r, size(r, 1)), "cfdj_mg_residual")
    finally
        ccall((:cfdj_mg_destroy, libcfdj), Cvoid, (Ptr{Cvoid},), h[])
    end
    init_rms = hist[1]
    println("0 $init_rms $(init_rms / init_rms)")
    open(resfile, "w") do res
        for k ∈ 1:it[]
            if mod(k, freq) == 0
                rms = hist[k+1]
                write(res, "$k $rms $(rms / init_rms)\n")
                println("$k $rms $(rms / init_rms)")
            end
        end
    end
    write(out, "L-2 Norm=$(hist[it[]+1])\n")
    write(out, "Maximum Norm=$(maximum(abs.(r)))\n")
    write(out, "Iterations=$(it[])\n")
    return
end

"mg_N.jl:7-114 (n-level V-cycle)."
mg_N(Δx, Δy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out, n_level, freq=1) =
    mg_run(Δx, Δy, nx, ny, r, f, u_n, (v1, v2, v3), max_iter, tol, out, n_level, freq,
           "mg_residual.txt")

"mg.jl:7-85 (two levels): the coarse grid is relaxed v3 times (mg.jl:66) and the corrected
fine grid v2 times (mg.jl:77) -- the reverse of mg_N.jl:91,103, hence (v1, v3, v2)."
mg(Δx, Δy, nx, ny, r, f, u_n, v1, v2, v3, max_iter, tol, out, freq=100) =
    mg_run(Δx, Δy, nx, ny, r, f, u_n, (v1, v3, v2), max_iter, tol, out, 2, freq, "residual.txt")

"Destroy every cached device handle (VM, Poisson plans, cavities)."
function release!()
    for vm in values(VM_CACHE) destroy!(vm) end
    empty!(VM_CACHE)
    for h in values(FPS_CACHE) ccall((:cfdj_fps_destroy, libcfdj), Cvoid, (Ptr{Cvoid},), h) end
    empty!(FPS_CACHE)
    for h in values(CAVITY_CACHE) ccall((:cfdj_cavity_destroy, libcfdj), Cvoid, (Ptr{Cvoid},), h) end
    empty!(CAVITY_CACHE)
    return nothing
end

"hybrid.jl:14-86 / pseudospectral_*.jl:13-89 on the GPU; kind = 0 hybrid, 1 2/3 rule, 2 3/2 rule."
function spectral_numerical(nx, ny, nt, Δx, Δy, Δt, re, x, y, wn, ns; kind=0, ε=1e-6, device=-1)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:cfdj_spec_create, libcfdj), Cint,
                (Cint, Cint, Cdouble, Cdouble, Cdouble, Cdouble, Cint, Cint, Ptr{Ptr{Cvoid}}),
                nx, ny, Δx, Δy, re, ε, kind, device, h), "cfdj_spec_create")
    ut = Array{Float64}(undef, nx + 1, ny + 1)
    try
        check(ccall((:cfdj_spec_upload, libcfdj), Cint, (Ptr{Cvoid}, Ptr{Cdouble}, Clong),
                    h[], wn, size(wn, 1)), "cfdj_spec_upload")
        freq = nt ÷ ns
        m = 1
        for k ∈ 1:nt
            check(ccall((:cfdj_spec_step, libcfdj), Cint, (Ptr{Cvoid}, Cdouble, Cint),
                        h[], Δt, 1), "cfdj_spec_step")
            if mod(k, freq) == 0
                @show k
                check(ccall((:cfdj_spec_download, libcfdj), Cint,
                            (Ptr{Cvoid}, Ptr{Cdouble}, Clong), h[], ut, size(ut, 1)),
                      "cfdj_spec_download")
                open("vm$m.txt", "w") do io
                    for j ∈ 1:ny + 1, i ∈ 1:nx + 1
                        write(io, "$(x[i]) $(y[j]) $(ut[i, j])\n")
                    end
                end
                m += 1
            end
        end
        check(ccall((:cfdj_spec_download, libcfdj), Cint, (Ptr{Cvoid}, Ptr{Cdouble}, Clong),
                    h[], ut, size(ut, 1)), "cfdj_spec_download")
    finally
        ccall((:cfdj_spec_destroy, libcfdj), Cvoid, (Ptr{Cvoid},), h[])
    end
    return ut
end

end # module
