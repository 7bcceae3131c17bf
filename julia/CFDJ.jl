# CFDJ.jl -- thin ccall shim over libcfdj.so (include/cfdj.h) so the reference's scripts
# can swap their hot path for the MI355X implementation:
#
#   include("../julia/CFDJ.jl"); using .CFDJ
#   vm.jl:139        un = CFDJ.numerical(nx, ny, nt, Δx, Δy, Δt, re, x, y, wn, ns)
#   Common.jl:136    CFDJ.fps(nx, ny, Δx, Δy, u, e, data, data1, f, s)
#   vm.jl:26         CFDJ.vm_rhs(nx, ny, Δx, Δy, re, w, u, e, data, data1, r, s, f)
#
# Same positional arguments and in-place semantics as the Julia originals; FFT scratch
# arguments are accepted and ignored (the GPU handle owns its buffers).  Errors from the
# library are raised as ErrorException (argument errors as BoundsError, like the reference).
# Untested in CI: this image has no `julia` (SURVEY.md §0.3).
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
    finalizer(v -> ccall((:cfdj_vm_destroy, libcfdj), Cvoid, (Ptr{Cvoid},), v.h), vm)
    return vm
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
    vm = VM(nx, ny, Δx, Δy, re)
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
    vm = VM(nx, ny, Δx, Δy, re)
    check(ccall((:cfdj_vm_rhs, libcfdj), Cint,
                (Ptr{Cvoid}, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                vm.h, w, size(w, 1), r, size(r, 1), s, size(s, 1)), "cfdj_vm_rhs")
    f[1:nx, 1:ny] .= .-w[2:nx+1, 2:ny+1]
    return nothing
end

"Common.jl:97-125: s[2:nx+1, 2:ny+1] = FD-FFT Poisson solution of ∇²s = f."
function fps(nx, ny, Δx, Δy, u, e, data, data1, f, s, ε=1e-6)
    check(ccall((:cfdj_fps, libcfdj), Cint,
                (Cint, Cint, Cdouble, Cdouble, Cdouble, Ptr{Cdouble}, Clong, Ptr{Cdouble}, Clong),
                nx, ny, Δx, Δy, ε, f, size(f, 1), pointer(s, 2 + size(s, 1)), size(s, 1)),
          "cfdj_fps")
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
