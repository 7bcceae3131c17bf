"""Text field formats of the reference, written the way Julia's string interpolation
prints a Float64, so the reference's plotting scripts (`readdlm`) read our output unchanged.

    vm.jl:81-85, 130-146          "x y ω" per node, j outer / i inner, (nx+1)(ny+1) lines
                                  (vm$m.txt, vm0.txt, field_final.txt)
    lid_driven_cavity.jl:201-214  "n rms" per step (res_plot.txt) and "x y ω ψ" per node
                                  (field_final.txt)
    19/plotting.jl:14-31          reader: readdlm, column 3 reshaped to (nx+1, ny+1)

Julia prints the shortest round-trip decimal (as Python's repr), but in its own layout:
plain notation for 1e-4 <= |v| < 1e6 ("0.0001", "100000.0"), otherwise "d.ddde±x" with at
least one fraction digit and no exponent padding ("1.0e-5", "1.234567e6"), "NaN", "Inf".
"""
from __future__ import annotations

import math

import numpy as np


def julia_str(v: float) -> str:
    """The text of `"$(v)"` for a Float64 v in Julia (Base.show / Ryu shortest)."""
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Inf" if v > 0 else "-Inf"
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    sign = "-" if v < 0 else ""
    # shortest round-trip digits and the decimal exponent, from repr
    r = repr(abs(v))
    if "e" in r:
        m, e = r.split("e")
        digits = m.replace(".", "")
        e10 = int(e) + (m.index(".") if "." in m else len(m)) - 1
    else:
        ip, _, fp = r.partition(".")
        if ip != "0":
            digits = (ip + fp).rstrip("0") or "0"
            e10 = len(ip) - 1
        else:
            nz = len(fp) - len(fp.lstrip("0"))
            digits = fp.lstrip("0")
            e10 = -nz - 1
    digits = digits.lstrip("0").rstrip("0") or "0"
    if -5 < e10 < 6:  # plain notation
        if e10 >= 0:
            ip = digits[:e10 + 1].ljust(e10 + 1, "0")
            fp = digits[e10 + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-e10 - 1) + digits
        return f"{sign}{ip}.{fp}"
    return f"{sign}{digits[0]}.{digits[1:] or '0'}e{e10}"


def _write_rows(path, columns):
    cols = [np.asarray(c, dtype=np.float64).ravel() for c in columns]
    with open(path, "w") as io:
        for row in zip(*(c.tolist() for c in cols)):
            io.write(" ".join(julia_str(a) for a in row) + "\n")


def _node_columns(x, y, *fields):
    """(x[i], y[j], f[i, j]...) with j outer, i inner (Julia `for j for i`)."""
    nxp, nyp = np.shape(fields[0])
    X = np.broadcast_to(np.asarray(x[:nxp], dtype=np.float64)[:, None], (nxp, nyp))
    Y = np.broadcast_to(np.asarray(y[:nyp], dtype=np.float64)[None, :], (nxp, nyp))
    # column-major flattening = i fastest
    return [X.ravel(order="F"), Y.ravel(order="F")] + \
           [np.asarray(f, dtype=np.float64).ravel(order="F") for f in fields]


def write_field(path, x, y, *fields):
    """vm.jl:81-85 ("x y ω") or lid_driven_cavity.jl:208-213 ("x y ω ψ")."""
    _write_rows(path, _node_columns(x, y, *fields))


def write_res_plot(path, rms):
    """lid_driven_cavity.jl:201-206: "n rms[n]" for n = 1..nt (n printed as an integer)."""
    with open(path, "w") as io:
        for n, v in enumerate(np.asarray(rms, dtype=np.float64).tolist(), start=1):
            io.write(f"{n} {julia_str(v)}\n")


def read_field(path, nx, ny, column=2):
    """19/plotting.jl:14-31: readdlm, then column `column` (0-based) reshaped to the
    (nx+1, ny+1) node array (Julia reshape = column-major)."""
    data = np.loadtxt(path, ndmin=2)
    return np.asarray(data[:, column]).reshape((nx + 1, ny + 1), order="F")


__all__ = ["julia_str", "write_field", "write_res_plot", "read_field"]
