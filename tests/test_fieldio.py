"""Text field formats: vm.jl:81-85 / 130-146 and
lid_driven_cavity.jl:201-214, read back as 19/plotting.jl:14-31 does (readdlm + reshape).

Julia number formatting pinned by known answers of Base.show for Float64 (plain for
1e-4 <= |v| < 1e6, else "d.de±x"); the round trip is exact because both print the shortest
round-trip decimal.
"""
import numpy as np
import pytest

from cfd_julia_amd.fieldio import julia_str, read_field, write_field, write_res_plot


@pytest.mark.parametrize("v,s", [
    (0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (0.5, "0.5"), (-2.5, "-2.5"),
    (1e-4, "0.0001"), (0.0001234, "0.0001234"), (1e-5, "1.0e-5"), (3e-5, "3.0e-5"),
    (-1.5e-300, "-1.5e-300"), (100000.0, "100000.0"), (999999.0, "999999.0"),
    (1e6, "1.0e6"), (1234567.0, "1.234567e6"), (2.0 ** 30, "1.073741824e9"),
    (1e16, "1.0e16"), (6.283185307179586, "6.283185307179586"),
    (0.04908738521234052, "0.04908738521234052"), (float("nan"), "NaN"),
    (float("inf"), "Inf"), (float("-inf"), "-Inf"), (5e-324, "5.0e-324"),
    (1.7976931348623157e308, "1.7976931348623157e308"),
])
def test_julia_float_text(v, s):
    assert julia_str(v) == s


def test_julia_float_round_trip():
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.standard_normal(2000) * 10.0 ** rng.integers(-12, 12, 2000),
                        rng.standard_normal(200)])
    for a in v.tolist():
        assert float(julia_str(a)) == a


def test_field_order_and_read_back(tmp_path):
    nx, ny = 6, 4
    x = np.arange(nx + 1) * 0.25
    y = np.arange(ny + 1) * 0.5
    rng = np.random.default_rng(1)
    w = np.asfortranarray(rng.standard_normal((nx + 1, ny + 1)))
    s = np.asfortranarray(rng.standard_normal((nx + 1, ny + 1)))
    write_field(tmp_path / "f.txt", x, y, w, s)
    lines = (tmp_path / "f.txt").read_text().splitlines()
    assert len(lines) == (nx + 1) * (ny + 1)
    # j outer, i inner: line 1 is (i=2, j=1), line nx+1 is (i=1, j=2)
    assert lines[1].split() == [julia_str(x[1]), julia_str(y[0]), julia_str(w[1, 0]),
                                julia_str(s[1, 0])]
    assert lines[nx + 1].split()[:2] == [julia_str(x[0]), julia_str(y[1])]
    assert np.array_equal(read_field(tmp_path / "f.txt", nx, ny, 2), w)
    assert np.array_equal(read_field(tmp_path / "f.txt", nx, ny, 3), s)


def test_res_plot(tmp_path):
    rms = np.array([0.1, 1e-7, 2.5e-12])
    write_res_plot(tmp_path / "r.txt", rms)
    assert (tmp_path / "r.txt").read_text() == "1 0.1\n2 1.0e-7\n3 2.5e-12\n"
