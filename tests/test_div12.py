"""The assembly's divide-free x / 12 (csrc/mof_assemble.hip div12: the f term
"... * T_area / 12" of compute_f, compute_optical_flow.py:311) restated in C
with the same IEEE operations and checked against the true quotient on the
host: random bit patterns over every exponent (normal and subnormal
quotients), random values in the f terms' range, and the structured
significands next to rounding midpoints. The GPU parity tests check the
device build bit for bit through f (tests/test_gpu_parity.py)."""
import ctypes
import subprocess

C_SRC = r"""
#include <math.h>
#include <stdint.h>
#include <string.h>
static double div12(double x) {
    const double c = 1.0 / 12.0;
    const double q0 = x * c;
    if (!(fabs(q0) >= 0x1p-1020)) return x / 12.0;
    const double q = fma(fma(-q0, 12.0, x), c, q0);
    return isfinite(q0) ? q : q0;
}
static uint64_t next(uint64_t *s) {  /* splitmix64 */
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static int same(double a, double b) { return memcmp(&a, &b, 8) == 0 || (isnan(a) && isnan(b)); }
/* mode 0: random bit patterns; 1: |x| in [1e-12, 1e3]; 2: significands
   m = 3k + {0,1,2} near the top and bottom of the binade, every exponent */
int64_t check(int mode, int64_t n, uint64_t seed) {
    int64_t bad = 0;
    uint64_t s = seed;
    for (int64_t i = 0; i < n; ++i) {
        double x;
        uint64_t r = next(&s);
        if (mode == 0) {
            memcpy(&x, &r, 8);
        } else if (mode == 1) {
            x = ldexp((double)(r >> 11), -53) * pow(10.0, -12.0 + 15.0 * (double)(next(&s) >> 11) / 9007199254740992.0);
            if (r & 1) x = -x;
        } else {
            uint64_t m = (r & 1) ? (1ull << 52) + (next(&s) % 64) : (1ull << 53) - 1 - (next(&s) % 64);
            int e = (int)(next(&s) % 2098) - 1126;
            x = ldexp((double)m, e);
        }
        if (!same(div12(x), x / 12.0)) ++bad;
    }
    return bad;
}
"""


def _lib(tmp_path):
    src = tmp_path / "div12.c"
    so = tmp_path / "div12.so"
    src.write_text(C_SRC)
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                           "-o", str(so), str(src), "-lm"])
    lib = ctypes.CDLL(str(so))
    lib.check.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_uint64]
    lib.check.restype = ctypes.c_int64
    return lib


def test_div12_equals_ieee_quotient(tmp_path):
    lib = _lib(tmp_path)
    for mode, n in ((0, 20_000_000), (1, 20_000_000), (2, 20_000_000)):
        assert lib.check(mode, n, 12345 + mode) == 0, mode


def test_div12_without_fallback_fails_only_below_normal(tmp_path):
    """The small-quotient fallback is needed (and only there): without it the
    sequence misrounds some subnormal quotients."""
    src = C_SRC.replace("if (!(fabs(q0) >= 0x1p-1020)) return x / 12.0;", "")
    (tmp_path / "nofb").mkdir()
    import pathlib
    d = pathlib.Path(tmp_path / "nofb")
    (d / "div12.c").write_text(src)
    so = d / "div12.so"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                           "-o", str(so), str(d / "div12.c"), "-lm"])
    lib = ctypes.CDLL(str(so))
    lib.check.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_uint64]
    lib.check.restype = ctypes.c_int64
    assert lib.check(0, 20_000_000, 12345) > 0  # random bit patterns reach subnormal quotients
    assert lib.check(1, 5_000_000, 7) == 0  # the f terms' range never needs it
