"""C-ABI host-side tests (no GPU needed): the library loads, exports every symbol the
header declares, validates like the reference constructor, and computes the host
tables bit-for-bit like the reference (tests/golden)."""
import os
import re

import numpy as np
import pytest

import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    capi.lib()
    return capi


def header_functions():
    txt = open(os.path.join(ROOT, "include", "meyda_gpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mgx_[a-z_0-9]+)\s*\(", txt)))


def test_exports_every_header_symbol(capi):
    funcs = header_functions()
    assert len(funcs) >= 15
    assert sorted(capi.EXPORTS) == funcs
    L = capi.lib()
    for f in funcs:
        assert hasattr(L, f), f


def test_abi_version_and_names(capi):
    L = capi.lib()
    assert L.mgx_abi_version() == 2
    for i, name in enumerate(capi.FEATURE_NAMES):
        assert L.mgx_feature_name(i).decode() == name
        assert L.mgx_feature_index(name.encode()) == i
    assert L.mgx_feature_index(b"nope") == -1
    assert L.mgx_feature_name(99) is None
    # src/feature-info.js types: number=0, array=1, multipleArrays=2
    info = {n: L.mgx_feature_info(i) for i, n in enumerate(capi.FEATURE_NAMES)}
    assert info["rms"] == 0 and info["mfcc"] == 1 and info["loudness"] == 2
    assert info["complexSpectrum"] == 2 and info["amplitudeSpectrum"] == 1 and info["buffer"] == 1


def test_is_power_of_two_matches_reference(capi):
    # src/utils.js:13-19 halves while even; 1 is a power of two, 0 and 6 are not.
    L = capi.lib()
    for n, want in [(1, 1), (2, 1), (512, 1), (0, 0), (6, 0), (1023, 0), (2.5, 0), (-4, 0)]:
        assert L.mgx_is_power_of_two(float(n)) == want, n


def test_not_power_of_two_is_rejected_first(capi):
    with pytest.raises(capi.MgxError) as ei:
        capi.Plan(buffer_size=1000)
    assert ei.value.status == -2
    assert "not a power of two" in str(ei.value)


def test_bad_descriptor(capi):
    import ctypes
    d = capi.make_desc()
    d.struct_size = 3
    h = ctypes.c_void_p()
    assert capi.lib().mgx_plan_create(ctypes.byref(d), ctypes.byref(h)) == -1
    assert b"struct_size" in capi.lib().mgx_last_error()
    d = capi.make_desc()
    d.num_bark_bands = 12
    assert capi.lib().mgx_plan_create(ctypes.byref(d), ctypes.byref(h)) == -3


def test_plan_flags_match_header(capi):
    import ctypes
    txt = open(os.path.join(ROOT, "include", "meyda_gpu.h")).read()
    flags = {k: int(v) for k, v in re.findall(r"#define (MGX_FLAG_[A-Z_]+) (\d+)u", txt)}
    assert flags == {"MGX_FLAG_DCT_SEQUENTIAL": capi.FLAG_DCT_SEQUENTIAL, "MGX_FLAG_MFCC_REFERENCE": capi.FLAG_MFCC_REFERENCE,
                     "MGX_FLAG_RESIDENT": capi.FLAG_RESIDENT}
    assert capi.make_desc(resident=True).flags == capi.FLAG_RESIDENT
    d = capi.make_desc()
    d.flags = 8  # no such flag: rejected with the descriptor, before any device is touched
    h = ctypes.c_void_p()
    assert capi.lib().mgx_plan_create(ctypes.byref(d), ctypes.byref(h)) == -1
    assert b"unknown plan flags" in capi.lib().mgx_last_error()


@pytest.mark.parametrize("n", [512, 1024, 2048])
def test_host_tables_bit_exact(capi, n):
    g = golden_io.load(n)
    t = capi.host_tables(buffer_size=n)
    assert np.array_equal(t["hanning"].view(np.uint32), g["hann"].view(np.uint32))
    assert np.array_equal(t["hamming"].view(np.uint32), g["hamming"].view(np.uint32))
    assert np.array_equal(t["window"].view(np.uint32), g["hann"].view(np.uint32))
    assert np.array_equal(t["bark_scale"].view(np.uint32), g["bark"].view(np.uint32))
    assert np.array_equal(t["bark_limits"], g["bblimits"])
    assert np.array_equal(t["mel_bins"], g["mel_bins"])
    assert np.array_equal(t["dct"].view(np.uint32), g["dct"].view(np.uint32))
    t40 = capi.host_tables(buffer_size=n, num_mel_bands=40)
    assert np.array_equal(t40["mel_bins"], g["mel40_bins"])
    assert np.array_equal(t40["dct"].view(np.uint32), g["dct40"].view(np.uint32))
    th = capi.host_tables(buffer_size=n, window="hamming")
    assert np.array_equal(th["window"].view(np.uint32), g["hamming"].view(np.uint32))


def test_no_silent_cpu_fallback(capi):
    # Without a gfx950 device the plan must fail loudly (no CPU path exists).
    if capi.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(capi.MgxError) as ei:
        capi.Plan(buffer_size=1024)
    assert ei.value.status == -6


@pytest.mark.parametrize("n", [1, 2, 4])
def test_host_tables_tiny_buffer_sizes(capi, n):
    # isPowerOfTwo accepts 1 (src/utils.js:13-19), so new Meyda(ctx, src, 1) builds tables:
    # N/2 = 0 bins leaves barkScale[-1] undefined in computeBarkBandLimits
    # (loudness.js:24-45): no limit moves and the last is length - 1 = -1.
    t = capi.host_tables(buffer_size=n)
    L = n // 2
    assert t["bark_limits"][-1] == L - 1
    if L == 0:
        assert np.all(t["bark_limits"][:-1] == 0)
    assert t["hanning"].shape == (n,) and t["bark_scale"].shape == (n,)


def test_mel_weight_division_is_correctly_rounded(tmp_path):
    """kernels.hip mel_reference_order: the weight t/d of two small integers comes from
    r = 1/d as q0 = t r, e = fma(-q0, d, t), fma(e, r, q0). Exhaustively equal to the IEEE
    quotient (what mfcc.js:44-50 computes) for every 0 <= t <= d <= 4096."""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    src = tmp_path / "div.c"
    src.write_text(r"""
#include <math.h>
#include <stdio.h>
int main(void) {
  long bad = 0;
  for (int d = 1; d <= 4096; ++d) {
    volatile double dd = d, r = 1.0 / dd;
    for (int t = 0; t <= d; ++t) {
      volatile double tt = t, ref = tt / dd;
      const double q0 = tt * r;
      if (fma(fma(-q0, dd, tt), r, q0) != ref) ++bad;
    }
  }
  printf("%ld\n", bad);
  return 0;
}
""")
    exe = tmp_path / "div"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"])
    assert subprocess.check_output([str(exe)]).decode().strip() == "0"


def test_dct_scale_division_is_correctly_rounded(tmp_path):
    """kernels.hip div_by: the DCT's v / ncoef (mfcc.js:91) as q0 = v r, fma(fma(-q0, d, v), r, q0)
    with r = 1/d (Markstein). Equal to the IEEE quotient for every divisor 1..64 on 2^21
    random doubles per divisor spread over 2^-60..2^60 and both signs, plus the exact
    multiples; zeros and non-finite v keep q0."""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    src = tmp_path / "divby.c"
    src.write_text(r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x6D657964u;
static uint64_t next(void) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double div_by(double v, double d, double r) {
  const double q0 = v * r;
  const double q = fma(fma(-q0, d, v), r, q0);
  return (q0 != 0.0 && fabs(q0) < HUGE_VAL) ? q : q0;
}
static int same(double a, double b) { return memcmp(&a, &b, 8) == 0 || (a != a && b != b); }
int main(void) {
  long bad = 0;
  for (int d = 1; d <= 64; ++d) {
    volatile double dd = d, r = 1.0 / dd;
    for (int i = 0; i < (1 << 21); ++i) {
      const uint64_t u = next();
      double v = ldexp((double)(u >> 11) * 0x1p-53 + 0.5, (int)(u % 121) - 60);
      if (u & 1024) v = -v;
      volatile double vv = v;
      if (!same(div_by(vv, dd, r), vv / dd)) ++bad;
      volatile double m = (double)(int64_t)(u >> 40) * dd;  /* exact multiples */
      if (!same(div_by(m, dd, r), m / dd)) ++bad;
    }
    const double sp[] = {0.0, -0.0, HUGE_VAL, -HUGE_VAL, NAN};
    for (int k = 0; k < 5; ++k) if (!same(div_by(sp[k], dd, r), sp[k] / dd)) ++bad;
  }
  printf("%ld\n", bad);
  return 0;
}
""")
    exe = tmp_path / "divby"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"])
    assert subprocess.check_output([str(exe)], timeout=120).decode().strip() == "0"
