"""Host-side memory safety: the library's host code, a host-only driver and
the N-API addon built with AddressSanitizer + UndefinedBehaviorSanitizer (`make asan`,
build/asan/), run with clang's ASan runtime preloaded. The driver fuzzes the RIFF/WAVE walk
(every truncation and seeded mutations of files of every format, each in an exactly-sized
heap block), builds the host tables of every power-of-two size and band count into
exactly-sized buffers, and checks argument validation; the JS facade's host-side checks
then run through the sanitized addon. No GPU is needed."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")


def runtime():
    rt = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    if not rt or not os.path.exists(os.path.join(ASAN, "host_checks")):
        pytest.skip("sanitizer build absent (make asan)")
    return rt[0]


def env():
    e = dict(os.environ, LD_PRELOAD=runtime(), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
             UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return e


def test_host_checks_under_asan_ubsan():
    r = subprocess.run([os.path.join(ASAN, "host_checks")], capture_output=True, text=True, env=env(), timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host_checks: ok (0 failures)" in r.stdout
    assert "wav_parse:" in r.stdout


def test_js_facade_through_sanitized_addon():
    if not shutil.which("node"):
        pytest.skip("node is not installed")
    e = env()
    e["MEYDA_AMD_ADDON"] = os.path.join(ASAN, "addon", "meyda_napi.node")
    r = subprocess.run(["node", "--expose-gc", os.path.join(ROOT, "tests", "js", "facade_cpu.js")],
                       capture_output=True, text=True, env=e, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "facade_cpu: 9 checks passed" in r.stdout
