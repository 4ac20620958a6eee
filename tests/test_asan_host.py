"""AddressSanitizer + UBSan build of the host-only code (CPU).

`make -C csrc asan` instruments the host halves of every source (CSV / PLY
parsers on mmap'd or streamed input, the pattern, multigrid and
decomposition plan builders, the ABI wrappers). Two runs:
  * tests/asan/asan_host.cpp drives the host-only entry points with
    well-formed and malformed CSV / PLY files, out-of-range indices and
    partition ids (any invalid access aborts it);
  * the Python CPU tests of those entry points run against the instrumented
    libmofhip (MOFHIP_LIB), with the sanitizer runtime preloaded into the
    interpreter.
No GPU code is launched; the sanitizers apply to host code only.
"""
import glob
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "manifold-based-optical-flow-method_amd", "csrc")
ASAN_DIR = os.path.join(CSRC, "build_asan")


def _runtime():
    libs = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return libs[-1] if libs else None


@pytest.fixture(scope="module")
def asan_build():
    if _runtime() is None:
        pytest.skip("clang ASan runtime not found")
    subprocess.check_call(["make", "-C", CSRC, "-j8", "asan"], stdout=subprocess.DEVNULL)
    return ASAN_DIR


def test_asan_driver(asan_build, tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([os.path.join(asan_build, "asan_host"), str(tmp_path)], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "asan_host: ok" in out.stdout
    assert "Sanitizer" not in out.stderr


def test_python_cpu_tests_under_asan(asan_build):
    lib = os.path.join(asan_build, "libmofhip_asan.so")
    env = dict(os.environ, MOFHIP_LIB=lib, LD_PRELOAD=_runtime(),
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0")
    probe = ("import mofhip._lib as L; L.lib(); "
             "print(any('libmofhip_asan.so' in l for l in open('/proc/self/maps')))")
    chk = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=300,
                         cwd=os.path.join(REPO, "manifold-based-optical-flow-method_amd"))
    assert chk.returncode == 0 and chk.stdout.strip() == "True", chk.stderr[-2000:]
    files = [os.path.join(REPO, "tests", f) for f in
             ("test_csv_io.py", "test_surface.py", "test_amg_host.py", "test_abi.py", "test_dd.py")]
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider", *files],
                         env=env, capture_output=True, text=True, timeout=900, cwd=REPO)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
