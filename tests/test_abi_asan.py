"""SURVEY 5 (race detection / sanitizers): the C ABI's argument checks and
error paths under host AddressSanitizer.  ``make asan`` (also run by
__graft_entry__.build()) builds the library with its host code instrumented
(-Xarch_host -fsanitize=address), and the ABI tests (tests/test_abi_errors.py: every
entry point fed bad sizes and null pointers, formatted error messages through
nr_last_error; tests/test_abi.py: every declared symbol exported) run against
it in a child process with the ASan runtime preloaded.  Any heap / stack /
global overflow or use-after-free in those paths aborts the child with an
AddressSanitizer report."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(REPO, "build", "asan", "libnerf_pl_amd_asan.so")


def _runtime():
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"],
                         capture_output=True, text=True, timeout=60)
    path = out.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_abi_checks_are_clean_under_asan():
    rt = _runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    subprocess.run(["make", "-C", REPO, "-j", "8", "asan"], check=True, capture_output=True,
                   timeout=1200)
    env = dict(os.environ, LD_PRELOAD=rt, NERF_PL_AMD_LIB=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        "tests/test_abi_errors.py", "tests/test_abi.py"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out
