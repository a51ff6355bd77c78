"""Sanitizers (the reference has none; the build runs its CPU
restatement under AddressSanitizer + UndefinedBehaviorSanitizer).

The oracle's golden / known-answer tests (tests/test_golden.py, the oracle
half of tests/test_nms.py) are re-run in a child Python with the
`make -C oracle asan` build of oracle/o3d_oracle.c (O3DML_ORACLE_LIB) and the
sanitizer runtimes preloaded; any heap overflow, use after free or undefined
behaviour (signed overflow, misaligned or out-of-range shifts, ...) aborts the
child.  GPU code is not sanitized (not available on this pool); its
run-to-run determinism is tests/test_gpu_determinism.py."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    try:
        p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True, check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not available")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    env = dict(os.environ)
    env.update(O3DML_ORACLE_LIB=os.path.join(ROOT, "oracle", "_build", "liboracle_asan.so"),
               LD_PRELOAD=f"{asan}:{ubsan}", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(ROOT, "tests", "test_golden.py"), os.path.join(ROOT, "tests", "test_nms.py")],
                       env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout
