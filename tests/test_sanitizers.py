"""The host half under AddressSanitizer + UBSan: tests/c/Makefile `asan` compiles the
library's host-only sources (scene builders, makeBVH restatement, SAH / skeleton rebuild, Ylitie
collapse, rt_prepare_scene validation) and oracle/oracle.c for the CPU with the sanitizers, and
tests/c/host_check.cpp drives them: every named scene for two seeds, seeded descriptor mutations,
a deep spine, nested frames, builder misuse, and small oracle renders. Any report aborts the run."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TC = os.path.join(ROOT, "tests", "c")


def test_host_half_is_sanitizer_clean():
    subprocess.run(["make", "-s", "-C", TC, "asan"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(TC, "build", "host_check_asan")], capture_output=True, text=True, timeout=600,
                       env=env)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "host_check: clean (0 failures)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
