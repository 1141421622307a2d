"""integration/RenderAMD.hs (the Haskell FFI module; no GHC here, so never compiled) mirrored in C:
tests/c/ffi_sequence.c re-flattens builder scenes the way RenderAMD.flattenScene does (post-order,
one record per occurrence) and runs runRenderAMD's call sequence through include/rt.h. Compiled
with gcc against the in-tree librtamd.so; the rendering half needs the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "ray-tracing_amd", "build")


def _exe(tmp_path_factory):
    out = os.path.join(str(tmp_path_factory.mktemp("ffi")), "ffi_sequence")
    subprocess.run(["gcc", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "ffi_sequence.c"), "-o", out, "-L", BUILD, "-lrtamd",
                    f"-Wl,-rpath,{BUILD}"], check=True)
    return out


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    return _exe(tmp_path_factory)


def test_ffi_sequence_flattening_cpu(exe):
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and r.stdout.count("flattened") == 4


@pytest.mark.gpu
def test_ffi_sequence_renders_gpu(exe):
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and r.stdout.count("identical bytes") == 4
