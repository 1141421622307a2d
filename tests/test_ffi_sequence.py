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


def test_reference_patch_applies(tmp_path):
    """integration/reference.patch (what the reference needs for integration/RenderAMD.hs: the Lib
    exports, splitmix as a library dependency, the link flags) applies cleanly to the reference's
    package.yaml and src/Lib.hs, and covers every package the module imports."""
    ref = "/root/reference"
    if not os.path.isdir(ref):
        pytest.skip("the reference checkout is not present on this machine")
    import shutil
    os.makedirs(tmp_path / "src")
    shutil.copy(os.path.join(ref, "package.yaml"), tmp_path / "package.yaml")
    shutil.copy(os.path.join(ref, "src", "Lib.hs"), tmp_path / "src" / "Lib.hs")
    patch = os.path.join(ROOT, "integration", "reference.patch")
    r = subprocess.run(["patch", "-p1", "-i", patch], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    pkg = (tmp_path / "package.yaml").read_text()
    lib = (tmp_path / "src" / "Lib.hs").read_text()
    assert "- splitmix" in pkg and "extra-libraries: rtamd" in pkg
    assert "Camera(..)" in lib and "Rectangle(..)" in lib and "RGB(..)" in lib
    hs = open(os.path.join(ROOT, "integration", "RenderAMD.hs")).read()
    imports = {"System.Random.SplitMix": "splitmix", "System.Random.Internal": "random", "Codec.Picture": "JuicyPixels",
               "Control.Monad.State.Strict": "mtl", "Data.Vector": "vector"}
    for mod, package in imports.items():
        if f"import           {mod}" in hs or f"import qualified {mod}" in hs:
            assert f"- {package}" in pkg, (mod, package)
