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


def _load_dump(path):
    """Parse ffi_sequence.c's <scene>.bin: the flattened descriptor (as an rt_scene_desc over numpy
    buffers), the params, the column generators and the GPU outputs of both tiers."""
    import ctypes as C

    import numpy as np

    import rtamd
    raw = open(path, "rb").read()
    hdr = np.frombuffer(raw, dtype="<i4", count=13)
    assert hdr[0] == 0x53465452 and hdr[1] == 1
    W, H, spp, depth, nn, nm, nt, npl, ni, world, lights = (int(x) for x in hdr[2:])
    off = 13 * 4
    pool_bytes = int(np.frombuffer(raw, dtype="<i8", count=1, offset=off)[0])
    off += 8
    bg = np.frombuffer(raw, dtype="<f8", count=3, offset=off)
    off += 24
    keep = []

    def take(ctype, n):
        nonlocal off
        size = C.sizeof(ctype) * n
        buf = (ctype * max(n, 1))()
        C.memmove(buf, raw[off:off + size], size)
        off += size
        keep.append(buf)
        return C.cast(buf, C.POINTER(ctype)) if n else None

    d = rtamd.rt_scene_desc()
    d.nodes, d.n_nodes, d.world_root, d.lights_root = take(rtamd.rt_node, nn), nn, world, lights
    d.materials, d.n_materials = take(rtamd.rt_material, nm), nm
    d.textures, d.n_textures = take(rtamd.rt_texture, nt), nt
    d.perlins, d.n_perlins = take(rtamd.rt_perlin, npl), npl
    d.images, d.n_images = take(rtamd.rt_image, ni), ni
    d.image_pool, d.image_pool_bytes = take(C.c_uint8, pool_bytes), pool_bytes
    d.background[:] = [float(x) for x in bg]

    def arr(dtype, count, shape):
        nonlocal off
        a = np.frombuffer(raw, dtype=dtype, count=count, offset=off).reshape(shape).copy()
        off += np.dtype(dtype).itemsize * count
        return a

    px = W * H * 3
    gens = arr("<u8", 2 * W, (W, 2))
    out = {"A": (arr("u1", px, (H, W, 3)), arr("<f8", px, (H, W, 3)), arr("<u8", 2 * W, (W, 2))),
           "B": (arr("u1", px, (H, W, 3)), arr("<f8", px, (H, W, 3)), None)}
    assert off == len(raw)

    class _Flat:  # what pyoracle.render reads: .desc
        pass
    sc = _Flat()
    sc.desc, sc._keep = d, keep
    return sc, (W, H, spp, depth), gens, out


CAMS = {"cornell": "cornell", "next_week_final": "next_week", "random": "random_scene", "cornell_smoke": "cornell"}
SCENES = {"cornell": "cornell", "next_week_final": "next_week_final", "random": "random",
          "cornell_smoke": "cornell_smoke"}


def test_ffi_flattening_renders_like_the_builder_cpu(exe, tmp_path):
    """RenderAMD.flattenScene's records (one per occurrence, as ffi_sequence.c re-flattens them) render
    under the CPU oracle exactly as the builder's own descriptor: same bytes, linear averages and tier-A
    end generators (the walk order, media draws and textures do not depend on record sharing)."""
    import numpy as np

    import pyoracle
    import rtamd
    r = subprocess.run([exe, "dump", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    e = np.arange(64 * 32 * 3, dtype=np.int64)
    earth = ((e * 37 + 11) & 0xFF).astype(np.uint8).reshape(32, 64, 3)  # ffi_sequence.c's synthetic raster
    for name, camname in CAMS.items():
        sc, (W, H, spp, depth), gens, _ = _load_dump(os.path.join(str(tmp_path), f"{name}.bin"))
        ref, g1 = rtamd.make_scene(SCENES[name], rtamd.randGen(1024), earth=earth)
        assert tuple(int(v) for v in gens[0]) == g1
        cam = rtamd.camera(camname, W, H)
        for mode in (rtamd.RT_RNG_EXACT, rtamd.RT_RNG_PHILOX):
            p = rtamd.make_params(W, H, spp, depth, mode, seed=1024)
            cg = gens if mode == rtamd.RT_RNG_EXACT else None
            a = pyoracle.render(sc, cam, p, col_gens=cg)
            b = pyoracle.render(ref, cam, p, col_gens=cg)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1], equal_nan=True), (name, mode)
            if cg is not None:
                assert np.array_equal(a[2], b[2])


@pytest.mark.gpu
def test_ffi_sequence_renders_gpu(exe, tmp_path):
    """runRenderAMD's call sequence on the GPU (rt_create_multi over every visible device, RCCL gather
    of the tier-B shards), checked two ways: against the builder's own descriptor rendered on one
    device (bytes and end generators identical), and against the CPU oracle rendering the same
    flattened records the program uploaded (tiers A and B: the north-star tolerance, tier-A end
    generators exact)."""
    import numpy as np

    import pyoracle
    import rtamd
    from conftest import parity
    r = subprocess.run([exe, "gpu", str(tmp_path)], capture_output=True, text=True, timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and r.stdout.count("identical bytes") == 4
    for name, camname in CAMS.items():
        sc, (W, H, spp, depth), gens, out = _load_dump(os.path.join(str(tmp_path), f"{name}.bin"))
        cam = rtamd.camera(camname, W, H)
        for tier, mode in (("A", rtamd.RT_RNG_EXACT), ("B", rtamd.RT_RNG_PHILOX)):
            p = rtamd.make_params(W, H, spp, depth, mode, seed=1024)
            rgb_o, lin_o, gens_o, _ = pyoracle.render(sc, cam, p, col_gens=gens if tier == "A" else None)
            rgb_g, lin_g, gens_g = out[tier]
            ok, eq, dmax = parity(lin_g, lin_o, rgb_g, rgb_o)
            print(f"ffi {name} tier {tier} {W}x{H}x{spp}: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, "
                  f"max |d| {dmax:.3g}")
            assert ok >= 0.999 and eq >= 0.999, (name, tier, ok, eq)
            if tier == "A":
                assert np.array_equal(gens_g, gens_o), f"{name}: tier-A end generators differ from the oracle's"


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
