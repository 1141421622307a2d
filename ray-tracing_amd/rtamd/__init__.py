"""rtamd — Python host mirror of the reference's render API over the C ABI (include/rt.h).

The reference (shaunplee/ray-tracing) is Haskell; its host API is the set of constructors in
src/Lib.hs (sphere, movingSphere, rect, cuboid, translate, rotate, constantMedium, makeBVH,
makePerlin, newCamera), the scene library src/Scenes.hs, and the render entry

    mkRenderStaticEnv :: Scene -> Camera -> (Int, Int) -> Int -> Int -> Int -> RenderStaticEnv
    runRender         :: RenderStaticEnv -> [RandGen] -> [Vector RGB]      (src/Lib.hs:92-108,1491)

This module exposes the same surface (same names, same argument meaning) on top of
librtamd.so, whose render path is hand-written HIP for gfx950. There is no CPU fallback: if the
shared library (or a GPU, for rendering) is missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTAMD_LIB", os.path.join(_HERE, "..", "build", "librtamd.so"))

# ----------------------------------------------------------------------------- C structs
RT_NODE_BVH, RT_NODE_SPHERE, RT_NODE_MOVING_SPHERE = 0, 1, 2
RT_NODE_RECT_XY, RT_NODE_RECT_XZ, RT_NODE_RECT_YZ = 3, 4, 5
RT_NODE_CUBOID, RT_NODE_TRANSLATE, RT_NODE_ROTATE = 6, 7, 8
RT_NODE_CONSTANT_MEDIUM, RT_NODE_UNHITTABLE, RT_NODE_EXT = 9, 10, 11
RT_RNG_EXACT, RT_RNG_PHILOX = 0, 1
RT_FLAG_NAN_CULL = 1
RT_FLAG_REFERENCE_CULL = 2
RT_FLAG_NAN_ZERO = 4  # parity diagnostic: NaN sample channels add 0 (rt.h)
RT_FLAG_SHARED_LIBM = 8  # tier A parity aid: the portable include/rt_libm.h transcendentals on both sides
RT_UPLOAD_REFERENCE_BVH = 1
RT_DEBUG_RESUMABLE = 4  # rt_debug_closest_hits: the render loop's resumable binary walk
RT_DEBUG_WIDE = 8       # rt_debug_closest_hits: the resumable walk over the 4-wide fp32-box tree
RT_DEBUG_QNODE = 16     # ... over its quantised form (rt_qnode) with sphere quadruples (spheres-only worlds)
RT_BVH_ORDERED = 0x40000000
RT_BVH_MEDIA_FIRST = 0x10000000
MATH_OPS = {"div": 0, "div_exact": 1, "sqrt": 2, "sin": 3, "cos": 4, "atan": 5, "asin": 6, "log": 7, "pow": 8,
            "ghc_atan2": 9, "tan": 10, "pow5": 11, "sl_sin": 12, "sl_cos": 13, "sl_atan": 14, "sl_asin": 15,
            "sl_log": 16, "sl_ghc_atan2": 17}  # sl_*: include/rt_libm.h (RT_FLAG_SHARED_LIBM)

# rt_debug_probe / oracle_probe: function -> op id, doubles per input / output record (rt.h)
PROBES = {"scatter": 0, "htbl_random": 1, "htbl_pdf": 2, "texture": 3, "get_ray": 4, "box": 5}
PROBE_IN = (18, 3, 6, 6, 2, 14)
PROBE_OUT = (14, 4, 2, 3, 8, 3)

XYPlane, XZPlane, YZPlane = 0, 1, 2
XAxis, YAxis, ZAxis = 0, 1, 2
RT_OK, RT_E_INVALID, RT_E_HIP, RT_E_NOMEM, RT_E_UNSUPPORTED, RT_E_STATE, RT_E_COMM = 0, -1, -2, -3, -4, -5, -6
RT_MAX_DEVICES = 16

SCENES = {
    "cornell": 0, "cornell_smoke": 1, "simple_light": 2, "earth": 3, "two_perlin_spheres": 4,
    "two_spheres": 5, "random_book_one": 6, "random": 7, "next_week_final": 8,
    "three_spheres": 9, "stress_spheres": 10,
}
CAMERAS = {"cornell": 0, "two_spheres": 1, "random_scene": 2, "next_week": 3}


class rt_node(C.Structure):
    _fields_ = [("f", C.c_double * 6), ("type", C.c_int32), ("a", C.c_int32), ("b", C.c_int32), ("c", C.c_int32)]


class rt_material(C.Structure):
    _fields_ = [("type", C.c_int32), ("texture", C.c_int32), ("param", C.c_double)]


class rt_texture(C.Structure):
    _fields_ = [("type", C.c_int32), ("a", C.c_int32), ("b", C.c_int32), ("c", C.c_int32), ("f", C.c_double * 4)]


class rt_perlin(C.Structure):
    _fields_ = [("ranvec", C.c_double * 768), ("perm_x", C.c_int32 * 256), ("perm_y", C.c_int32 * 256),
                ("perm_z", C.c_int32 * 256)]


class rt_image(C.Structure):
    _fields_ = [("offset", C.c_int64), ("width", C.c_int32), ("height", C.c_int32)]


class rt_scene_desc(C.Structure):
    _fields_ = [
        ("nodes", C.POINTER(rt_node)), ("n_nodes", C.c_int32), ("world_root", C.c_int32),
        ("lights_root", C.c_int32), ("n_materials", C.c_int32), ("materials", C.POINTER(rt_material)),
        ("textures", C.POINTER(rt_texture)), ("n_textures", C.c_int32), ("n_perlins", C.c_int32),
        ("perlins", C.POINTER(rt_perlin)), ("images", C.POINTER(rt_image)), ("n_images", C.c_int32),
        ("_pad", C.c_int32), ("image_pool", C.POINTER(C.c_uint8)), ("image_pool_bytes", C.c_int64),
        ("background", C.c_double * 3),
    ]


class rt_camera(C.Structure):
    _fields_ = [(n, C.c_double * 3) for n in ("origin", "llc", "horiz", "vert", "u", "v", "w")] + [
        ("lens_radius", C.c_double), ("t0", C.c_double), ("t1", C.c_double)]


class rt_launch_info(C.Structure):
    _fields_ = [("variant", C.c_uint32), ("loop", C.c_int32), ("lds_staged", C.c_int32), ("leaf_lds", C.c_int32),
                ("waves", C.c_int32), ("grid", C.c_int32), ("block", C.c_int32), ("dyn_lds_bytes", C.c_int32),
                ("work_items", C.c_int64), ("chunk", C.c_int32), ("wide_nodes", C.c_int32),
                ("chunk_batches", C.c_int32), ("_pad", C.c_int32)]


class rt_scene_info(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_nodes", "n_wide_nodes", "n_leaves", "world_root", "stack_need",
                                         "wide_stack_need")] + [("features", C.c_uint32), ("variant", C.c_uint32)] + [
        (n, C.c_int32) for n in ("rebuilt_bvh", "mixed_wide", "replace_ok", "ref_walk")]


class rt_frame_timing(C.Structure):
    _fields_ = [("n_devices", C.c_int32), ("device_allocs", C.c_int32), ("kernel_ms", C.c_double * RT_MAX_DEVICES),
                ("gather_ms", C.c_double), ("assemble_ms", C.c_double), ("frame_ms", C.c_double)]


class rt_render_params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32), ("max_depth", C.c_int32),
                ("rng_mode", C.c_int32), ("flags", C.c_uint32), ("seed", C.c_uint64), ("tile", C.c_int32),
                ("shard_rank", C.c_int32), ("shard_count", C.c_int32), ("_pad", C.c_int32)]


assert C.sizeof(rt_node) == 64 and C.sizeof(rt_material) == 16 and C.sizeof(rt_texture) == 48
assert C.sizeof(rt_perlin) == 9216 and C.sizeof(rt_camera) == 192 and C.sizeof(rt_render_params) == 48
assert C.sizeof(rt_scene_desc) == 112

# Every symbol include/rt.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "rt_abi_version", "rt_last_error", "rt_rand_gen", "rt_random_double", "rt_builder_create",
    "rt_builder_destroy", "rt_builder_gen", "rt_tex_constant", "rt_tex_checker", "rt_tex_perlin",
    "rt_tex_image", "rt_mat_lambertian", "rt_mat_metal", "rt_mat_dielectric", "rt_mat_diffuse_light",
    "rt_mat_isotropic", "rt_obj_sphere", "rt_obj_moving_sphere", "rt_obj_rect", "rt_obj_cuboid",
    "rt_obj_translate", "rt_obj_rotate", "rt_obj_constant_medium", "rt_obj_unhittable", "rt_obj_bvh",
    "rt_builder_finish", "rt_scene_named", "rt_camera_new", "rt_camera_named", "rt_write_ppm",
    "rt_device_count", "rt_create", "rt_destroy", "rt_upload_scene", "rt_render", "rt_shard_geometry",
    "rt_render_shard_async", "rt_assemble_async", "rt_assemble_linear_async", "rt_last_kernel_ms",
    "rt_debug_closest_hits", "rt_debug_math", "rt_render_work", "rt_upload_scene_ex", "rt_rebuild_bvh",
    "rt_wide_bvh", "rt_tree_stack_need", "rt_last_launch", "rt_write_pfm", "rt_debug_probe",
    "rt_prepare_scene", "rt_render_step_profile", "rt_create_multi", "rt_ctx_devices", "rt_last_frame_timing",
    "rt_debug_exact_trace", "rt_quantize_wide",
]

# include/rt_wide.h: one 4-wide node (128 B)
WNODE_DTYPE = np.dtype([("lo", "<f4", (3, 4)), ("hi", "<f4", (3, 4)), ("child", "<i4", (4,)), ("pad", "<i4", (4,))])

_lib = None


class RTError(RuntimeError):
    pass


def _share_torch_hip_runtime():
    """One HIP runtime per process. PyTorch-ROCm ships its own libamdhip64 (soname
    libamdhip64.so.7, like /opt/rocm's). If librtamd.so were loaded first, its DT_NEEDED would pull
    /opt/rocm's copy and torch would later map a second runtime that finds no GPU. Loading torch's
    copy globally first makes librtamd bind to it (same soname), whichever is imported first."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    # (RCCL, which librtamd.so links for the multi-device gather, is not preloaded this way: torch's
    # librccl.so carries /opt/rocm's soname librccl.so.1, so the process maps one RCCL whichever library
    # is loaded first, and preloading torch's copy globally aborts the interpreter at exit)
    hip = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(hip):
        C.CDLL(hip, mode=C.RTLD_GLOBAL)


def lib() -> C.CDLL:
    """Load librtamd.so (raises if it has not been built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RTError(f"librtamd.so not found at {LIB_PATH}; run __graft_entry__.build() / make")
        _share_torch_hip_runtime()
        L = C.CDLL(LIB_PATH)
        D, I, U64 = C.c_double, C.c_int, C.c_uint64
        P = C.POINTER
        sig = {
            "rt_abi_version": (I, []), "rt_last_error": (C.c_char_p, []),
            "rt_rand_gen": (None, [C.c_int64, P(U64)]), "rt_random_double": (D, [P(U64)]),
            "rt_builder_create": (I, [P(U64), P(C.c_void_p)]), "rt_builder_destroy": (None, [C.c_void_p]),
            "rt_builder_gen": (None, [C.c_void_p, P(U64)]),
            "rt_tex_constant": (I, [C.c_void_p, D, D, D]), "rt_tex_checker": (I, [C.c_void_p, I, I]),
            "rt_tex_perlin": (I, [C.c_void_p, D]),
            "rt_tex_image": (I, [C.c_void_p, P(C.c_uint8), I, I]),
            "rt_mat_lambertian": (I, [C.c_void_p, I]), "rt_mat_metal": (I, [C.c_void_p, I, D]),
            "rt_mat_dielectric": (I, [C.c_void_p, D]), "rt_mat_diffuse_light": (I, [C.c_void_p, I]),
            "rt_mat_isotropic": (I, [C.c_void_p, I]),
            "rt_obj_sphere": (I, [C.c_void_p, P(D), D, I]),
            "rt_obj_moving_sphere": (I, [C.c_void_p, P(D), P(D), D, D, D, I]),
            "rt_obj_rect": (I, [C.c_void_p, I, D, D, D, D, D, I]),
            "rt_obj_cuboid": (I, [C.c_void_p, P(D), P(D), I]),
            "rt_obj_translate": (I, [C.c_void_p, P(D), I]), "rt_obj_rotate": (I, [C.c_void_p, I, D, I]),
            "rt_obj_constant_medium": (I, [C.c_void_p, D, I, I]), "rt_obj_unhittable": (I, [C.c_void_p]),
            "rt_obj_bvh": (I, [C.c_void_p, P(I), I, I, D, D]),
            "rt_builder_finish": (I, [C.c_void_p, I, I, P(D), P(rt_scene_desc)]),
            "rt_scene_named": (I, [C.c_void_p, I, D, D, P(C.c_uint8), I, I, C.c_int64, P(rt_scene_desc)]),
            "rt_camera_new": (None, [P(D), P(D), P(D), D, D, D, D, D, D, P(rt_camera)]),
            "rt_camera_named": (I, [I, I, I, P(rt_camera)]),
            "rt_write_ppm": (I, [P(C.c_uint8), I, I, C.c_char_p, C.c_size_t, P(C.c_size_t)]),
            "rt_device_count": (I, [P(I)]), "rt_create": (I, [I, P(C.c_void_p)]),
            "rt_destroy": (None, [C.c_void_p]), "rt_upload_scene": (I, [C.c_void_p, P(rt_scene_desc)]),
            "rt_render": (I, [C.c_void_p, P(rt_camera), P(rt_render_params), P(U64), P(C.c_uint8), P(D), P(U64)]),
            "rt_shard_geometry": (I, [P(rt_render_params), P(C.c_int64), P(C.c_int64), P(C.c_int64)]),
            "rt_render_shard_async": (I, [C.c_void_p, P(rt_camera), P(rt_render_params), C.c_void_p, C.c_void_p,
                                          C.c_void_p]),
            "rt_assemble_async": (I, [C.c_void_p, P(rt_render_params), C.c_void_p, C.c_void_p, C.c_void_p]),
            "rt_assemble_linear_async": (I, [C.c_void_p, P(rt_render_params), C.c_void_p, C.c_void_p, C.c_void_p]),
            "rt_last_kernel_ms": (I, [C.c_void_p, P(D)]),
            "rt_debug_closest_hits": (I, [C.c_void_p, P(D), I, D, D, U64, C.c_uint32, P(D)]),
            "rt_debug_math": (I, [C.c_void_p, I, P(D), P(D), I, P(D)]),
            "rt_render_work": (I, [C.c_void_p, P(rt_camera), P(rt_render_params), P(U64)]),
            "rt_upload_scene_ex": (I, [C.c_void_p, P(rt_scene_desc), C.c_uint32]),
            "rt_rebuild_bvh": (I, [P(rt_scene_desc), P(rt_node), I, P(I), P(I)]),
            "rt_wide_bvh": (I, [P(rt_node), I, I, C.c_void_p, I, P(I), P(I)]),
            "rt_quantize_wide": (I, [C.c_void_p, I, C.c_void_p]),
            "rt_tree_stack_need": (I, [P(rt_node), I, I, P(I)]),
            "rt_last_launch": (I, [C.c_void_p, P(rt_launch_info)]),
            "rt_write_pfm": (I, [P(D), I, I, I, C.c_char_p, C.c_size_t, P(C.c_size_t)]),
            "rt_debug_probe": (I, [C.c_void_p, P(rt_camera), I, P(D), I, U64, P(D)]),
            "rt_prepare_scene": (I, [P(rt_scene_desc), C.c_uint32, P(rt_scene_info)]),
            "rt_render_step_profile": (I, [C.c_void_p, P(rt_camera), P(rt_render_params), P(U64), P(U64)]),
            "rt_create_multi": (I, [I, P(I), P(C.c_void_p)]),
            "rt_ctx_devices": (I, [C.c_void_p, P(I), P(I), I]),
            "rt_last_frame_timing": (I, [C.c_void_p, P(rt_frame_timing)]),
            "rt_debug_exact_trace": (I, [C.c_void_p, P(rt_camera), P(rt_render_params), P(U64), I, P(D), I, P(I)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise RTError(f"{what} failed ({rc}): {lib().rt_last_error().decode()}")
    return rc


def _dp(a: Sequence[float]):
    return (C.c_double * len(a))(*[float(x) for x in a])


# ----------------------------------------------------------------------------- RNG (src/Random.hs)
def randGen(s: int) -> Tuple[int, int]:
    """randGen s = mkStdGen s (src/Random.hs:20-21); returns the SMGen (seed, gamma)."""
    g = (C.c_uint64 * 2)()
    lib().rt_rand_gen(int(s), g)
    return int(g[0]), int(g[1])


def randomDouble(gen: Tuple[int, int]) -> Tuple[float, Tuple[int, int]]:
    """randomDouble (src/Random.hs:23-25): (draw, next generator)."""
    g = (C.c_uint64 * 2)(*gen)
    x = lib().rt_random_double(g)
    return x, (int(g[0]), int(g[1]))


# ----------------------------------------------------------------------------- scenes
class Scene:
    """A built scene: the flattened (world, lights, background) of src/Lib.hs:84.

    Owns the rt_builder whose memory the descriptor points into."""

    def __init__(self, builder: "Builder", desc: rt_scene_desc):
        self._builder = builder
        self.desc = desc

    @property
    def nodes(self) -> np.ndarray:
        return _struct_array(self.desc.nodes, self.desc.n_nodes, rt_node)

    @property
    def materials(self) -> np.ndarray:
        return _struct_array(self.desc.materials, self.desc.n_materials, rt_material)

    @property
    def textures(self) -> np.ndarray:
        return _struct_array(self.desc.textures, self.desc.n_textures, rt_texture)

    @property
    def perlins(self) -> np.ndarray:
        return _struct_array(self.desc.perlins, self.desc.n_perlins, rt_perlin)


def _struct_array(ptr, n, ctype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=np.dtype(np.void, C.sizeof(ctype)))
    buf = (ctype * n).from_address(C.addressof(ptr.contents))
    return np.ctypeslib.as_array(buf).copy()


class Builder:
    """Scene construction with a threaded RandGen (src/Lib.hs constructors + makeBVH/makePerlin)."""

    def __init__(self, gen: Tuple[int, int]):
        g = (C.c_uint64 * 2)(*gen)
        h = C.c_void_p()
        _check(lib().rt_builder_create(g, C.byref(h)), "rt_builder_create")
        self._h = h
        self._earth = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.rt_builder_destroy(h)
            self._h = None

    @property
    def gen(self) -> Tuple[int, int]:
        g = (C.c_uint64 * 2)()
        lib().rt_builder_gen(self._h, g)
        return int(g[0]), int(g[1])

    # textures / materials
    def constantColor(self, r, g, b) -> int:
        return _check(lib().rt_tex_constant(self._h, r, g, b), "ConstantColor")

    def checkerTexture(self, odd: int, even: int) -> int:
        return _check(lib().rt_tex_checker(self._h, odd, even), "CheckerTexture")

    def makePerlin(self, scale: float) -> int:
        return _check(lib().rt_tex_perlin(self._h, scale), "makePerlin")

    def imageTexture(self, rgb: Optional[np.ndarray]) -> int:
        if rgb is None:
            return _check(lib().rt_tex_image(self._h, None, 0, 0), "ImageTexture")
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w, _ = rgb.shape
        return _check(lib().rt_tex_image(self._h, rgb.ctypes.data_as(C.POINTER(C.c_uint8)), w, h), "ImageTexture")

    def lambertian(self, tex: int) -> int:
        return _check(lib().rt_mat_lambertian(self._h, tex), "Lambertian")

    def metal(self, tex: int, fuzz: float) -> int:
        return _check(lib().rt_mat_metal(self._h, tex, fuzz), "Metal")

    def dielectric(self, ref_idx: float) -> int:
        return _check(lib().rt_mat_dielectric(self._h, ref_idx), "Dielectric")

    def diffuseLight(self, tex: int) -> int:
        return _check(lib().rt_mat_diffuse_light(self._h, tex), "DiffuseLight")

    def isotropic(self, tex: int) -> int:
        return _check(lib().rt_mat_isotropic(self._h, tex), "Isotropic")

    # hittables
    def sphere(self, center, radius, mat) -> int:
        return _check(lib().rt_obj_sphere(self._h, _dp(center), radius, mat), "sphere")

    def movingSphere(self, c0, c1, t0, t1, radius, mat) -> int:
        return _check(lib().rt_obj_moving_sphere(self._h, _dp(c0), _dp(c1), t0, t1, radius, mat), "movingSphere")

    def rect(self, plane, a0, a1, b0, b1, k, mat) -> int:
        return _check(lib().rt_obj_rect(self._h, plane, a0, a1, b0, b1, k, mat), "rect")

    def cuboid(self, pmin, pmax, mat) -> int:
        return _check(lib().rt_obj_cuboid(self._h, _dp(pmin), _dp(pmax), mat), "cuboid")

    def translate(self, offset, child) -> int:
        return _check(lib().rt_obj_translate(self._h, _dp(offset), child), "translate")

    def rotate(self, axis, angle, child) -> int:
        return _check(lib().rt_obj_rotate(self._h, axis, angle, child), "rotate")

    def constantMedium(self, density, tex, boundary) -> int:
        return _check(lib().rt_obj_constant_medium(self._h, density, tex, boundary), "constantMedium")

    def unhittable(self) -> int:
        return _check(lib().rt_obj_unhittable(self._h), "Unhittable")

    def makeBVH(self, mtime: Optional[Tuple[float, float]], items: Sequence[int]) -> int:
        arr = (C.c_int * len(items))(*items)
        t0, t1 = mtime if mtime is not None else (0.0, 0.0)
        return _check(lib().rt_obj_bvh(self._h, arr, len(items), int(mtime is not None), t0, t1), "makeBVH")

    def finish(self, world: int, lights: int, background) -> Scene:
        d = rt_scene_desc()
        _check(lib().rt_builder_finish(self._h, world, lights, _dp(background), C.byref(d)), "finish")
        return Scene(self, d)


def rebuilt_scene(scene: Scene) -> Scene:
    """The scene as the device traverses it by default: the world tree re-bounded by the SAH
    rebuild of rt_rebuild_bvh (same leaves, same lights tree)."""
    n, root = C.c_int(0), C.c_int(0)
    _check(lib().rt_rebuild_bvh(C.byref(scene.desc), None, 0, C.byref(n), C.byref(root)), "rt_rebuild_bvh")
    arr = (rt_node * n.value)()
    _check(lib().rt_rebuild_bvh(C.byref(scene.desc), arr, n.value, C.byref(n), C.byref(root)), "rt_rebuild_bvh")
    d = rt_scene_desc()
    C.pointer(d)[0] = scene.desc
    d.nodes = C.cast(arr, C.POINTER(rt_node))
    d.n_nodes = n.value
    d.world_root = root.value
    s = Scene(scene._builder, d)
    s._keep = (arr, scene)
    return s


def prepare_scene(scene, reference_bvh: bool = False) -> dict:
    """rt_prepare_scene: the host half of the upload, no device needed (validation with the upload's
    error codes, and the device copy it would make). `scene` is a Scene or an rt_scene_desc."""
    d = scene.desc if isinstance(scene, Scene) else scene
    info = rt_scene_info()
    _check(lib().rt_prepare_scene(C.byref(d), RT_UPLOAD_REFERENCE_BVH if reference_bvh else 0, C.byref(info)),
           "rt_prepare_scene")
    return {k: getattr(info, k) for k, _ in rt_scene_info._fields_}


def wide_bvh(scene: Scene, root: Optional[int] = None) -> Tuple[np.ndarray, int]:
    """rt_wide_bvh: the 4-wide collapse of the binary tree at `root` (default: the scene's world
    root) as WNODE_DTYPE records, and the walk's stack bound."""
    n, need = C.c_int(0), C.c_int(0)
    r = scene.desc.world_root if root is None else root
    _check(lib().rt_wide_bvh(scene.desc.nodes, scene.desc.n_nodes, r, None, 0, C.byref(n), C.byref(need)),
           "rt_wide_bvh")
    out = np.zeros(n.value, dtype=WNODE_DTYPE)
    _check(lib().rt_wide_bvh(scene.desc.nodes, scene.desc.n_nodes, r, out.ctypes.data_as(C.c_void_p), n.value,
                             C.byref(n), C.byref(need)), "rt_wide_bvh")
    return out, need.value


QNODE_DTYPE = np.dtype([("origin", "<f4", 3), ("scale", "<f4", 3), ("qlo", "<u4", 3), ("qhi", "<u4", 3),
                        ("child", "<i4", 4)])


def quantize_wide(wnodes: np.ndarray) -> np.ndarray:
    """rt_quantize_wide: the 64-byte quantised form (rt_qnode) of WNODE_DTYPE records."""
    w = np.ascontiguousarray(wnodes, dtype=WNODE_DTYPE)
    out = np.zeros(len(w), dtype=QNODE_DTYPE)
    _check(lib().rt_quantize_wide(w.ctypes.data_as(C.c_void_p), len(w), out.ctypes.data_as(C.c_void_p)),
           "rt_quantize_wide")
    return out


def tree_stack_need(scene: Scene, root: Optional[int] = None) -> int:
    """rt_tree_stack_need: the binary walk's stack bound (entries) for the tree at `root`
    (default: the scene's world root), as rt_upload_scene sizes the LDS stacks."""
    need = C.c_int(0)
    r = scene.desc.world_root if root is None else root
    _check(lib().rt_tree_stack_need(scene.desc.nodes, scene.desc.n_nodes, r, C.byref(need)), "rt_tree_stack_need")
    return need.value


def make_scene(name: str, gen: Tuple[int, int], t0: float = 0.0, t1: float = 1.0,
               earth: Optional[np.ndarray] = None, param: int = 0) -> Tuple[Scene, Tuple[int, int]]:
    """A src/Scenes.hs builder: returns (scene, g1) like `makeXScene t0 t1 gen`."""
    b = Builder(gen)
    d = rt_scene_desc()
    if earth is not None:
        earth = np.ascontiguousarray(earth, dtype=np.uint8)
        b._earth = earth
        ep, eh, ew = earth.ctypes.data_as(C.POINTER(C.c_uint8)), earth.shape[0], earth.shape[1]
    else:
        ep, eh, ew = None, 0, 0
    _check(lib().rt_scene_named(b._h, SCENES[name], t0, t1, ep, ew, eh, int(param), C.byref(d)), "rt_scene_named")
    return Scene(b, d), b.gen


def newCamera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, t0, t1) -> rt_camera:
    """newCamera (src/Lib.hs:1269-1295)."""
    cam = rt_camera()
    lib().rt_camera_new(_dp(lookfrom), _dp(lookat), _dp(vup), vfov, aspect, aperture, focus_dist, t0, t1,
                        C.byref(cam))
    return cam


def camera(name: str, width: int, height: int) -> rt_camera:
    """cornellCamera / twoSpheresSceneCamera / randomSceneCamera / nextWeekFinalSceneCamera."""
    cam = rt_camera()
    _check(lib().rt_camera_named(CAMERAS[name], width, height, C.byref(cam)), "rt_camera_named")
    return cam


# ----------------------------------------------------------------------------- render
@dataclass
class RenderStaticEnv:
    """mkRenderStaticEnv scene camera (w, h) ns maxDepth nThreads (src/Lib.hs:92-108)."""
    scene: Scene
    camera: rt_camera
    size: Tuple[int, int]
    num_samples: int
    max_depth: int
    num_threads: int = 1  # stored but unused, as in the reference (Lib.hs:108,182-184)


def mkRenderStaticEnv(scene, camera, size, ns, max_depth, n_threads=1) -> RenderStaticEnv:
    return RenderStaticEnv(scene, camera, tuple(size), int(ns), int(max_depth), int(n_threads))


def make_params(width, height, spp, max_depth, rng_mode=RT_RNG_PHILOX, seed=1024, flags=0, tile=8,
                shard_rank=0, shard_count=1) -> rt_render_params:
    p = rt_render_params()
    p.width, p.height, p.spp, p.max_depth = width, height, spp, max_depth
    p.rng_mode, p.flags, p.seed, p.tile = rng_mode, flags, seed, tile
    p.shard_rank, p.shard_count = shard_rank, shard_count
    return p


def device_count() -> int:
    n = C.c_int(0)
    _check(lib().rt_device_count(C.byref(n)), "rt_device_count")
    return n.value


class Context:
    """One HIP device (one process per GPU), or with `devices`, one context over several GPUs driven
    from this thread (rt_create_multi: tier-B renders are tile-sharded over the devices and gathered
    to the first with RCCL)."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        h = C.c_void_p()
        if devices is None:
            _check(lib().rt_create(device, C.byref(h)), "rt_create")
        else:
            devs = (C.c_int * len(devices))(*devices)
            _check(lib().rt_create_multi(len(devices), devs, C.byref(h)), "rt_create_multi")
            device = int(devices[0])
        self._h = h
        self.device = device
        self._scene = None

    def devices(self) -> List[int]:
        """rt_ctx_devices: the ctx's HIP devices (RCCL rank order)."""
        n = C.c_int(0)
        out = (C.c_int * RT_MAX_DEVICES)()
        _check(lib().rt_ctx_devices(self._h, C.byref(n), out, RT_MAX_DEVICES), "rt_ctx_devices")
        return [int(out[i]) for i in range(n.value)]

    def frame_timing(self) -> dict:
        """rt_last_frame_timing: per-device render kernel ms, RCCL gather ms, assemble ms, frame ms of the
        last rt_render, and the device allocations it made (0 for a repeated frame of one size)."""
        t = rt_frame_timing()
        _check(lib().rt_last_frame_timing(self._h, C.byref(t)), "rt_last_frame_timing")
        return {"n_devices": t.n_devices, "device_allocs": t.device_allocs,
                "kernel_ms": [t.kernel_ms[i] for i in range(t.n_devices)],
                "gather_ms": t.gather_ms, "assemble_ms": t.assemble_ms, "frame_ms": t.frame_ms}

    def close(self):
        if self._h is not None:
            lib().rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene: Scene, reference_bvh: bool = False):
        _check(lib().rt_upload_scene_ex(self._h, C.byref(scene.desc), RT_UPLOAD_REFERENCE_BVH if reference_bvh else 0),
               "rt_upload_scene")
        self._scene = scene

    def render(self, cam: rt_camera, params: rt_render_params, col_gens: Optional[np.ndarray] = None,
               linear: bool = False, want_gens: bool = False):
        """Full image, blocking. Returns (rgb8[H,W,3], linear[H,W,3] | None, gens[W,2] | None)."""
        W, H = params.width, params.height
        rgb = np.zeros((H, W, 3), dtype=np.uint8)
        lin = np.zeros((H, W, 3), dtype=np.float64) if linear else None
        gens_in = None
        if params.rng_mode == RT_RNG_EXACT:
            if col_gens is None:
                raise RTError("tier A (RT_RNG_EXACT) needs col_gens: 2*width uint64 words")
            gens_in = np.ascontiguousarray(col_gens, dtype=np.uint64).reshape(-1)
            if gens_in.size != 2 * W:
                raise RTError("col_gens must hold 2*width words")
        gens_out = np.zeros((W, 2), dtype=np.uint64) if want_gens else None
        P = C.POINTER
        _check(lib().rt_render(
            self._h, C.byref(cam), C.byref(params),
            gens_in.ctypes.data_as(P(C.c_uint64)) if gens_in is not None else None,
            rgb.ctypes.data_as(P(C.c_uint8)),
            lin.ctypes.data_as(P(C.c_double)) if lin is not None else None,
            gens_out.ctypes.data_as(P(C.c_uint64)) if gens_out is not None else None), "rt_render")
        return rgb, lin, gens_out

    def render_shard_async(self, cam, params, d_slab_rgb: int, d_slab_lin: int = 0, stream: int = 0):
        _check(lib().rt_render_shard_async(self._h, C.byref(cam), C.byref(params), C.c_void_p(d_slab_rgb),
                                           C.c_void_p(d_slab_lin or None), C.c_void_p(stream or None)),
               "rt_render_shard_async")

    def assemble_async(self, params, d_slabs: int, d_image: int, stream: int = 0):
        _check(lib().rt_assemble_async(self._h, C.byref(params), C.c_void_p(d_slabs), C.c_void_p(d_image),
                                       C.c_void_p(stream or None)), "rt_assemble_async")

    def assemble_linear_async(self, params, d_slabs: int, d_image: int, stream: int = 0):
        _check(lib().rt_assemble_linear_async(self._h, C.byref(params), C.c_void_p(d_slabs), C.c_void_p(d_image),
                                              C.c_void_p(stream or None)), "rt_assemble_linear_async")

    WORK_FIELDS = ("segments", "box_tests", "prim_tests", "other_tests", "light_pdfs", "philox_blocks", "samples",
                   "wide_nodes")

    def render_work(self, cam, params) -> dict:
        """Device-measured work of one tier-B render (counting build): totals per field."""
        w = (C.c_uint64 * 16)()
        _check(lib().rt_render_work(self._h, C.byref(cam), C.byref(params), w), "rt_render_work")
        out = dict(zip(self.WORK_FIELDS, [int(x) for x in w[:8]]))
        tot = max(1, int(w[8]) + int(w[9]) + int(w[10]))
        out["phase_split"] = {"acquire_camera": int(w[8]) / tot, "traverse": int(w[9]) / tot, "shade": int(w[10]) / tot}
        # replacement loop only: live-lane slots of 4-wide node steps, leaf steps and outer iterations
        out["lane_slots"] = {"wide_steps": int(w[11]), "leaf_steps": int(w[12]), "outer_iterations": int(w[13])}
        out["leaf_hits"] = int(w[14])  # replacement loop only: leaf tests that found a hit
        out["tie_redos"] = int(w[15])  # replacement loop only: walks (or samples) redone for an exact tie
        return out

    STEP_KINDS = ("box", "wide", "leaf", "medium", "frame")

    def step_profile(self, cam, params) -> dict:
        """rt_render_step_profile: the walk's steps by the set of node kinds their lanes were at:
        {"box+leaf": (ticks, steps), ...} (s_memtime ticks, counting build). Binary and mixed walks: the kinds
        of the lanes that stepped; the 4-wide walk (round 6): "wide" (node steps), "leaf" (leaf steps),
        "box+wide" (node steps in which some lane walks a tie redo on the caller's tree)."""
        w, p = (C.c_uint64 * 16)(), (C.c_uint64 * 64)()
        _check(lib().rt_render_step_profile(self._h, C.byref(cam), C.byref(params), w, p), "rt_render_step_profile")
        out = {}
        for m in range(32):
            if p[32 + m]:
                name = "+".join(k for i, k in enumerate(self.STEP_KINDS) if m >> i & 1) or "none"
                out[name] = (int(p[m]), int(p[32 + m]))
        return out

    def last_launch(self) -> dict:
        """rt_last_launch: which kernel the last tier-B render launch ran (variant bits, loop, LDS
        staging, waves per SIMD, grid, block, dynamic LDS, work-items, samples per work-item)."""
        info = rt_launch_info()
        _check(lib().rt_last_launch(self._h, C.byref(info)), "rt_last_launch")
        return {k: getattr(info, k) for k, _ in rt_launch_info._fields_}

    def last_kernel_ms(self) -> float:
        ms = C.c_double(0)
        _check(lib().rt_last_kernel_ms(self._h, C.byref(ms)), "rt_last_kernel_ms")
        return ms.value

    def closest_hits(self, rays: np.ndarray, tmin: float, tmax: float, seed: int = 0, flags: int = 0) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 7)
        out = np.zeros((rays.shape[0], 12), dtype=np.float64)
        P = C.POINTER
        _check(lib().rt_debug_closest_hits(self._h, rays.ctypes.data_as(P(C.c_double)), rays.shape[0], tmin, tmax,
                                           seed, flags, out.ctypes.data_as(P(C.c_double))), "rt_debug_closest_hits")
        return out

    def exact_trace(self, cam, params, col_gens, col: int, cap: int = 1 << 20) -> np.ndarray:
        """rt_debug_exact_trace: tier A, column `col`'s path segments (rows of 10 doubles: row, sample, seg,
        o, d, seed bits), as pyoracle.exact_trace records them."""
        gi = np.ascontiguousarray(col_gens, dtype=np.uint64).reshape(-1)
        out = np.zeros((cap, 10), dtype=np.float64)
        n = C.c_int(0)
        P = C.POINTER
        _check(lib().rt_debug_exact_trace(self._h, C.byref(cam), C.byref(params), gi.ctypes.data_as(P(C.c_uint64)),
                                          col, out.ctypes.data_as(P(C.c_double)), cap, C.byref(n)),
               "rt_debug_exact_trace")
        return out[: n.value].copy()

    def probe(self, op: str, inputs: np.ndarray, seed: int = 0, cam: Optional[rt_camera] = None) -> np.ndarray:
        """rt_debug_probe: one hot-path function per record on the device (PROBES: layouts)."""
        k = PROBES[op]
        x = np.ascontiguousarray(inputs, dtype=np.float64).reshape(-1, PROBE_IN[k])
        out = np.zeros((x.shape[0], PROBE_OUT[k]), dtype=np.float64)
        P = C.POINTER
        _check(lib().rt_debug_probe(self._h, C.byref(cam) if cam is not None else None, k,
                                    x.ctypes.data_as(P(C.c_double)), x.shape[0], seed,
                                    out.ctypes.data_as(P(C.c_double))), "rt_debug_probe")
        return out

    def math(self, op: str, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
        y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, dtype=np.float64).reshape(-1)
        out = np.zeros_like(x)
        P = C.POINTER
        _check(lib().rt_debug_math(self._h, MATH_OPS[op], x.ctypes.data_as(P(C.c_double)),
                                   y.ctypes.data_as(P(C.c_double)), x.size, out.ctypes.data_as(P(C.c_double))),
               "rt_debug_math")
        return out


def shard_geometry(params: rt_render_params) -> Tuple[int, int, int]:
    tt, ps, sp = C.c_int64(), C.c_int64(), C.c_int64()
    _check(lib().rt_shard_geometry(C.byref(params), C.byref(tt), C.byref(ps), C.byref(sp)), "rt_shard_geometry")
    return tt.value, ps.value, sp.value


def runRender(env: RenderStaticEnv, gens: Sequence[Tuple[int, int]], device: int = 0,
              ctx: Optional[Context] = None) -> List[np.ndarray]:
    """runRender (src/Lib.hs:1491): tier A, generator x for column x; rows top first.

    As the reference's `VV.zip gs row` (src/Lib.hs:1519), every row holds min(len(gens), W) pixels:
    extra generators are ignored, and with fewer generators than columns the rows are truncated to
    the first len(gens) columns (a column's stream depends only on its own generator and position,
    so the missing columns are rendered with copies of the first generator and cut off)."""
    W, H = env.size
    gens = list(gens)[:W]
    cols = len(gens)
    if cols == 0 or H <= 0:
        return [np.zeros((0, 3), dtype=np.uint8) for _ in range(max(0, H))]
    full = gens + [gens[0]] * (W - cols)
    own = ctx is None
    ctx = ctx or Context(device)
    try:
        ctx.upload(env.scene)
        p = make_params(W, H, env.num_samples, env.max_depth, RT_RNG_EXACT)
        rgb, _, _ = ctx.render(env.camera, p, np.array(full, dtype=np.uint64))
    finally:
        if own:
            ctx.close()
    return [rgb[i, :cols].copy() for i in range(H)]


def column_gens(g1: Tuple[int, int], width: int, seed: int = 1024) -> np.ndarray:
    """The deterministic harness for app/Main.hs:47-49: column 0 = g1 (post-scene generator),
    column x >= 1 = randGen (seed + x) in place of the clock-seeded newRandGen."""
    out = np.zeros((width, 2), dtype=np.uint64)
    out[0] = g1
    for x in range(1, width):
        out[x] = randGen(seed + x)
    return out


def write_ppm(rgb: np.ndarray) -> bytes:
    """P3 text exactly as app/Main.hs:59-63 / printRow (src/Lib.hs:299-305)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W, _ = rgb.shape
    n = C.c_size_t(0)
    P = C.POINTER
    _check(lib().rt_write_ppm(rgb.ctypes.data_as(P(C.c_uint8)), W, H, None, 0, C.byref(n)), "rt_write_ppm")
    buf = C.create_string_buffer(n.value)
    _check(lib().rt_write_ppm(rgb.ctypes.data_as(P(C.c_uint8)), W, H, buf, n.value, C.byref(n)), "rt_write_ppm")
    return buf.raw[: n.value]


def write_pfm(linear: np.ndarray, f64: bool = False) -> bytes:
    """rt_write_pfm: the per-pixel averages (H x W x 3 doubles, top row first) as PFM (float32, bottom
    row first) or, with f64, the lossless "PF64" variant."""
    lin = np.ascontiguousarray(linear, dtype=np.float64)
    H, W, _ = lin.shape
    n = C.c_size_t(0)
    P = C.POINTER
    _check(lib().rt_write_pfm(lin.ctypes.data_as(P(C.c_double)), W, H, int(f64), None, 0, C.byref(n)), "rt_write_pfm")
    buf = C.create_string_buffer(n.value)
    _check(lib().rt_write_pfm(lin.ctypes.data_as(P(C.c_double)), W, H, int(f64), buf, n.value, C.byref(n)),
           "rt_write_pfm")
    return buf.raw[: n.value]


def read_pfm(data: bytes) -> np.ndarray:
    """Parse rt_write_pfm output back to H x W x 3 float64, top row first."""
    magic, dims, scale, rest = data.split(b"\n", 3)
    W, H = (int(x) for x in dims.split())
    dt = "<f8" if magic == b"PF64" else ("<f4" if float(scale) < 0 else ">f4")
    a = np.frombuffer(rest, dtype=dt, count=W * H * 3).astype(np.float64).reshape(H, W, 3)
    return a[::-1].copy()


# ----------------------------------------------------------------------------- tiling (host mirror)
def shard_pixel_map(params: rt_render_params) -> np.ndarray:
    """Slab work index -> image pixel index (row * W + x) or -1 for padding, for one shard.
    Host restatement of the kernel's work_pixel() mapping (tile-major, 8x8 blocks per tile)."""
    tt, per_shard, slab = shard_geometry(params)
    tile = params.tile or 8
    shards = max(1, params.shard_count)
    tiles_x = (params.width + tile - 1) // tile
    w = np.arange(slab, dtype=np.int64)
    tp = tile * tile
    lt, within = w // tp, w % tp
    gt = params.shard_rank + lt * shards
    blk, lane = within >> 6, within & 63
    bpr = tile >> 3
    px = (gt % tiles_x) * tile + (blk % bpr) * 8 + (lane & 7)
    row = (gt // tiles_x) * tile + (blk // bpr) * 8 + (lane >> 3)
    ok = (gt < tt) & (px < params.width) & (row < params.height)
    return np.where(ok, row * params.width + px, -1)


def assemble_host(slabs: np.ndarray, params: rt_render_params) -> np.ndarray:
    """Host restatement of the assemble kernel: (shards, slab, 3) -> (H, W, 3)."""
    W, H = params.width, params.height
    img = np.zeros((H * W, 3), dtype=slabs.dtype)
    for r in range(slabs.shape[0]):
        p = make_params(W, H, params.spp, params.max_depth, params.rng_mode, params.seed, params.flags,
                        params.tile, r, slabs.shape[0])
        m = shard_pixel_map(p)
        ok = m >= 0
        img[m[ok]] = slabs[r][ok]
    return img.reshape(H, W, 3)
