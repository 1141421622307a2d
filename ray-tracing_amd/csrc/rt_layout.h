// rt_layout.h — the device copy of a scene as the host prepares it and the kernels read it: node-id
// tags, stack bounds, kernel feature flags and variants, the device material record. Plain C++ (no
// HIP), shared by the host-only scene preparation (rt_prepare.cpp, also built under ASan/UBSan) and
// the kernels (rt_device.h).
#pragma once
#include <stdint.h>

#include "rt.h"
#include "rt_wide.h"

#ifndef RT_BLOCK
#define RT_BLOCK 128 /* threads per workgroup (2 waves) */
#endif
#ifndef RT_STACK
#define RT_STACK 32 /* traversal stack entries per lane (LDS) */
#endif
#ifndef RT_WSTACK
#define RT_WSTACK 48 /* the same for the 4-wide walk (up to 3 siblings stacked per level) */
#endif
#define RT_LIGHT_DEPTH 2  /* max BVH depth of the lights tree (host-validated) */
#define RT_MAX_FRAMES 4   /* max nesting of instance frames on the replacement loop (host-validated) */
#define RT_FRAME 0x40000000 /* stack-entry tag: instance frame marker */
#define RT_WNODE 0x10000000 /* node-id tag (mixed walks, F_MIXW): a 4-wide node of a re-bounded subtree */
#define RT_ISBOX 0x08000000 /* node-id tag: a BVH node (set by the upload on the device copy's BVH children
                               and on the roots), so that a walk schedules box steps without a load */
#define RT_WROOT 0x20000000 /* rt_node.c flag of an RT_BVH_ORDERED node whose subtree has a 4-wide tree, */
#define RT_WROOT_MASK 0x3ffffff /* whose root index is (c >> 2) & RT_WROOT_MASK (mixed walks) */
#define RT_ISMED 0x04000000 /* node-id tag: a ConstantMedium (set like RT_ISBOX), so that a walk can hold the
                               lanes at media back without a load (node ids stay below 2^26) */
#define RT_IDTAGS (RT_ISBOX | RT_ISMED) /* the kind tags every walk masks off a node id */
#define RT_SAMEBOX RT_IDTAGS /* both tags (a BVH node is no medium): the left child of a reference-order BVH node
                                whose box is bit-identical to its parent's, entered right after the parent's
                                passing test under the same bound: its own test would pass too */
#define RT_SUB 0x20000000   /* node-id tag (walks in the reference's order): inside a re-bounded,
                               media-free subtree (below an RT_BVH_ORDERED node) */
#define RT_CHAIN_PRIM 0x100 /* device node type flag: Translate/Rotate chain ending in a primitive */
/* Leaf-table copies of instance frames (mixed walks): the frame chain opened from this leaf is described by
   the copy itself, so the walk opens it without loading the chain's records. FUSED: one frame (this node),
   whose child `a` is not an instance frame opened with it; FUSED2: two frames, this one and its child `a`, a
   Rotate (sin f[3], cos f[4], axis (type >> RT_FRAME_AX2_SHIFT) & 3). Either way (int)f[5] is where the walk
   goes on inside: the innermost child, or RT_WNODE | the 4-wide tree of that child when it has one (its
   children's fp32 boxes cull what its own exact box test would). */
#define RT_FRAME_FUSED 0x200
#define RT_FRAME_FUSED2 0x400
#define RT_FRAME_AX2_SHIFT 11
#define RT_TYPE_MASK 0xff

namespace rtd {

// Scene features a kernel variant is compiled for (host picks the variant per scene).
enum : unsigned {
  F_RECT = 1u,    // Rect / Cuboid nodes
  F_MOVING = 2u,  // MovingSphere
  F_INST = 4u,    // Translate / Rotate
  F_MEDIA = 8u,   // ConstantMedium (+ Isotropic)
  F_LIGHTS = 16u, // a lights tree (Lambertian light sampling / pdf)
  F_TEX = 32u,    // Checker / Perlin / Image textures (and sphere u, v)
  F_FRAMES = 512u,  // instance frames (Translate/Rotate over a BVH) in the resumable walk
  F_ALL = 63u | 512u,
  F_UV = 64u,     // always compute sphere (u, v) (debug queries)
  F_COUNT = 128u, // counting build: per-lane work counters (DESIGN.md "Roofline")
  F_WIDE = 256u,  // resumable walk over the 4-wide fp32-box tree (rt_wide.h) instead of the binary one
  F_MIXW = 1024u, // the mixed walk (media / frame worlds) enters 4-wide fp32-box trees built over the
                  // re-bounded subtrees (RT_WROOT nodes) instead of walking them node by node
  F_SLIBM = 2048u, // tier A with RT_FLAG_SHARED_LIBM: sin / cos / log / atan / asin from include/rt_libm.h
                   // (the oracle's too) instead of OCML
  F_QNODE = 4096u, // (spheres-only F_WIDE kernels reading the tree from global memory) the quantised 4-wide
                   // nodes (rt_qnode) and the leaves' sphere quadruples instead of the 128 / 64-byte records
  F_SLEAF = 8192u, // (spheres-only F_WIDE kernels) leaf tests read the leaves' 32-byte sphere quadruples
                   // (Scene::sleaves, staged in LDS by the compact kernel) instead of the 64-byte records
  F_W8 = 16384u    // (spheres-only F_WIDE kernels reading the tree from global memory; A/B, RTAMD_W8=1) an
                   // 8-wide tree: node p is the 4-wide record pair (2p, 2p + 1), rt_bvh.cpp build_wide8_bvh
};

// Kernel variants: spheres-only (configs 1, 2, 5), Cornell-like (rects, instances, lights), full.
constexpr unsigned kVarSpheres = 0u;
constexpr unsigned kVarCornell = F_RECT | F_INST | F_LIGHTS;
// the full variant without light sampling (lights Unhittable: next_week_final, the textured
// scenes), whose Lambertian scatter needs no lights-tree code
constexpr unsigned kVarFullDark = (F_ALL & ~F_LIGHTS) | F_MIXW;
// the full variant with light sampling
constexpr unsigned kVarFull = F_ALL | F_MIXW;
inline unsigned variant_for(unsigned f) {
  if ((f & ~kVarSpheres) == 0) return kVarSpheres;
  if ((f & ~kVarCornell) == 0) return kVarCornell;
  return (f & F_LIGHTS) ? kVarFull : kVarFullDark;
}
inline bool is_full(unsigned var) { return (var & F_FRAMES) != 0; }

// Device material: the rt_material record plus whether its texture tree reads (u, v).
struct DMat {
  int type;
  int tex;
  double param;
  int needs_uv;
  int _pad;
};

}  // namespace rtd
