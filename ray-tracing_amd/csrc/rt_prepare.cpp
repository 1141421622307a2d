// rt_prepare.cpp — the host half of rt_upload_scene: validation of a caller's descriptor, the world
// tree the device walks (rt_bvh.cpp: SAH rebuild, skeleton rebuild, 4-wide collapse), the mixed walk's
// wide subtrees, and the tagged device copy of every array. Plain C++ with no HIP: rt_render.hip
// copies the result to the device, and `make -C tests/c asan` builds it (with rt_bvh.cpp,
// rt_scene.cpp, rt_scenes.cpp) under AddressSanitizer + UBSan for the malformed-descriptor tests.
#include "rt_prepare.h"
#ifndef RT_FRAME_BATCH
#define RT_FRAME_BATCH 0
#endif

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <string>
#include <cstring>
#include <vector>

using namespace rtd;

namespace rt {
int rebuild_world_bvh(std::vector<rt_node>& nodes, int root);
int rebuild_for_device(std::vector<rt_node>& nodes, int root);
int unfold_media(std::vector<rt_node>& nodes, int root);
bool build_wide_bvh(const std::vector<rt_node>& nodes, int root, std::vector<rt_wnode>& out, int* stack_need);
bool quantize_wide(const std::vector<rt_wnode>& in, std::vector<rt_qnode>& out);
bool build_wide8_bvh(const std::vector<rt_node>& nodes, int root, std::vector<rt_wnode>& out, int* stack_need);
}  // namespace rt

namespace rt {
namespace {

struct Validator {
  const rt_scene_desc* d;
  std::vector<rt_node> nodes;  // device copy (type flags added)
  std::vector<int> stack_need, chain_prim, frame_depth;  // frame_depth: nesting of instance frames
  std::string err;

  // a child precedes its parent (the DAG is then acyclic) and is never a payload record
  bool child_ok(int parent, int child) {
    return child >= 0 && child < parent && d->nodes[child].type != RT_NODE_EXT;
  }

  bool run() {
    const int n = d->n_nodes;
    if (n <= 0 || !d->nodes) return fail("scene has no nodes");
    nodes.assign(d->nodes, d->nodes + n);
    stack_need.assign(n, 0);
    chain_prim.assign(n, 0);
    frame_depth.assign(n, 0);
    for (int i = 0; i < n; ++i) {
      rt_node& x = nodes[i];
      const int t = x.type;
      switch (t) {
        case RT_NODE_BVH:
          if (!child_ok(i, x.a) || !child_ok(i, x.b)) return fail("BVH child must precede its parent");
          if (x.c <= 0) return fail("BVH size must be positive");
          // an ordered (rebuilt) node's c is exactly the flag, RT_BVH_MEDIA_FIRST or not, and its split axis:
          // the walks read other bits of c as internal tags (RT_WROOT and a wide root index, set only by
          // the upload)
          if ((x.c & RT_BVH_ORDERED) && (x.c & ~(RT_BVH_ORDERED | RT_BVH_MEDIA_FIRST)) > 2)
            return fail("RT_BVH_ORDERED node must carry only its split axis (0..2) in c");
          stack_need[i] = rt::bvh_stack_need(x, stack_need[x.a], stack_need[x.b]);
          frame_depth[i] = std::max(frame_depth[x.a], frame_depth[x.b]);
          break;
        case RT_NODE_SPHERE:
        case RT_NODE_RECT_XY:
        case RT_NODE_RECT_XZ:
        case RT_NODE_RECT_YZ:
        case RT_NODE_CUBOID:
          if (x.a < 0 || x.a >= d->n_materials) return fail("primitive material out of range");
          chain_prim[i] = 1;
          break;
        case RT_NODE_MOVING_SPHERE:
          if (x.a < 0 || x.a >= d->n_materials) return fail("primitive material out of range");
          if (i + 1 >= n || d->nodes[i + 1].type != RT_NODE_EXT) return fail("MovingSphere needs its EXT record");
          chain_prim[i] = 1;
          break;
        case RT_NODE_TRANSLATE:
        case RT_NODE_ROTATE:
          if (!child_ok(i, x.a)) return fail("instance child must precede its parent");
          if (t == RT_NODE_ROTATE && (x.b < 0 || x.b > 2)) return fail("rotate axis out of range");
          if (chain_prim[x.a]) {
            chain_prim[i] = 1;
            x.type |= RT_CHAIN_PRIM;
          } else {
            stack_need[i] = 1 + stack_need[x.a];
            frame_depth[i] = 1 + frame_depth[x.a];
          }
          break;
        case RT_NODE_CONSTANT_MEDIUM:
          if (!child_ok(i, x.a)) return fail("medium boundary must precede the medium");
          if (!chain_prim[x.a])
            return unsup("ConstantMedium boundary must be a primitive or a Translate/Rotate chain of one");
          if (x.b < 0 || x.b >= d->n_materials) return fail("medium material out of range");
          // f[1]: 0, or the occurrence key + 1 of a medium already unfolded (rt_rebuild_bvh output)
          if (!(x.f[1] == 0.0 || (x.f[1] >= 1.0 && x.f[1] <= 2147483648.0 && x.f[1] == std::floor(x.f[1]))))
            return fail("ConstantMedium f[1] must be 0 or an occurrence key + 1 in [1, 2^31]");
          break;
        case RT_NODE_UNHITTABLE:
        case RT_NODE_EXT:
          break;
        default:
          return fail("unknown node type");
      }
    }
    if (d->world_root < 0 || d->world_root >= n || d->nodes[d->world_root].type == RT_NODE_EXT)
      return fail("world root out of range");
    if (stack_need[d->world_root] > RT_STACK - 2) return unsup("scene BVH too deep for the LDS traversal stack");
    if (d->lights_root >= n || (d->lights_root >= 0 && d->nodes[d->lights_root].type == RT_NODE_EXT))
      return fail("lights root out of range");
    if (d->lights_root >= 0 && !check_lights(d->lights_root, 0)) return false;
    return true;
  }
  bool has_media(int id) {
    const rt_node& x = d->nodes[id];
    if (x.type == RT_NODE_CONSTANT_MEDIUM) return true;
    if (x.type == RT_NODE_BVH) return has_media(x.a) || has_media(x.b);
    if (x.type == RT_NODE_TRANSLATE || x.type == RT_NODE_ROTATE) return has_media(x.a);
    return false;
  }
  bool check_lights(int id, int depth) {
    if (has_media(id)) return unsup("lights tree must not contain ConstantMedium");
    if (stack_need[id] > RT_STACK - 2) return unsup("lights tree too deep");
    const rt_node& x = d->nodes[id];
    if (x.type == RT_NODE_BVH) {
      if (x.c & RT_BVH_ORDERED) return fail("lights BVH node must carry its size (htblSize), not RT_BVH_ORDERED");
      if (depth >= RT_LIGHT_DEPTH) return unsup("lights BVH deeper than RT_LIGHT_DEPTH");
      return check_lights(x.a, depth + 1) && check_lights(x.b, depth + 1);
    }
    return true;
  }
  bool fail(const char* m) {
    err = m;
    code = RT_E_INVALID;
    return false;
  }
  bool unsup(const char* m) {
    err = m;
    code = RT_E_UNSUPPORTED;
    return false;
  }
  int code = RT_OK;
};

bool tex_needs_uv(const rt_scene_desc* d, int tid, int guard = 0) {
  if (tid < 0 || tid >= d->n_textures || guard > 64) return false;
  const rt_texture& t = d->textures[tid];
  if (t.type == RT_TEX_IMAGE) return true;
  if (t.type == RT_TEX_CHECKER) return tex_needs_uv(d, t.a, guard + 1) || tex_needs_uv(d, t.b, guard + 1);
  return false;
}

unsigned scene_features(const rt_scene_desc* d) {
  unsigned f = 0;
  for (int i = 0; i < d->n_nodes; ++i) {
    switch (d->nodes[i].type) {
      case RT_NODE_BVH:
      case RT_NODE_SPHERE: break;
      case RT_NODE_MOVING_SPHERE: f |= F_MOVING; break;
      case RT_NODE_TRANSLATE:
      case RT_NODE_ROTATE: f |= F_INST; break;
      case RT_NODE_CONSTANT_MEDIUM: f |= F_MEDIA; break;
      default: f |= F_RECT; break;  // rects, cuboids, and anything needing the full dispatch
    }
  }
  if (d->world_root >= 0 && d->world_root < d->n_nodes && d->nodes[d->world_root].type == RT_NODE_UNHITTABLE)
    f |= F_RECT;
  if (d->lights_root >= 0) f |= F_LIGHTS;
  for (int i = 0; i < d->n_textures; ++i)
    if (d->textures[i].type != RT_TEX_CONSTANT) f |= F_TEX;
  return f;
}

// An instance frame's leaf-table copy describes the frames it opens (RT_FRAME_FUSED, rt_layout.h): the
// mixed walk then opens them from the copy it has loaded already instead of loading each record of the
// chain in turn (C4: translate (rotate (1000 spheres))).
void fuse_frame(const std::vector<rt_node>& flat, const std::vector<int>& wroot, rt_node& leaf) {
  auto is_frame = [&](const rt_node& x) {
    const int ty = x.type & RT_TYPE_MASK;
    return (ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE) && !(x.type & RT_CHAIN_PRIM);
  };
  if (!is_frame(leaf)) return;
  auto target = [&](int id) { return (double)(wroot[id] >= 0 ? (RT_WNODE | wroot[id]) : id); };
  const rt_node& c1 = flat[leaf.a];
  if (!is_frame(c1)) {
    leaf.type |= RT_FRAME_FUSED;
    leaf.f[5] = target(leaf.a);
  } else if ((c1.type & RT_TYPE_MASK) == RT_NODE_ROTATE && !is_frame(flat[c1.a]) && c1.b >= 0 && c1.b <= 2) {
    leaf.type |= RT_FRAME_FUSED | RT_FRAME_FUSED2 | (c1.b << RT_FRAME_AX2_SHIFT);
    leaf.f[3] = c1.f[0];
    leaf.f[4] = c1.f[1];
    leaf.f[5] = target(c1.a);
  }
}

void mixed_wide_trees(PreparedScene& P, const std::vector<rt_node>& host, const std::vector<rt_node>& flat, int world,
                      int ref_need) {
  std::vector<rt_node>& dev = P.nodes;
  const int n = (int)dev.size();
  if (n >= RT_WNODE) return;  // (ids must stay clear of the RT_WNODE tag)
  std::vector<int> roots;
  // The top `bin` levels of each re-bounded subtree stay binary (exact fp64 box tests, RTAMD_MIXW_BIN,
  // default 0): the 4-wide trees start below them. lvl: -1 outside re-bounded subtrees, else the binary
  // levels above this node inside one; kIn: inside a 4-wide tree already.
  const char* bin_env = std::getenv("RTAMD_MIXW_BIN");
  const int bin = bin_env ? std::max(0, std::min(8, std::atoi(bin_env))) : 0;
  constexpr int kIn = 1 << 20;
  std::vector<char> seen((size_t)n * (bin + 3), 0);
  auto is_bvh_at = [&](int id) { return (flat[id].type & RT_TYPE_MASK) == RT_NODE_BVH; };
  std::function<void(int, int)> find = [&](int id, int lvl) {
    const size_t key = (size_t)id * (bin + 3) + (size_t)(lvl < 0 ? 0 : (lvl >= kIn ? bin + 2 : 1 + std::min(lvl, bin)));
    if (seen[key]) return;
    seen[key] = 1;
    const rt_node& x = flat[id];
    const int ty = x.type & RT_TYPE_MASK;
    if (ty == RT_NODE_BVH) {
      const bool ord = (x.c & RT_BVH_ORDERED) != 0;
      if (ord && (x.c & RT_BVH_MEDIA_FIRST)) {  // a hoisted medium (rt_bvh.cpp skeleton): in no 4-wide tree
        find(x.b, lvl);
        return;
      }
      int next = lvl;
      if (ord && lvl < kIn) {
        const int here = lvl < 0 ? 0 : lvl;
        if (here >= bin || !is_bvh_at(x.a) || !is_bvh_at(x.b)) {
          roots.push_back(id);
          next = kIn;
        } else {
          next = here + 1;
        }
      }
      find(x.a, next);  // (frames inside re-bounded subtrees hold subtrees of their own)
      find(x.b, next);
    } else if ((ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE) && !(x.type & RT_CHAIN_PRIM)) {
      find(x.a, -1);  // a frame: its child starts a new region
    }
  };
  find(world, -1);
  if (roots.empty()) return;
  std::vector<rt_wnode> wide;
  std::vector<int> wroot(n, -1), wneed_root(n, 0);
  for (int r : roots) {
    std::vector<rt_wnode> part;
    int need = 0;
    if (!rt::build_wide_bvh(host, r, part, &need)) return;
    const int base = (int)wide.size();
    if (base + (int)part.size() > RT_WROOT_MASK) return;
    for (rt_wnode& w : part)
      for (int k = 0; k < RT_WIDE; ++k)
        if (w.child[k] >= 0) w.child[k] = (w.child[k] + base) | RT_WNODE;
    wide.insert(wide.end(), part.begin(), part.end());
    wroot[r] = base;
  }
  // the leaf table (as for the 4-wide walk): each referenced leaf once, c = its flat id
  std::vector<rt_node> leaves;
  std::vector<int> slot(n, -1);
  for (rt_wnode& w : wide)
    for (int k = 0; k < RT_WIDE; ++k) {
      if (w.child[k] >= 0) continue;
      const int id = ~w.child[k];
      if (slot[id] < 0) {
        slot[id] = (int)leaves.size();
        leaves.push_back(flat[id]);
        leaves.back().c = id;
        if ((flat[id].type & RT_TYPE_MASK) == RT_NODE_MOVING_SPHERE) leaves.push_back(flat[id + 1]);
        fuse_frame(flat, wroot, leaves.back());
      }
      w.child[k] = ~slot[id];
#if RT_FRAME_BATCH
      // an instance frame's slot loses bit 26 (every walk decodes ~(x | RT_ISMED)), so that walk_until
      // tells lanes at frames without a load
      const int fty = flat[id].type & RT_TYPE_MASK;
      if ((fty == RT_NODE_TRANSLATE || fty == RT_NODE_ROTATE) && !(flat[id].type & RT_CHAIN_PRIM))
        w.child[k] &= ~RT_ISMED;
#endif
    }
  // Stack bound of the mixed walk: skeleton nodes left first, re-bounded binary nodes either child
  // first, a frame one entry, a wide node up to 3 stacked siblings (wide_node writes 3 slots) above the
  // deepest of its children — a wide node's leaf that is a frame opens it.
  std::vector<int> memo(n, -1);
  std::function<int(int)> need_of;
  std::function<int(int)> wneed = [&](int w) {
    int deepest = 0;
    for (int k = 0; k < RT_WIDE; ++k) {
      const int ch = wide[w].child[k];
      deepest = std::max(deepest, ch >= 0 ? wneed(ch & ~RT_WNODE) : need_of(leaves[~(ch | RT_ISMED)].c));
    }
    return 3 + deepest;
  };
  need_of = [&](int id) -> int {
    if (memo[id] >= 0) return memo[id];
    const rt_node& x = flat[id];
    const int ty = x.type & RT_TYPE_MASK;
    int r = 0;
    if (ty == RT_NODE_BVH) {
      if (wroot[id] >= 0) r = wneed(wroot[id]);
      else if ((x.c & RT_BVH_ORDERED) && !(x.c & RT_BVH_MEDIA_FIRST)) r = 1 + std::max(need_of(x.a), need_of(x.b));
      else r = std::max(1 + need_of(x.a), need_of(x.b));
    } else if ((ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE) && !(x.type & RT_CHAIN_PRIM)) {
      r = 1 + need_of(x.a);
    }
    return memo[id] = r;
  };
  const int need = need_of(world);
  // (+ 3: the walk's 2 entries of headroom, and one more for the leaf postponement's parked next node,
  // rt_trace.h kMixPostpone; beyond that the binary walk's bound stays)
  if (need + 3 > RT_WSTACK) return;
  for (int r : roots) dev[r].c = RT_BVH_ORDERED | (dev[r].c & 3) | RT_WROOT | (wroot[r] << 2);
  P.wnodes = std::move(wide);
  P.leaves = std::move(leaves);
  P.stack_need = std::max(need, ref_need);
  P.mixed_wide = true;
}

bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}

int fail_with(int code, const std::string& s) {
  set_error(s);
  return code;
}

}  // namespace

int prepare_scene(const rt_scene_desc* din, uint32_t flags, PreparedScene& P) {
  P = PreparedScene{};
  if (!din) return fail_with(RT_E_INVALID, "null argument");
  if (din->n_nodes <= 0 || !din->nodes || din->world_root < 0 || din->world_root >= din->n_nodes)
    return fail_with(RT_E_INVALID, "rt_upload_scene: bad node array or world root");
  if (din->n_materials < 0 || din->n_textures < 0 || din->n_perlins < 0 || din->n_images < 0 ||
      (din->n_materials > 0 && !din->materials) || (din->n_textures > 0 && !din->textures) ||
      (din->n_perlins > 0 && !din->perlins) || (din->n_images > 0 && !din->images))
    return fail_with(RT_E_INVALID, "rt_upload_scene: negative count or null array");
  // World-tree rebuild (rt_bvh.cpp) unless the caller or RTAMD_REFERENCE_BVH=1 asks for the
  // reference's own makeBVH tree; never for trees holding media.
  std::vector<rt_node> nodes(din->nodes, din->nodes + din->n_nodes);
  rt_scene_desc dd = *din;
  const char* env = std::getenv("RTAMD_REFERENCE_BVH");
  const bool keep = (flags & RT_UPLOAD_REFERENCE_BVH) || (env && env[0] == '1');
  // validate the original first so that unfolding and the rebuild only ever see well-formed DAGs
  Validator v0{din};
  if (!v0.run()) return fail_with(v0.code, "rt_upload_scene: " + v0.err);
  // every medium occurrence its own record, keyed (tier-B draws; rt_bvh.cpp unfold_media): the caller's
  // tree as the walks take it in the reference's order (tier A, exact-tie redos)
  const int unfolded = unfold_media(nodes, din->world_root);
  if (unfolded == -2)
    return fail_with(RT_E_INVALID, "rt_upload_scene: medium keys (f[1] = key + 1) must be set on every medium "
                                   "occurrence of the world or on none, distinct integers below 2^31");
  if (unfolded < 0)
    return fail_with(RT_E_UNSUPPORTED, "rt_upload_scene: the world's medium occurrences unfold to more than 2^22 records");
  dd.world_root = unfolded;
  if (!keep) {
    // Worlds without media or instance frames: a whole new tree over the same leaves (exact ties are
    // redone on the caller's tree). Worlds with media or frames: the same over leaves that include the
    // media and the frames, with the trees inside frames re-bounded too; RTAMD_SKELETON=0 keeps the
    // caller's tree as is.
    dd.world_root = rebuild_for_device(nodes, unfolded);
  }
  if ((int)nodes.size() >= RT_ISMED)
    return fail_with(RT_E_INVALID, "rt_upload_scene: too many nodes (ids must stay below 2^26)");
  dd.nodes = nodes.data();
  dd.n_nodes = (int)nodes.size();
  const rt_scene_desc* d = &dd;
  Validator v{d};
  if (!v.run()) return fail_with(v.code, "rt_upload_scene: " + v.err);
  for (int i = 0; i < d->n_textures; ++i) {
    const rt_texture& t = d->textures[i];
    if (t.type < RT_TEX_CONSTANT || t.type > RT_TEX_IMAGE) return fail_with(RT_E_INVALID, "rt_upload_scene: bad texture");
    if (t.type == RT_TEX_CHECKER && (t.a < 0 || t.a >= i || t.b < 0 || t.b >= i))
      return fail_with(RT_E_INVALID, "rt_upload_scene: checker children must precede the checker");
    if (t.type == RT_TEX_PERLIN && (t.a < 0 || t.a >= d->n_perlins))
      return fail_with(RT_E_INVALID, "rt_upload_scene: bad perlin id");
    if (t.type == RT_TEX_IMAGE && t.a >= 0) {
      if (t.a >= d->n_images) return fail_with(RT_E_INVALID, "rt_upload_scene: bad image id");
      const rt_image& im = d->images[t.a];
      if (im.width != t.b || im.height != t.c || im.width <= 0 || im.height <= 0 || im.offset < 0 ||
          im.offset + (int64_t)im.width * im.height * 3 > d->image_pool_bytes)
        return fail_with(RT_E_INVALID, "rt_upload_scene: image raster out of the pool");
    }
  }
  for (int i = 0; i < d->n_perlins; ++i) {  // (noise indexes ranvec with XORs of perm entries)
    const rt_perlin& q = d->perlins[i];
    for (int k = 0; k < 256; ++k)
      if ((unsigned)q.perm_x[k] > 255u || (unsigned)q.perm_y[k] > 255u || (unsigned)q.perm_z[k] > 255u)
        return fail_with(RT_E_INVALID, "rt_upload_scene: perlin permutation entry out of [0, 255]");
  }
  P.mats.resize(d->n_materials);
  for (int i = 0; i < d->n_materials; ++i) {
    const rt_material& m = d->materials[i];
    if (m.type < RT_MAT_LAMBERTIAN || m.type > RT_MAT_ISOTROPIC) return fail_with(RT_E_INVALID, "rt_upload_scene: bad material");
    if (m.type != RT_MAT_DIELECTRIC && (m.texture < 0 || m.texture >= d->n_textures))
      return fail_with(RT_E_INVALID, "rt_upload_scene: material texture out of range");
    P.mats[i] = DMat{m.type, m.texture, m.param, m.type != RT_MAT_DIELECTRIC && tex_needs_uv(d, m.texture), 0};
  }
  if (d->image_pool_bytes < 0 || (d->image_pool_bytes > 0 && !d->image_pool))
    return fail_with(RT_E_INVALID, "rt_upload_scene: image_pool is null but image_pool_bytes > 0");
  P.rebuilt_bvh = dd.world_root != unfolded;
  // BVH children that are BVH nodes carry RT_ISBOX in the device copy, media RT_ISMED (every walk masks
  // them off), so that the walks' step scheduling knows a node's kind without loading it
  const std::vector<rt_node> untagged = v.nodes;  // (the mixed walk's wide trees are built from it)
  auto is_bvh_id = [](const std::vector<rt_node>& ns, int id) { return (ns[id].type & RT_TYPE_MASK) == RT_NODE_BVH; };
  auto kind_tag = [&](int id) {
    const int ty = untagged[id].type & RT_TYPE_MASK;
    return ty == RT_NODE_BVH ? RT_ISBOX : (ty == RT_NODE_CONSTANT_MEDIUM ? RT_ISMED : 0);
  };
  for (rt_node& x : v.nodes)
    if ((x.type & RT_TYPE_MASK) == RT_NODE_BVH) {
      // a reference-order node always enters its left child next, under the bound its own test had: a
      // left child with the same box (makeBVH over a span dominated by one huge object, e.g. the fog
      // sphere of next_week_final) passes whenever the parent passed (RT_SAMEBOX)
      const bool same = !(x.c & RT_BVH_ORDERED) && is_bvh_id(untagged, x.a) &&
                        std::memcmp(untagged[x.a].f, x.f, 6 * sizeof(double)) == 0;
      x.a |= same ? RT_SAMEBOX : kind_tag(x.a);
      x.b |= kind_tag(x.b);
    }
  P.nodes = std::move(v.nodes);
  P.world = d->world_root | kind_tag(d->world_root);
  P.world_ref = unfolded | kind_tag(unfolded);
  P.world_root = d->world_root;
  P.lights = d->lights_root;
  P.features = scene_features(d);
  // (tie redo walks the caller's tree: size the stacks for both)
  P.stack_need = std::max(v.stack_need[d->world_root], v.stack_need[unfolded]);
  // The replacement loop takes every world whose frames nest at most RT_MAX_FRAMES deep (its Side
  // slots); worlds with media or frames walk the caller's tree in the reference's order.
  P.frame_depth = std::max(v.frame_depth[d->world_root], v.frame_depth[unfolded]);
  const bool frames = v.frame_depth[d->world_root] > 0;
  P.replace_ok = v.frame_depth[d->world_root] <= RT_MAX_FRAMES;
  P.ref_walk = (P.features & F_MEDIA) || frames;
  if (frames) P.features |= F_FRAMES;
  if (P.replace_ok && !P.ref_walk) {  // 4-wide fp32-box tree over the same world tree (unflagged node copy)
    std::vector<rt_wnode> wide;
    int need = 0;
    // RTAMD_W8=1 (A/B only): spheres-only worlds get the 8-wide tree as record pairs (F_W8 kernels; walked
    // from global memory, 4 entries of stack headroom)
    const char* w8env = std::getenv("RTAMD_W8");
    const bool w8 = w8env && w8env[0] == '1' && variant_for(P.features) == kVarSpheres;
    if ((w8 ? (build_wide8_bvh(nodes, d->world_root, wide, &need) && need + 4 <= 2 * RT_WSTACK)
            : (build_wide_bvh(nodes, d->world_root, wide, &need) && need + 3 <= RT_WSTACK)) &&
        (size_t)wide.size() < (size_t)INT32_MAX / 2) {
      P.w8 = w8;
      // The walk's leaf table: the leaves the wide tree references, each copied once (a moving
      // sphere with its EXT record), with `c` = the flat node id; leaf references ~id become ~slot.
      std::vector<rt_node> leaves;
      std::vector<int> slot(P.nodes.size(), -1);
      for (rt_wnode& w : wide)
        for (int k = 0; k < RT_WIDE; ++k) {
          if (w.child[k] >= 0) continue;
          const int id = ~w.child[k];
          if (slot[id] < 0) {
            slot[id] = (int)leaves.size();
            leaves.push_back(P.nodes[id]);
            leaves.back().c = id;
            if ((P.nodes[id].type & RT_TYPE_MASK) == RT_NODE_MOVING_SPHERE) leaves.push_back(P.nodes[id + 1]);
          }
          w.child[k] = ~slot[id];
        }
      // spheres-only worlds: the leaves' 32-byte sphere quadruples (centre, radius) beside the full
      // records — the compact LDS-staged kernel stages them (round 6) — and, RTAMD_QNODE=1 (A/B only), the
      // quantised nodes (rt_qnode) for the global-memory kernels. Measured on C5 at 100 spp, same box:
      // 1023 ms with 128-byte nodes, 1173 with quantised nodes (the plane decoding's VALU), 1030 with
      // only the 32-byte sphere leaves: the walk is not bound by the tree's footprint
      bool spheres = variant_for(P.features) == kVarSpheres;
      for (const rt_node& x : leaves) spheres &= (x.type & RT_TYPE_MASK) == RT_NODE_SPHERE;
      if (spheres) {
        P.sleaves.resize(4 * leaves.size());
        for (size_t i = 0; i < leaves.size(); ++i)
          for (int k = 0; k < 4; ++k) P.sleaves[4 * i + k] = leaves[i].f[k];
      }
      const char* qenv = std::getenv("RTAMD_QNODE");
      if (w8 || !(spheres && qenv && qenv[0] == '1' && quantize_wide(wide, P.qnodes))) P.qnodes.clear();
      P.wnodes = std::move(wide);
      P.leaves = std::move(leaves);
      P.wide_stack_need = std::max(need, v.stack_need[unfolded]);
    }
  }
  if (P.replace_ok && P.ref_walk && !env_off("RTAMD_MIXW"))
    mixed_wide_trees(P, nodes, untagged, d->world_root, v.stack_need[unfolded]);
  return RT_OK;
}

}  // namespace rt

extern "C" int rt_prepare_scene(const rt_scene_desc* desc, uint32_t flags, rt_scene_info* out) {
  if (!desc || !out) {
    rt::set_error("rt_prepare_scene: null argument");
    return RT_E_INVALID;
  }
  rt::PreparedScene P;
  const int rc = rt::prepare_scene(desc, flags, P);
  if (rc) return rc;
  rt_scene_info& o = *out;
  o = rt_scene_info{};
  o.n_nodes = (int)P.nodes.size();
  o.n_wide_nodes = (int)P.wnodes.size();
  o.n_leaves = (int)P.leaves.size();
  o.world_root = P.world_root;
  o.stack_need = P.stack_need;
  o.wide_stack_need = P.wide_stack_need;
  o.features = P.features;
  o.variant = variant_for(P.features);
  o.rebuilt_bvh = P.rebuilt_bvh;
  o.mixed_wide = P.mixed_wide;
  o.replace_ok = P.replace_ok;
  o.ref_walk = P.ref_walk;
  return RT_OK;
}
