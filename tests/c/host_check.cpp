// host_check.cpp — the host half of the library and the oracle under AddressSanitizer + UBSan
// (tests/c/Makefile `asan`; tests/test_sanitizers.py runs it). No GPU and no HIP: it links the
// host-only sources (rt_scene.cpp, rt_scenes.cpp, rt_bvh.cpp, rt_prepare.cpp) and oracle/oracle.c.
//
//   1. every named scene (src/Scenes.hs) for two seeds: build, rt_rebuild_bvh, rt_wide_bvh,
//      rt_tree_stack_need, rt_prepare_scene (SAH / skeleton rebuild, Ylitie collapse, mixed-walk
//      trees; the makeBVH restatement of src/Lib.hs:941-968 runs inside the builders);
//   2. seeded mutations of their descriptors (node fields, textures, materials, Perlin tables):
//      rt_prepare_scene must return RT_OK or an error code;
//   3. degenerate trees: a deep skewed spine (exponentially spaced centroids), a BVH over one item,
//      nested instance frames beyond RT_MAX_FRAMES, a lights tree deeper than 2;
//   4. the builder API with bad arguments;
//   5. the oracle: small tier-A / tier-B renders, closest hits and function probes;
//   6. the device copy's node-id kind tags (rt::prepare_scene): RT_ISBOX on BVH children, RT_ISMED on
//      media, RT_SAMEBOX only on the left child of a reference-order node with a bit-identical box,
//      and mixed-walk leaf slots that decode into the leaf table.
// Any sanitizer report aborts the process (-fno-sanitize-recover=all); exit 0 = clean.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt.h"
#include "rt_prepare.h"

extern "C" {
int oracle_render(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_params* p,
                  const uint64_t* col_gens, uint8_t* rgb, double* linear, uint64_t* out_gens, int nthreads);
int oracle_closest_hits(const rt_scene_desc* scene, const double* rays, int n, double tmin, double tmax,
                        uint64_t seed, double* out);
int oracle_probe(const rt_scene_desc* scene, const rt_camera* cam, int op, const double* in, int n, uint64_t seed,
                 double* out);
}

namespace {

int failures = 0;
#define CHECK(cond, ...)                   \
  do {                                     \
    if (!(cond)) {                         \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);            \
      std::printf("\n");                   \
      ++failures;                          \
    }                                      \
  } while (0)

uint64_t rng_state = 0x9e3779b97f4a7c15ULL;
uint64_t next_u64() {  // splitmix64 (test driver only)
  uint64_t z = (rng_state += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
int pick(int n) { return (int)(next_u64() % (uint64_t)n); }

struct Built {
  rt_builder* b = nullptr;
  rt_scene_desc d{};
  ~Built() { rt_builder_destroy(b); }
};

bool build_named(Built& s, int id, int64_t seed, const std::vector<uint8_t>& earth) {
  uint64_t g[2];
  rt_rand_gen(seed, g);
  if (rt_builder_create(g, &s.b)) return false;
  const bool img = id == RT_SCENE_EARTH || id == RT_SCENE_NEXT_WEEK_FINAL;
  return rt_scene_named(s.b, id, 0.0, 1.0, img ? earth.data() : nullptr, img ? 64 : 0, img ? 32 : 0,
                        id == RT_SCENE_STRESS_SPHERES ? 3000 : 0, &s.d) == RT_OK;
}

bool ok_code(int rc) { return rc == RT_OK || rc == RT_E_INVALID || rc == RT_E_UNSUPPORTED; }

void trees(const rt_scene_desc& d, const char* what) {
  int n = 0, root = 0;
  CHECK(rt_rebuild_bvh(&d, nullptr, 0, &n, &root) == RT_OK, "%s rebuild size", what);
  std::vector<rt_node> nodes((size_t)n);
  CHECK(rt_rebuild_bvh(&d, nodes.data(), n, &n, &root) == RT_OK, "%s rebuild", what);
  int need = 0;
  CHECK(rt_tree_stack_need(nodes.data(), n, root, &need) == RT_OK, "%s stack need", what);
  int wn = 0, wneed = 0;
  const int rc = rt_wide_bvh(nodes.data(), n, root, nullptr, 0, &wn, &wneed);
  if (rc == RT_OK) {
    std::vector<unsigned char> w((size_t)wn * 128);
    CHECK(rt_wide_bvh(nodes.data(), n, root, w.data(), wn, &wn, &wneed) == RT_OK, "%s wide", what);
  }
  for (uint32_t f : {0u, (uint32_t)RT_UPLOAD_REFERENCE_BVH}) {
    rt_scene_info info;
    CHECK(rt_prepare_scene(&d, f, &info) == RT_OK, "%s prepare(%u): %s", what, f, rt_last_error());
  }
}

// seeded mutations of a valid descriptor: the preparation must answer with a code, never crash
void mutate(const rt_scene_desc& d0, int rounds, const char* what) {
  std::vector<rt_node> nodes(d0.nodes, d0.nodes + d0.n_nodes);
  std::vector<rt_texture> texs(d0.textures, d0.textures + d0.n_textures);
  std::vector<rt_material> mats(d0.materials, d0.materials + d0.n_materials);
  std::vector<rt_perlin> perl(d0.perlins, d0.perlins + d0.n_perlins);
  int counts[3] = {0, 0, 0};
  for (int r = 0; r < rounds; ++r) {
    std::vector<rt_node> n = nodes;
    std::vector<rt_texture> t = texs;
    std::vector<rt_material> m = mats;
    std::vector<rt_perlin> p = perl;
    rt_scene_desc d = d0;
    const int edits = 1 + pick(3);
    for (int e = 0; e < edits; ++e) {
      const int vals[] = {-1, 0, 1, 2, 3, 6, 9, 11, 0x40000000 | 2, 0x2fffffff, (int)n.size(), (int)n.size() - 1};
      const int v = vals[pick(12)];
      switch (pick(7)) {
        case 0: n[pick((int)n.size())].type = v; break;
        case 1: n[pick((int)n.size())].a = v; break;
        case 2: n[pick((int)n.size())].b = v; break;
        case 3: n[pick((int)n.size())].c = v; break;
        case 4:
          if (!t.empty()) (pick(2) ? t[pick((int)t.size())].a : t[pick((int)t.size())].type) = v;
          break;
        case 5:
          if (!m.empty()) (pick(2) ? m[pick((int)m.size())].texture : m[pick((int)m.size())].type) = v;
          break;
        default:
          if (!p.empty()) p[pick((int)p.size())].perm_y[pick(256)] = v;
          else d.world_root = v;
      }
    }
    d.nodes = n.data();
    d.textures = t.empty() ? nullptr : t.data();
    d.materials = m.empty() ? nullptr : m.data();
    d.perlins = p.empty() ? nullptr : p.data();
    rt_scene_info info;
    const int rc = rt_prepare_scene(&d, (r & 1) ? RT_UPLOAD_REFERENCE_BVH : 0u, &info);
    CHECK(ok_code(rc), "%s mutation %d: code %d", what, r, rc);
    counts[rc == RT_OK ? 0 : (rc == RT_E_INVALID ? 1 : 2)]++;
  }
  std::printf("host_check: %s mutations ok=%d invalid=%d unsupported=%d\n", what, counts[0], counts[1], counts[2]);
}

void degenerate_trees() {
  uint64_t g[2];
  rt_rand_gen(7, g);
  {  // a skewed spine: centroids 2^k apart, so every SAH split peels one sphere off
    rt_builder* b = nullptr;
    CHECK(rt_builder_create(g, &b) == RT_OK, "builder");
    const int tex = rt_tex_constant(b, 0.5, 0.5, 0.5), mat = rt_mat_lambertian(b, tex);
    std::vector<int> items;
    for (int k = 0; k < 60; ++k) {
      const double c[3] = {std::ldexp(1.0, k / 2), 0.0, 0.0};
      items.push_back(rt_obj_sphere(b, c, 0.25, mat));
    }
    const int w = rt_obj_bvh(b, items.data(), (int)items.size(), 0, 0.0, 0.0);
    const double bg[3] = {0.7, 0.8, 1.0};
    rt_scene_desc d{};
    CHECK(rt_builder_finish(b, w, -1, bg, &d) == RT_OK, "spine finish");
    trees(d, "spine");
    mutate(d, 300, "spine");
    rt_builder_destroy(b);
  }
  {  // a BVH over one item (makeBVH's duplicated leaf), frames nested 6 deep, lights 3 deep
    rt_builder* b = nullptr;
    CHECK(rt_builder_create(g, &b) == RT_OK, "builder");
    const int tex = rt_tex_constant(b, 0.5, 0.5, 0.5), mat = rt_mat_lambertian(b, tex);
    const double c[3] = {0, 0, -1}, off[3] = {0.1, 0.0, 0.0};
    int s = rt_obj_sphere(b, c, 0.5, mat);
    int one = rt_obj_bvh(b, &s, 1, 0, 0.0, 0.0);
    int x = one;
    for (int k = 0; k < 6; ++k) x = (k & 1) ? rt_obj_rotate(b, k % 3, 10.0 * k, x) : rt_obj_translate(b, off, x);
    int pair[2] = {x, rt_obj_sphere(b, off, 0.2, mat)};
    const int w = rt_obj_bvh(b, pair, 2, 0, 0.0, 0.0);
    std::vector<int> ls;
    for (int k = 0; k < 9; ++k) ls.push_back(rt_obj_rect(b, k % 3, 0, 1, 0, 1, k, mat));
    const int lights = rt_obj_bvh(b, ls.data(), (int)ls.size(), 0, 0.0, 0.0);
    const double bg[3] = {0, 0, 0};
    rt_scene_desc d{};
    CHECK(rt_builder_finish(b, w, lights, bg, &d) == RT_OK, "frames finish");
    rt_scene_info info;
    const int rc = rt_prepare_scene(&d, 0, &info);
    CHECK(rc == RT_E_UNSUPPORTED, "lights tree 4 deep must be unsupported, got %d", rc);
    d.lights_root = -1;
    CHECK(rt_prepare_scene(&d, 0, &info) == RT_OK && !info.replace_ok, "6 nested frames: per-sample loop");
    mutate(d, 300, "frames");
    rt_builder_destroy(b);
  }
}

void builder_misuse() {
  uint64_t g[2];
  rt_rand_gen(3, g);
  rt_builder* b = nullptr;
  CHECK(rt_builder_create(g, &b) == RT_OK, "builder");
  const double c[3] = {0, 0, 0};
  CHECK(rt_mat_lambertian(b, 5) < 0, "material over a missing texture");
  CHECK(rt_tex_checker(b, 0, 1) < 0, "checker over missing textures");
  CHECK(rt_obj_sphere(b, c, 1.0, 3) < 0, "sphere with a missing material");
  CHECK(rt_obj_translate(b, c, 10) < 0, "translate of a missing child");
  const int bad_items[2] = {4, -2};
  CHECK(rt_obj_bvh(b, bad_items, 2, 0, 0.0, 0.0) < 0, "bvh over missing items");
  CHECK(rt_obj_bvh(b, nullptr, 0, 0, 0.0, 0.0) < 0, "bvh over nothing");
  CHECK(rt_tex_image(b, nullptr, 0, 0) >= 0, "image Nothing");
  rt_scene_desc d{};
  const double bg[3] = {0, 0, 0};
  CHECK(rt_builder_finish(b, 99, -1, bg, &d) < 0, "finish with a missing world");
  rt_builder_destroy(b);
  rt_scene_info info;
  CHECK(rt_prepare_scene(nullptr, 0, &info) == RT_E_INVALID, "null desc");
  rt_scene_desc empty{};
  CHECK(rt_prepare_scene(&empty, 0, &info) == RT_E_INVALID, "empty desc");
}

void oracle_runs(const rt_scene_desc& d, int cam_id, const char* what) {
  rt_camera cam;
  CHECK(rt_camera_named(cam_id, 24, 12, &cam) == RT_OK, "camera");
  for (int mode : {RT_RNG_PHILOX, RT_RNG_EXACT}) {
    rt_render_params p{};
    p.width = 24;
    p.height = 12;
    p.spp = 2;
    p.max_depth = 6;
    p.rng_mode = mode;
    p.seed = 1024;
    std::vector<uint64_t> gens(2 * 24), out_gens(2 * 24);
    for (int x = 0; x < 24; ++x) rt_rand_gen(1024 + x, &gens[2 * x]);
    std::vector<uint8_t> rgb(24 * 12 * 3);
    std::vector<double> lin(24 * 12 * 3);
    CHECK(oracle_render(&d, &cam, &p, gens.data(), rgb.data(), lin.data(), out_gens.data(), 1) == 0, "%s render %d",
          what, mode);
  }
  const int n = 64;
  std::vector<double> rays(7 * n), out(12 * n);
  for (int i = 0; i < n; ++i) {
    const double s = (i % 8) / 8.0, t = (i / 8) / 8.0;
    for (int k = 0; k < 3; ++k) {
      rays[7 * i + k] = cam.origin[k];
      rays[7 * i + 3 + k] = cam.llc[k] + s * cam.horiz[k] + t * cam.vert[k] - cam.origin[k];
    }
    rays[7 * i + 6] = 0.5;
  }
  CHECK(oracle_closest_hits(&d, rays.data(), n, 0.001, 1e300, 7, out.data()) == 0, "%s closest hits", what);
  std::vector<double> st(2 * n), ray_out(8 * n);
  for (int i = 0; i < 2 * n; ++i) st[i] = (i % 17) / 17.0;
  CHECK(oracle_probe(&d, &cam, 4, st.data(), n, 9, ray_out.data()) == 0, "%s getRay probe", what);
  if (d.n_textures > 0) {
    std::vector<double> tin(6 * n), tout(3 * n);
    for (int i = 0; i < n; ++i) {
      tin[6 * i] = i % d.n_textures;
      for (int k = 1; k < 6; ++k) tin[6 * i + k] = ((i * 7 + k * 3) % 19) / 19.0 - 0.3;
    }
    CHECK(oracle_probe(&d, &cam, 3, tin.data(), n, 9, tout.data()) == 0, "%s texture probe", what);
  }
}

// 6. Kind tags of the device copy (the walks schedule steps by them without a load, RT_SAMEBOX skips a box
// test): every tag must match the child it is on. Returns the number of RT_SAMEBOX tags.
int device_tags(const rt_scene_desc& d, const char* what) {
  rt::PreparedScene P;
  CHECK(rt::prepare_scene(&d, 0, P) == RT_OK, "%s prepare: %s", what, rt_last_error());
  const int n = (int)P.nodes.size();
  auto type_of = [&](int id) { return P.nodes[id].type & RT_TYPE_MASK; };
  int same = 0;
  for (int i = 0; i < n; ++i) {
    const rt_node& x = P.nodes[i];
    if ((x.type & RT_TYPE_MASK) != RT_NODE_BVH) continue;
    for (int side = 0; side < 2; ++side) {
      const int c = side ? x.b : x.a, id = c & ~RT_IDTAGS, tag = c & RT_IDTAGS;
      CHECK(id >= 0 && id < n, "%s node %d child id %d", what, i, id);
      if (id < 0 || id >= n) continue;
      const int ty = type_of(id);
      if (tag == RT_SAMEBOX) {
        ++same;
        CHECK(side == 0 && ty == RT_NODE_BVH && !(x.c & RT_BVH_ORDERED) &&
                  std::memcmp(P.nodes[id].f, x.f, 6 * sizeof(double)) == 0,
              "%s node %d: RT_SAMEBOX on a child that is not its left, same-box BVH child", what, i);
      } else {
        const int want = ty == RT_NODE_BVH ? RT_ISBOX : (ty == RT_NODE_CONSTANT_MEDIUM ? RT_ISMED : 0);
        CHECK(tag == want, "%s node %d child %d: tag %x, kind %d", what, i, id, tag, ty);
      }
    }
  }
  for (const rt_wnode& w : P.wnodes)
    for (int k = 0; k < RT_WIDE; ++k) {
      const int ch = w.child[k];
      if (ch >= 0) {
        CHECK((ch & ~RT_WNODE) < (int)P.wnodes.size(), "%s wide child %x", what, ch);
      } else {
        const int slot = ~(ch | RT_ISMED);
        CHECK(slot >= 0 && slot < (int)P.leaves.size(), "%s leaf slot %d of %zu", what, slot, P.leaves.size());
      }
    }
  return same;
}

}  // namespace

int main() {
  std::vector<uint8_t> earth(64 * 32 * 3);
  for (size_t i = 0; i < earth.size(); ++i) earth[i] = (uint8_t)(i * 37);
  const int cams[11] = {RT_CAM_CORNELL, RT_CAM_CORNELL, RT_CAM_TWO_SPHERES, RT_CAM_TWO_SPHERES, RT_CAM_TWO_SPHERES,
                        RT_CAM_TWO_SPHERES, RT_CAM_RANDOM_SCENE, RT_CAM_RANDOM_SCENE, RT_CAM_NEXT_WEEK,
                        RT_CAM_RANDOM_SCENE, RT_CAM_RANDOM_SCENE};
  for (int id = 0; id <= RT_SCENE_STRESS_SPHERES; ++id)
    for (int64_t seed : {1024, 77}) {
      Built s;
      char what[64];
      std::snprintf(what, sizeof what, "scene %d seed %lld", id, (long long)seed);
      CHECK(build_named(s, id, seed, earth), "%s build: %s", what, rt_last_error());
      trees(s.d, what);
      const int same = device_tags(s.d, what);
      // (next_week_final: the fog sphere's box is the root's and its two left descendants', in the device
      // tree and again in the caller's tree that tie redos walk)
      if (id == RT_SCENE_NEXT_WEEK_FINAL) CHECK(same >= 2, "%s: %d RT_SAMEBOX tags, expected at least 2", what, same);
      if (seed == 1024) {
        mutate(s.d, id == RT_SCENE_STRESS_SPHERES ? 100 : 400, what);
        oracle_runs(s.d, cams[id], what);
      }
    }
  degenerate_trees();
  builder_misuse();
  std::printf("host_check: %s (%d failures)\n", failures ? "FAILED" : "clean", failures);
  return failures ? 1 : 0;
}
