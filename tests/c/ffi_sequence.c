/*
 * ffi_sequence.c — the call sequence of integration/RenderAMD.hs (the Haskell FFI module, which
 * cannot be compiled here: no GHC), run in C through include/rt.h.
 *
 * RenderAMD.flattenScene walks the reference's Hittable tree (src/Lib.hs:521-585) in post-order and
 * emits one record per occurrence: shared values (the Cornell light in both trees, BVHNode h h, a
 * medium's boundary) are duplicated, every leaf gets its own material copy, every material its own
 * texture copy (checker children first), every Perlin / image texture its own table / raster. This
 * program re-flattens a builder-made scene (rt_scene_named: the restated Scenes.hs builders) the same
 * way from its roots, then:
 *   CPU: checks the re-flattened descriptor is well formed for the library (rt_rebuild_bvh,
 *        rt_tree_stack_need) and that the duplication is what the Haskell module produces;
 *   GPU (argv[1] == "gpu"): runs runRenderAMD's sequence — rt_create(0), rt_upload_scene, rt_render in
 *        tier A with one (seed, gamma) per column (the deterministic app/Main.hs:47-49 harness: column 0 =
 *        the builder's g1, column x = randGen (1024 + x)), rt_destroy — and runRenderAMDPhilox's (the same
 *        in tier B), and runRenderAMDPhiloxOn's (tier B on a rt_create_multi ctx over every visible GPU: the
 *        tile shards spread over the devices and gathered with RCCL), and checks the bytes and end-of-stream
 *        generators equal those of the builder's own descriptor rendered on one device. With argv[2] = a
 *        directory, it also writes <dir>/<scene>.bin: the flattened descriptor, the column generators
 *        and both tiers' outputs (RGB8, linear averages, tier-A end generators), which
 *        tests/test_ffi_sequence.py renders with the CPU oracle from the same flattened records.
 *   CPU, argv = "dump <dir>": writes the same files with zero outputs (the flattening checked on the
 *        CPU: the oracle renders the flattened records as it renders the builder's).
 * Exit 0 on success; prints one line per scene.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt.h"

typedef struct {
  rt_node* nodes; int n, cap;
  rt_material* mats; int nm, capm;
  rt_texture* texs; int nt, capt;
  rt_perlin* perlins; int np, capp;
  rt_image* images; int ni, capi;
  uint8_t* pool; int64_t pool_bytes, cap_pool;
} Flat;

#define PUSH(arr, n, cap, x)                                          \
  do {                                                                \
    if ((n) == (cap)) {                                               \
      (cap) = (cap) ? 2 * (cap) : 64;                                 \
      (arr) = realloc((arr), sizeof(*(arr)) * (size_t)(cap));         \
    }                                                                 \
    (arr)[(n)++] = (x);                                               \
  } while (0)

static const rt_scene_desc* S; /* the builder's descriptor being re-flattened */

/* textureValue's tree (src/Lib.hs:394-419) -> one copy per occurrence, children first */
static int flat_tex(Flat* f, int tid) {
  rt_texture t = S->textures[tid];
  if (t.type == RT_TEX_CHECKER) {
    t.a = flat_tex(f, t.a);
    t.b = flat_tex(f, t.b);
  } else if (t.type == RT_TEX_PERLIN) {
    PUSH(f->perlins, f->np, f->capp, S->perlins[t.a]);
    t.a = f->np - 1;
  } else if (t.type == RT_TEX_IMAGE && t.a >= 0) {
    const rt_image im = S->images[t.a];
    const int64_t bytes = (int64_t)im.width * im.height * 3;
    if (f->pool_bytes + bytes > f->cap_pool) {
      f->cap_pool = 2 * (f->pool_bytes + bytes);
      f->pool = realloc(f->pool, (size_t)f->cap_pool);
    }
    memcpy(f->pool + f->pool_bytes, S->image_pool + im.offset, (size_t)bytes);
    rt_image ni = {f->pool_bytes, im.width, im.height};
    f->pool_bytes += bytes;
    PUSH(f->images, f->ni, f->capi, ni);
    t.a = f->ni - 1;
  }
  PUSH(f->texs, f->nt, f->capt, t);
  return f->nt - 1;
}

static int flat_mat(Flat* f, int mid) {
  rt_material m = S->materials[mid];
  if (m.type != RT_MAT_DIELECTRIC) m.texture = flat_tex(f, m.texture);
  else m.texture = -1; /* (Dielectric has no texture: RenderAMD emits -1) */
  PUSH(f->mats, f->nm, f->capm, m);
  return f->nm - 1;
}

/* the Hittable tree, post-order (RenderAMD.flatHit) */
static int flat_hit(Flat* f, int id) {
  rt_node x = S->nodes[id];
  switch (x.type) {
    case RT_NODE_BVH: {
      const int a = flat_hit(f, x.a), b = flat_hit(f, x.b);
      x.a = a;
      x.b = b;
      break;
    }
    case RT_NODE_SPHERE:
    case RT_NODE_RECT_XY:
    case RT_NODE_RECT_XZ:
    case RT_NODE_RECT_YZ:
    case RT_NODE_CUBOID:
      x.a = flat_mat(f, x.a);
      break;
    case RT_NODE_MOVING_SPHERE: {
      x.a = flat_mat(f, x.a);
      PUSH(f->nodes, f->n, f->cap, x);
      PUSH(f->nodes, f->n, f->cap, S->nodes[id + 1]); /* its EXT record right after */
      return f->n - 2;
    }
    case RT_NODE_TRANSLATE:
    case RT_NODE_ROTATE:
      x.a = flat_hit(f, x.a);
      break;
    case RT_NODE_CONSTANT_MEDIUM: {
      const int b = flat_hit(f, x.a);
      x.a = b;
      x.b = flat_mat(f, x.b);
      break;
    }
    default:
      break; /* Unhittable */
  }
  PUSH(f->nodes, f->n, f->cap, x);
  return f->n - 1;
}

/* <dir>/<name>.bin (little-endian, native structs): "RTFS" v1; W H spp depth; n_nodes n_materials
   n_textures n_perlins n_images world lights; pool_bytes (i64); background[3]; the arrays; col gens
   (2W u64); tier A rgb8, linear (H*W*3 f64), end gens; tier B rgb8, linear */
static int dump(const char* dir, const char* name, const rt_scene_desc* d, int W, int H, int spp, int depth,
                const uint64_t* gens, const uint8_t* rgb_a, const double* lin_a, const uint64_t* go_a,
                const uint8_t* rgb_b, const double* lin_b) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s.bin", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  const int32_t hdr[13] = {0x53465452, 1, W, H, spp, depth, d->n_nodes, d->n_materials, d->n_textures,
                           d->n_perlins, d->n_images, d->world_root, d->lights_root};
  const size_t px = (size_t)W * H * 3;
  int ok = fwrite(hdr, sizeof hdr, 1, f) == 1 && fwrite(&d->image_pool_bytes, 8, 1, f) == 1 &&
           fwrite(d->background, 8, 3, f) == 3 &&
           fwrite(d->nodes, sizeof(rt_node), (size_t)d->n_nodes, f) == (size_t)d->n_nodes &&
           fwrite(d->materials, sizeof(rt_material), (size_t)d->n_materials, f) == (size_t)d->n_materials &&
           fwrite(d->textures, sizeof(rt_texture), (size_t)d->n_textures, f) == (size_t)d->n_textures &&
           fwrite(d->perlins, sizeof(rt_perlin), (size_t)d->n_perlins, f) == (size_t)d->n_perlins &&
           fwrite(d->images, sizeof(rt_image), (size_t)d->n_images, f) == (size_t)d->n_images &&
           fwrite(d->image_pool, 1, (size_t)d->image_pool_bytes, f) == (size_t)d->image_pool_bytes &&
           fwrite(gens, 8, 2 * (size_t)W, f) == 2 * (size_t)W && fwrite(rgb_a, 1, px, f) == px &&
           fwrite(lin_a, 8, px, f) == px && fwrite(go_a, 8, 2 * (size_t)W, f) == 2 * (size_t)W &&
           fwrite(rgb_b, 1, px, f) == px && fwrite(lin_b, 8, px, f) == px;
  ok = fclose(f) == 0 && ok;
  return !ok;
}

static int fail(const char* what) {
  fprintf(stderr, "FAIL %s: %s\n", what, rt_last_error());
  return 1;
}

static int run(int scene_id, const char* name, int cam_id, int W, int H, int spp, int gpu, const char* dir) {
  uint64_t g[2];
  rt_rand_gen(1024, g);
  rt_builder* b;
  if (rt_builder_create(g, &b)) return fail("rt_builder_create");
  /* a synthetic 64x32 earth raster (the real one is a fixture the C test does not parse) */
  uint8_t earth[64 * 32 * 3];
  for (int i = 0; i < 64 * 32 * 3; ++i) earth[i] = (uint8_t)(i * 37 + 11);
  rt_scene_desc a;
  if (rt_scene_named(b, scene_id, 0.0, 1.0, earth, 64, 32, 0, &a)) return fail("rt_scene_named");
  uint64_t g1[2];
  rt_builder_gen(b, g1);

  /* RenderAMD.flattenScene */
  S = &a;
  Flat f;
  memset(&f, 0, sizeof f);
  const int world = flat_hit(&f, a.world_root);
  const int lights = a.lights_root < 0 ? -1 : flat_hit(&f, a.lights_root);
  rt_scene_desc d = a;
  d.nodes = f.nodes;
  d.n_nodes = f.n;
  d.world_root = world;
  d.lights_root = lights;
  d.materials = f.mats;
  d.n_materials = f.nm;
  d.textures = f.texs;
  d.n_textures = f.nt;
  d.perlins = f.perlins;
  d.n_perlins = f.np;
  d.images = f.images;
  d.n_images = f.ni;
  d.image_pool = f.pool;
  d.image_pool_bytes = f.pool_bytes;

  /* CPU: well formed for the library, same stack bound, duplication as the Haskell module's */
  int n1 = 0, r1 = 0, need_a = 0, need_d = 0;
  if (rt_rebuild_bvh(&d, NULL, 0, &n1, &r1)) return fail("rt_rebuild_bvh(flattened)");
  if (rt_tree_stack_need(a.nodes, a.n_nodes, a.world_root, &need_a) ||
      rt_tree_stack_need(d.nodes, d.n_nodes, d.world_root, &need_d))
    return fail("rt_tree_stack_need");
  if (need_a != need_d) {
    fprintf(stderr, "FAIL %s: stack need %d vs %d\n", name, need_a, need_d);
    return 1;
  }
  if (d.n_nodes < a.n_nodes - 1 || d.n_materials < 1) {
    fprintf(stderr, "FAIL %s: flattened %d nodes from %d\n", name, d.n_nodes, a.n_nodes);
    return 1;
  }
  printf("%s: builder %d nodes / %d materials / %d textures -> flattened %d / %d / %d, stack need %d",
         name, a.n_nodes, a.n_materials, a.n_textures, d.n_nodes, d.n_materials, d.n_textures, need_d);

  int rc = 0;
  if (gpu) {
    rt_camera cam;
    if (rt_camera_named(cam_id, W, H, &cam)) return fail("rt_camera_named");
    int ndev = 0;
    if (rt_device_count(&ndev) || ndev < 1) return fail("rt_device_count");
    if (ndev > RT_MAX_DEVICES) ndev = RT_MAX_DEVICES;
    uint64_t* gens = malloc(sizeof(uint64_t) * 2 * (size_t)W);
    gens[0] = g1[0];
    gens[1] = g1[1];
    for (int x = 1; x < W; ++x) rt_rand_gen(1024 + x, gens + 2 * x);
    const size_t px = (size_t)W * H * 3;
    uint8_t *rgb_a = malloc(px), *rgb_d[2] = {malloc(px), malloc(px)}, *rgb_m = malloc(px);
    double* lin_d[2] = {malloc(px * 8), malloc(px * 8)};
    uint64_t *go_a = malloc(sizeof(uint64_t) * 2 * (size_t)W), *go_d = malloc(sizeof(uint64_t) * 2 * (size_t)W);
    for (int tier = 0; tier < 2 && !rc; ++tier) {
      rt_render_params p = {W, H, spp, 50, tier ? RT_RNG_PHILOX : RT_RNG_EXACT, 0, 1024, 16, 0, 1, 0};
      /* which 0: the builder's own descriptor on one device; 1: runRenderAMD / runRenderAMDPhilox
         (rt_create(0), rt_upload_scene of the flattened records, rt_render, rt_destroy); 2 (tier B):
         runRenderAMDPhiloxOn over every visible GPU (rt_create_multi, tile shards gathered with RCCL) */
      for (int which = 0; which < 2 + tier && !rc; ++which) {
        rt_ctx* ctx;
        if (which == 2 ? rt_create_multi(ndev, NULL, &ctx) : rt_create(0, &ctx))
          return fail(which == 2 ? "rt_create_multi" : "rt_create");
        uint8_t* out = which == 0 ? rgb_a : (which == 1 ? rgb_d[tier] : rgb_m);
        if (rt_upload_scene(ctx, which ? &d : &a)) rc = fail("rt_upload_scene");
        else if (rt_render(ctx, &cam, &p, gens, out, which == 1 ? lin_d[tier] : NULL, which == 1 ? go_d : go_a))
          rc = fail("rt_render");
        if (!rc) {
          rt_frame_timing t;
          if (rt_last_frame_timing(ctx, &t) || t.n_devices != (which == 2 ? ndev : 1)) rc = fail("rt_last_frame_timing");
        }
        rt_destroy(ctx);
      }
      if (!rc && memcmp(rgb_a, rgb_d[tier], px)) {
        fprintf(stderr, "FAIL %s: tier %c bytes differ\n", name, tier ? 'B' : 'A');
        rc = 1;
      }
      if (!rc && tier && memcmp(rgb_a, rgb_m, px)) {
        fprintf(stderr, "FAIL %s: tier B bytes differ on %d devices\n", name, ndev);
        rc = 1;
      }
      if (!rc && !tier && memcmp(go_a, go_d, sizeof(uint64_t) * 2 * (size_t)W)) {
        fprintf(stderr, "FAIL %s: tier A end generators differ\n", name);
        rc = 1;
      }
    }
    if (!rc) printf(", GPU tier A + B %dx%dx%d on %d device(s): identical bytes and end generators", W, H, spp, ndev);
    if (!rc && dir && dump(dir, name, &d, W, H, spp, 50, gens, rgb_d[0], lin_d[0], go_a, rgb_d[1], lin_d[1])) {
      fprintf(stderr, "FAIL %s: cannot write %s/%s.bin\n", name, dir, name);
      rc = 1;
    }
    free(gens), free(rgb_a), free(rgb_d[0]), free(rgb_d[1]), free(rgb_m), free(lin_d[0]), free(lin_d[1]), free(go_a),
        free(go_d);
  }
  if (!gpu && dir) { /* "dump" mode (no GPU): the flattened records and the generators, zero outputs */
    const size_t px = (size_t)W * H * 3;
    uint64_t* gens = calloc(2 * (size_t)W, sizeof(uint64_t));
    gens[0] = g1[0];
    gens[1] = g1[1];
    for (int x = 1; x < W; ++x) rt_rand_gen(1024 + x, gens + 2 * x);
    uint8_t* z8 = calloc(px, 1);
    double* zd = calloc(px, sizeof(double));
    if (dump(dir, name, &d, W, H, spp, 50, gens, z8, zd, gens, z8, zd)) {
      fprintf(stderr, "FAIL %s: cannot write %s/%s.bin\n", name, dir, name);
      rc = 1;
    }
    free(gens), free(z8), free(zd);
  }
  printf("\n");
  free(f.nodes), free(f.mats), free(f.texs), free(f.perlins), free(f.images), free(f.pool);
  rt_builder_destroy(b);
  return rc;
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && !strcmp(argv[1], "gpu");
  /* "gpu [dir]" renders (and dumps); "dump dir" only writes the flattened records (CPU) */
  const char* dir = argc > 2 && (gpu || !strcmp(argv[1], "dump")) ? argv[2] : NULL;
  int rc = 0;
  rc |= run(RT_SCENE_CORNELL_BOX, "cornell", RT_CAM_CORNELL, 40, 40, 4, gpu, dir);
  rc |= run(RT_SCENE_NEXT_WEEK_FINAL, "next_week_final", RT_CAM_NEXT_WEEK, 32, 24, 2, gpu, dir);
  rc |= run(RT_SCENE_RANDOM, "random", RT_CAM_RANDOM_SCENE, 40, 24, 2, gpu, dir);
  rc |= run(RT_SCENE_CORNELL_SMOKE, "cornell_smoke", RT_CAM_CORNELL, 32, 32, 2, gpu, dir);
  return rc;
}
