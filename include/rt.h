/*
 * rt.h — C ABI of the MI355X-native path tracer (drop-in for the render path of
 * shaunplee/ray-tracing).
 *
 * The reference has no FFI: its render boundary is the pure Haskell call
 *     runRender :: RenderStaticEnv -> [RandGen] -> [VV.Vector RGB]     (src/Lib.hs:1491)
 * with the environment built by
 *     mkRenderStaticEnv scene camera (w,h) ns maxDepth nThreads        (src/Lib.hs:92-108)
 * and   type Scene = (Hittable world, Hittable lights, Albedo background)  (src/Lib.hs:84).
 * This header replaces that call with plain C: the immutable Haskell `Scene` becomes a
 * flattened `rt_scene_desc` (arrays of POD records), the `Camera` becomes `rt_camera`,
 * `[RandGen]` becomes an array of SplitMix64 (seed, gamma) pairs, and the lazily streamed
 * `[Vector RGB]` becomes a caller-owned H*W*3 byte buffer (top row first, PPM order).
 *
 * Scene construction (Lib.hs constructors, makeBVH, makePerlin, Scenes.hs builders and
 * cameras) is exported too (rt_builder_*, rt_scene_named, rt_camera_*), so a host that
 * used the reference's Scenes.hs API finds the same surface here.
 *
 * Conventions: every function returns 0 on success and a negative RT_E* code on error;
 * the message is available from rt_last_error() (thread-local). No torch / C++ types.
 */
#ifndef RT_H
#define RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

/* ------------------------------------------------------------------ error codes */
#define RT_OK 0
#define RT_E_INVALID (-1)   /* bad argument / malformed scene                       */
#define RT_E_HIP (-2)       /* HIP runtime error                                     */
#define RT_E_NOMEM (-3)     /* allocation failure                                    */
#define RT_E_UNSUPPORTED (-4)/* scene uses a construct the device path does not take */
#define RT_E_STATE (-5)     /* call order (e.g. render before upload)                */
#define RT_E_COMM (-6)      /* RCCL error (multi-device contexts)                    */

/* ------------------------------------------------------------------ scene records */

/* Flattened `Hittable` (src/Lib.hs:521-585). One 64-byte record per constructor. */
enum rt_node_type {
    RT_NODE_BVH = 0,             /* BVHNode left right box size        (Lib.hs:552-560) */
    RT_NODE_SPHERE = 1,          /* Sphere center radius material      (Lib.hs:522-528) */
    RT_NODE_MOVING_SPHERE = 2,   /* MovingSphere c0 c1 t0 t1 dur r mat (Lib.hs:529-543) */
    RT_NODE_RECT_XY = 3,         /* Rect (XYRect x0 x1 y0 y1 k mat)    (Lib.hs:608-620) */
    RT_NODE_RECT_XZ = 4,         /* Rect (XZRect x0 x1 z0 z1 k mat)    (Lib.hs:621-633) */
    RT_NODE_RECT_YZ = 5,         /* Rect (YZRect y0 y1 z0 z1 k mat)    (Lib.hs:634-646) */
    RT_NODE_CUBOID = 6,          /* Cuboid min max [6 rects]           (Lib.hs:545-551,594-605) */
    RT_NODE_TRANSLATE = 7,       /* Translate offset child             (Lib.hs:561-565) */
    RT_NODE_ROTATE = 8,          /* Rotate axis sin cos box child      (Lib.hs:566-576) */
    RT_NODE_CONSTANT_MEDIUM = 9, /* ConstantMedium (-1/density) mat boundary (Lib.hs:577-583) */
    RT_NODE_UNHITTABLE = 10,     /* Unhittable                         (Lib.hs:584) */
    RT_NODE_EXT = 11             /* payload continuation of the previous record (never a child) */
};

/*
 * Field use per type (f = 6 doubles, a/b/c = int32):
 *   BVH            f = box min xyz, box max xyz;   a = left, b = right
 *   SPHERE         f[0..2] = center, f[3] = radius; a = material
 *   MOVING_SPHERE  f[0..2] = center0, f[3..5] = center1; a = material;
 *                  the next record (type EXT) holds f[0]=time0, f[1]=time1, f[2]=duration, f[3]=radius
 *   RECT_XY/XZ/YZ  f[0..4] = (i0, i1, j0, j1, k) in the constructor's argument order; a = material
 *   CUBOID         f = min xyz, max xyz; a = material (the six rects are implied, Lib.hs:599-604)
 *   TRANSLATE      f[0..2] = offset; a = child
 *   ROTATE         f[0] = sin theta, f[1] = cos theta; a = child; b = axis (0 X, 1 Y, 2 Z)
 *   CONSTANT_MEDIUM f[0] = negative inverse density; a = boundary; b = phase material; f[1] = 0, or the
 *                  occurrence key + 1 of an unfolded medium record (rt_rebuild_bvh output; see
 *                  RT_RNG_PHILOX: the upload keys every medium occurrence of the caller's tree)
 * For every type c = htblSize of the node (Lib.hs:662-671): BVH its size, Translate/Rotate
 * the size of the child, Unhittable 0, everything else 1. (World-only BVH nodes appended by the
 * device-side rebuild carry 0x40000000 | split axis instead; they never occur in a lights tree.)
 */
#define RT_BVH_ORDERED 0x40000000 /* rebuilt world BVH node: c = this flag | split axis */
#define RT_BVH_MEDIA_FIRST 0x10000000 /* with RT_BVH_ORDERED: a rebuilt world's top node whose left child
                                         is a medium occurrence (not inside an instance frame), entered
                                         before the right child (the rest of the world) whatever the ray
                                         direction: its candidate bounds the walk from the start */

typedef struct rt_node {
    double f[6];
    int32_t type;
    int32_t a;
    int32_t b;
    int32_t c;
} rt_node; /* 64 bytes */

/* `Material` (src/Lib.hs:339-345). */
enum rt_material_type {
    RT_MAT_LAMBERTIAN = 0,
    RT_MAT_METAL = 1,
    RT_MAT_DIELECTRIC = 2,
    RT_MAT_DIFFUSE_LIGHT = 3,
    RT_MAT_ISOTROPIC = 4
};

typedef struct rt_material {
    int32_t type;
    int32_t texture; /* texture id (Lambertian, Metal, DiffuseLight, Isotropic) */
    double param;    /* Metal: fuzz; Dielectric: refractive index */
} rt_material;       /* 16 bytes */

/* `Texture` (src/Lib.hs:394-419). */
enum rt_texture_type {
    RT_TEX_CONSTANT = 0, /* f[0..2] = albedo */
    RT_TEX_CHECKER = 1,  /* a = odd texture, b = even texture */
    RT_TEX_PERLIN = 2,   /* a = perlin table id, f[0] = scale */
    RT_TEX_IMAGE = 3     /* a = image id (-1 = Nothing), b = width, c = height */
};

typedef struct rt_texture {
    int32_t type;
    int32_t a;
    int32_t b;
    int32_t c;
    double f[4];
} rt_texture; /* 48 bytes */

/* Perlin tables of `makePerlin` (src/Lib.hs:424-439). */
typedef struct rt_perlin {
    double ranvec[256][3];
    int32_t perm_x[256];
    int32_t perm_y[256];
    int32_t perm_z[256];
} rt_perlin; /* 9216 bytes */

/* RGB8 raster (the JuicyPixels `Image PixelRGB8` of src/Lib.hs:384-389), row-major, row 0 = top. */
typedef struct rt_image {
    int64_t offset; /* byte offset into rt_scene_desc.image_pool */
    int32_t width;
    int32_t height;
} rt_image;

typedef struct rt_scene_desc {
    const rt_node* nodes;
    int32_t n_nodes;
    int32_t world_root;  /* node id of the world Hittable */
    int32_t lights_root; /* node id of the lights Hittable; -1 = Unhittable */
    int32_t n_materials;
    const rt_material* materials;
    const rt_texture* textures;
    int32_t n_textures;
    int32_t n_perlins;
    const rt_perlin* perlins;
    const rt_image* images;
    int32_t n_images;
    int32_t _pad;
    const uint8_t* image_pool;
    int64_t image_pool_bytes;
    double background[3]; /* Albedo background (src/Lib.hs:84) */
} rt_scene_desc;

/* `Camera` (src/Lib.hs:1230-1251), as computed by newCamera (src/Lib.hs:1280-1295). */
typedef struct rt_camera {
    double origin[3];
    double llc[3];
    double horiz[3];
    double vert[3];
    double u[3];
    double v[3];
    double w[3];
    double lens_radius;
    double t0;
    double t1;
} rt_camera;

/* ------------------------------------------------------------------ render parameters */

/*
 * RNG stream layouts.
 *  RT_RNG_EXACT  (tier A): the reference's layout — one SplitMix64 generator per image
 *                column, threaded top row to bottom row, through every sample and bounce
 *                (src/Lib.hs:1491-1523, 1352-1371). Only width-parallel.
 *  RT_RNG_PHILOX (tier B): one Philox4x32-10 stream per (pixel, sample), key = seed,
 *                counter = {draw_pair, sample, pixel_id, 0}; each 128-bit block yields two
 *                64-bit words, converted exactly as random-1.2.0 `random :: Double`.
 *                A pixel's samples are summed in fixed chunks: chunk k holds samples
 *                [k*CH, min(spp, (k+1)*CH)) with CH = rt_sample_chunk(width*height, spp);
 *                each chunk is summed in sample order from 0, the chunk sums in chunk order
 *                from 0. (The chunks are the device's work-items; a definition fixed by
 *                (width, height, spp) keeps the image independent of scheduling and shard
 *                count.) Embarrassingly parallel.
 *                ConstantMedium (src/Lib.hs:1053-1080) in tier B: its draw is not the stream's next
 *                but the first word of the block at counter {stream words consumed so far, sample,
 *                pixel_id, 2^31 | key}, key = the occurrence's preorder rank among the medium
 *                occurrences of the caller's world tree (BVH left child first, into Translate/Rotate;
 *                one occurrence per path) or f[1] - 1 when set; and its candidate hit is computed over
 *                the boundary's whole inside, then accepted like a leaf's at t <= the bound. The
 *                closest hit is then the least t over every leaf in any walk order (exact ties are
 *                resolved in the reference's order), so media worlds walk re-bounded trees too.
 *                Tier A keeps the reference's own medium: the stream's next draw, under the walk's bound.
 */
#define RT_RNG_EXACT 0
#define RT_RNG_PHILOX 1
#define RT_CHUNK_SAMPLES 8      /* samples per chunk, at least (short chunks: a short tail per shard) */
#define RT_CHUNK_MAX 128         /* ...but at most this many chunks per pixel (bounds the chunk sums) */
#define RT_CHUNK_ITEMS (1 << 20) /* ...fewer samples when the frame would have fewer work-items */
/* CH = min(spp, max(8, ceil(spp / 128)), max(1, ceil(pixels * spp / 2^20))): 8-sample chunks
   (C2, C3/C4 at 1000 spp), longer ones for higher spp (C5 2000 spp: 16) so that a pixel has at most
   128, and shorter ones for small frames (config 1: 200x100x10 -> 1) so that they fill the device.
   (Round 4: 128, was 64 — 16-sample chunks left C4 a long per-shard tail at 8 GPUs.) */
static inline int rt_sample_chunk(int64_t pixels, int spp) {
  const int64_t fill = (pixels * (int64_t)spp + RT_CHUNK_ITEMS - 1) / RT_CHUNK_ITEMS;
  int ch = (spp + RT_CHUNK_MAX - 1) / RT_CHUNK_MAX;
  if (ch < RT_CHUNK_SAMPLES) ch = RT_CHUNK_SAMPLES;
  if (ch > spp) ch = spp;
  if (fill < ch) ch = (int)fill;
  return ch > 0 ? ch : 1;
}

/* Flags. */
#define RT_FLAG_NAN_CULL 1u /* tier B only: stop tracing a pixel once its sum is NaN
                               (its output byte is then fixed at 0, src/Lib.hs:287-288).
                               Output-identical; off by default. */
#define RT_FLAG_REFERENCE_CULL 2u /* cull BVH boxes with the reference's per-axis test only
                               (src/Lib.hs:798-814). Default: that test AND the joint slab test,
                               which only prunes boxes that cannot hold a hit. A world
                               with a finite BVH box coordinate beyond 2^100 always takes this flag. */
#define RT_FLAG_NAN_ZERO 4u /* tiers A and B, parity diagnostic (NOT the reference's semantics): a sample
                               contribution channel that is NaN is added as 0, so that the finite
                               part of every sample reaches the average. The reference's Lambertian
                               light-mixture quirk makes most pixels of the bench frames NaN (C2 mid
                               rows, all of C4 at 1000 spp); with this flag the same launches carry
                               every sample's finite colour to a comparable output (and tier A's and
                               tier B's finite parts can be compared as distributions). */
#define RT_FLAG_SHARED_LIBM 8u /* tier A only, parity aid: sin, cos, log, atan, asin (and x ** 5) from the
                               portable include/rt_libm.h instead of the device's OCML, the functions the
                               oracle evaluates in the same mode. A column's tier-A stream is one serial
                               chain, so a last-bit difference between two libms that flips any later branch
                               changes the rest of the column; with one libm on both sides the streams are
                               compared bit for bit on every scene. */

typedef struct rt_render_params {
    int32_t width;
    int32_t height;
    int32_t spp;       /* numSamples */
    int32_t max_depth; /* maxDepth */
    int32_t rng_mode;  /* RT_RNG_EXACT | RT_RNG_PHILOX */
    uint32_t flags;
    uint64_t seed;       /* tier B Philox key */
    int32_t tile;        /* tile edge in pixels for sharding: a multiple of 8 in [8, 256] (0 = default 8) */
    int32_t shard_rank;  /* this shard (0-based) */
    int32_t shard_count; /* number of shards (GPUs); tiles are dealt round-robin */
    int32_t _pad;
} rt_render_params;

/* ------------------------------------------------------------------ version / errors */
int rt_abi_version(void);
const char* rt_last_error(void);

/* ------------------------------------------------------------------ RNG (src/Random.hs) */
/* randGen s = mkStdGen s  (src/Random.hs:20-21): writes (seed, gamma). */
void rt_rand_gen(int64_t s, uint64_t out_gen[2]);
/* randomDouble (src/Random.hs:23-25): one draw, advances gen in place. */
double rt_random_double(uint64_t gen[2]);

/* ------------------------------------------------------------------ scene construction */
/* A builder owns the RandGen threaded through scene construction (makeBVH / makePerlin
 * draw from it, src/Lib.hs:941-943, 424-439) and the growing record arrays. Object ids
 * returned by the constructors are node ids. */
typedef struct rt_builder rt_builder;

int rt_builder_create(const uint64_t gen[2], rt_builder** out);
void rt_builder_destroy(rt_builder* b);
/* Current generator state (the `g1` handed back by the Scenes.hs builders). */
void rt_builder_gen(const rt_builder* b, uint64_t out_gen[2]);

int rt_tex_constant(rt_builder* b, double r, double g, double bl);
int rt_tex_checker(rt_builder* b, int odd_tex, int even_tex);
int rt_tex_perlin(rt_builder* b, double scale); /* makePerlin: consumes 768 + 3*255 draws */
int rt_tex_image(rt_builder* b, const uint8_t* rgb, int width, int height); /* rgb NULL = Nothing */

int rt_mat_lambertian(rt_builder* b, int tex);
int rt_mat_metal(rt_builder* b, int tex, double fuzz);
int rt_mat_dielectric(rt_builder* b, double ref_idx);
int rt_mat_diffuse_light(rt_builder* b, int tex);
int rt_mat_isotropic(rt_builder* b, int tex);

int rt_obj_sphere(rt_builder* b, const double center[3], double radius, int mat);
int rt_obj_moving_sphere(rt_builder* b, const double c0[3], const double c1[3], double t0, double t1,
                         double radius, int mat);
/* plane: 0 = XYPlane, 1 = XZPlane, 2 = YZPlane (src/Lib.hs:649-660) */
int rt_obj_rect(rt_builder* b, int plane, double a0, double a1, double b0, double b1, double k, int mat);
int rt_obj_cuboid(rt_builder* b, const double pmin[3], const double pmax[3], int mat);
int rt_obj_translate(rt_builder* b, const double offset[3], int child);
int rt_obj_rotate(rt_builder* b, int axis, double angle_deg, int child);
int rt_obj_constant_medium(rt_builder* b, double density, int tex, int boundary);
int rt_obj_unhittable(rt_builder* b);
/* makeBVH mtime items (src/Lib.hs:941-961); has_time = 0 for Nothing. Consumes draws. */
int rt_obj_bvh(rt_builder* b, const int* items, int n_items, int has_time, double t0, double t1);

/* Seal the scene: world root, lights root (-1 = Unhittable), background. The descriptor
 * points into builder-owned memory and stays valid until the builder is destroyed. */
int rt_builder_finish(rt_builder* b, int world, int lights, const double background[3],
                      rt_scene_desc* out_desc);

/* Named scenes of src/Scenes.hs (ids below). `earth` = ImageTexture raster or NULL (Nothing).
 * The builder must be fresh; its generator is threaded as in the reference. */
enum rt_scene_id {
    RT_SCENE_CORNELL_BOX = 0,       /* makeCornellBoxScene        Scenes.hs:32-73   */
    RT_SCENE_CORNELL_SMOKE = 1,     /* makeCornellSmokeBoxScene   Scenes.hs:75-118  */
    RT_SCENE_SIMPLE_LIGHT = 2,      /* makeSimpleLightScene       Scenes.hs:133-155 */
    RT_SCENE_EARTH = 3,             /* makeEarthScene             Scenes.hs:167-179 */
    RT_SCENE_TWO_PERLIN_SPHERES = 4,/* makeTwoPerlinSpheresScene  Scenes.hs:194-211 */
    RT_SCENE_TWO_SPHERES = 5,       /* makeTwoSpheresScene        Scenes.hs:213-237 */
    RT_SCENE_RANDOM_BOOK_ONE = 6,   /* makeRandomSceneBookOne     Scenes.hs:253-317 */
    RT_SCENE_RANDOM = 7,            /* makeRandomScene            Scenes.hs:321-399 */
    RT_SCENE_NEXT_WEEK_FINAL = 8,   /* makeNextWeekFinalScene     Scenes.hs:414-466 */
    RT_SCENE_THREE_SPHERES = 9,     /* config 1: ground + s1..s3 of Scenes.hs:263-279, BVH (0,1) */
    RT_SCENE_STRESS_SPHERES = 10    /* config 5: `param` random spheres + ground, BVH (0,1) */
};
int rt_scene_named(rt_builder* b, int scene_id, double t0, double t1, const uint8_t* earth_rgb,
                   int earth_w, int earth_h, int64_t param, rt_scene_desc* out_desc);

/* newCamera lookfrom lookat vup vfov aspect aperture focusDist t0 t1 (src/Lib.hs:1269-1295). */
void rt_camera_new(const double lookfrom[3], const double lookat[3], const double vup[3], double vfov,
                   double aspect, double aperture, double focus_dist, double t0, double t1,
                   rt_camera* out);
enum rt_camera_id {
    RT_CAM_CORNELL = 0,      /* cornellCamera             Scenes.hs:120-131 */
    RT_CAM_TWO_SPHERES = 1,  /* twoSpheresSceneCamera     Scenes.hs:181-192 */
    RT_CAM_RANDOM_SCENE = 2, /* randomSceneCamera         Scenes.hs:239-250 */
    RT_CAM_NEXT_WEEK = 3     /* nextWeekFinalSceneCamera  Scenes.hs:401-412 */
};
int rt_camera_named(int cam_id, int width, int height, rt_camera* out);

/* P3 PPM text exactly as app/Main.hs:59-61 + printRow/showRow (src/Lib.hs:299-305).
 * Writes at most cap bytes; *out_len = bytes required. */
int rt_write_ppm(const uint8_t* rgb, int width, int height, char* buf, size_t cap, size_t* out_len);
/* Float dump of the per-pixel averages (rt_render's out_linear, H*W*3 doubles, top row first) as PFM:
 * "PF\n<W> <H>\n-1.0\n" + little-endian float32 RGB, bottom row first (the PFM order); f64 != 0
 * writes doubles under the header "PF64" instead (lossless). Same buffer protocol as rt_write_ppm. */
int rt_write_pfm(const double* linear, int width, int height, int f64, char* buf, size_t cap, size_t* out_len);

/* ------------------------------------------------------------------ device path */
typedef struct rt_ctx rt_ctx;

int rt_device_count(int* out);
/* Bind one HIP device (one process per GPU). */
int rt_create(int device, rt_ctx** out);
/*
 * One context over n_devices GPUs, driven from one host thread ("rt_create(num_gpus)":
 * the ctx owns the devices and an RCCL communicator over them). devices: n_devices distinct HIP device
 * ids, or NULL for 0..n_devices-1; at most RT_MAX_DEVICES. RCCL ranks follow the list order.
 *   rt_upload_scene[_ex]: validates and prepares the scene once, then copies it to every device.
 *   rt_render, tier B: the image's tiles are dealt round-robin over the devices (shard r = the r-th
 *     device, the rt_render_shard_async layout with shard_count = n_devices), each device renders its
 *     slab on its own stream, the slabs are gathered to the first device with RCCL (ncclGather over
 *     xGMI, grouped over the devices' communicators), which assembles the image and copies it to the
 *     host. The bytes equal a one-device rt_render of the same params (tier B is shard-invariant).
 *   rt_render, tier A: the reference's per-column streams are one serial chain per column, so tier A
 *     does not shard: it renders on the first device.
 * Every other call on a multi-device ctx (the *_async building blocks, debug entries, counting
 * renders) acts on its first device. This replaces the reference's only parallelism, the row sparks
 * of runRender (src/Lib.hs:1519-1520), as called from app/Main.hs:50-58.
 */
#define RT_MAX_DEVICES 16
int rt_create_multi(int n_devices, const int* devices, rt_ctx** out);
/* Devices of a ctx: *out_n = count; out_devices (may be NULL) receives up to `cap` device ids. */
int rt_ctx_devices(const rt_ctx* ctx, int* out_n, int* out_devices, int cap);
/* Timing of the last rt_render on a ctx (HIP events on each device's launch stream), ms:
 * kernel_ms[r] = device r's render launches (chunk batches included), gather_ms = from the first
 * device's render end to the end of the RCCL gather on its stream (includes waiting for the slowest
 * device), assemble_ms = the assemble kernel, frame_ms = first launch to assembled image (before the
 * device-to-host copy). n_devices = 1 and gather_ms = 0 on a one-device ctx. device_allocs = device
 * allocations (hipMalloc) the call made over all the ctx's devices: the ctx keeps its frame buffers (slabs,
 * gathered slabs, image, chunk sums) and grows them on demand, so a repeated frame of one size makes none. */
typedef struct rt_frame_timing {
    int32_t n_devices;
    int32_t device_allocs;
    double kernel_ms[RT_MAX_DEVICES];
    double gather_ms;
    double assemble_ms;
    double frame_ms;
} rt_frame_timing;
int rt_last_frame_timing(rt_ctx* ctx, rt_frame_timing* out);
void rt_destroy(rt_ctx* ctx);
/* Copy a scene to device memory (caller-owned desc; arrays are copied). Validates it.
 * Every medium occurrence of the world tree becomes its own keyed record (RT_RNG_PHILOX above), and by
 * default the world tree is re-bounded by a binned-SAH BVH over the same leaves, media and instance
 * frames included (the trees inside frames re-bounded in their own coordinates), for traversal (closest
 * hits are tree-independent except for exact ties, which are redone on the caller's tree; DESIGN.md
 * §3); the lights tree is always the caller's. */
int rt_upload_scene(rt_ctx* ctx, const rt_scene_desc* desc);
#define RT_UPLOAD_REFERENCE_BVH 1u /* traverse the caller's (makeBVH's) world tree as is */
int rt_upload_scene_ex(rt_ctx* ctx, const rt_scene_desc* desc, uint32_t flags);
/* The rebuild rt_upload_scene applies, on the host: the node array with the new world BVH
 * appended (out_nodes NULL: size query) and the new world root (== the old one if ineligible). */
int rt_rebuild_bvh(const rt_scene_desc* desc, rt_node* out_nodes, int capacity, int* out_n, int* out_root);
/* The 4-wide collapse the device walk uses (rt_wide.h records, 128 B each) of the binary tree at
 * `root` of a node array (e.g. rt_rebuild_bvh's output): out NULL = size query. out_stack_need
 * = the walk's stack bound (entries). RT_E_UNSUPPORTED when the root is not a BVH node. */
int rt_wide_bvh(const rt_node* nodes, int n_nodes, int root, void* out, int capacity, int* out_n,
                int* out_stack_need);
/* The 64-byte quantised form (rt_qnode, rt_wide.h) of n 4-wide records (rt_wide_bvh output) that the
 * kernels reading the tree from global memory walk: out holds n records. RT_E_UNSUPPORTED when a node's
 * boxes cannot be put on an fp32 grid (planes beyond fp32 range). */
int rt_quantize_wide(const void* wnodes, int n, void* out);
/* The host half of rt_upload_scene, with no device: validates `desc` exactly as the upload does
 * (same error codes and rt_last_error text; RT_UPLOAD_REFERENCE_BVH as for the upload) and describes
 * the device copy it would upload. Malformed descriptors can be checked on a machine without a GPU. */
typedef struct rt_scene_info {
    int32_t n_nodes;         /* device node records (the caller's + the rebuilt tree) */
    int32_t n_wide_nodes;    /* 4-wide nodes (the world's, or the mixed walk's subtrees'; 0 = none) */
    int32_t n_leaves;        /* their leaf-table records */
    int32_t world_root;      /* the walked world tree's root (the rebuilt one's when rebuilt) */
    int32_t stack_need;      /* stack entries of the binary / mixed walk */
    int32_t wide_stack_need; /* stack entries of the 4-wide walk */
    uint32_t features;       /* scene feature bits (F_* in ray-tracing_amd/csrc/rt_layout.h) */
    uint32_t variant;        /* the render-kernel variant chosen for them */
    int32_t rebuilt_bvh;     /* the world tree was rebuilt (SAH, or skeleton + re-bounded subtrees) */
    int32_t mixed_wide;      /* media / frame world with 4-wide trees under its skeleton */
    int32_t replace_ok;      /* frames nest <= 4 deep: the ray-replacement loop applies */
    int32_t ref_walk;        /* media or frames: walked in the reference's order */
} rt_scene_info;
int rt_prepare_scene(const rt_scene_desc* desc, uint32_t flags, rt_scene_info* out);
/* Stack entries the binary walk over the tree at `root` needs (the bound rt_upload_scene sizes
 * the LDS stacks with): left-first for the caller's nodes, either child first for rebuilt
 * (RT_BVH_ORDERED) nodes, one entry per open instance frame. */
int rt_tree_stack_need(const rt_node* nodes, int n_nodes, int root, int* out_need);

/*
 * Blocking full-image render (replaces runRender, src/Lib.hs:1491).
 *   col_gens     tier A: 2*width words (seed, gamma) per column, column 0 first
 *                (app/Main.hs:47-49); ignored in tier B.
 *   out_rgb8     H*W*3 bytes, top row first (pixelPositions, src/Lib.hs:1488-1489).
 *   out_linear   optional H*W*3 doubles: the per-pixel average before albedoToColor.
 *   out_col_gens optional (tier A): generators after the last row, 2*width words.
 * shard_rank/shard_count in params are ignored (whole image).
 */
int rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, const uint64_t* col_gens,
              uint8_t* out_rgb8, double* out_linear, uint64_t* out_col_gens);

/*
 * Multi-GPU building blocks (tier B only). The image is cut into tile x tile squares,
 * numbered row-major from the top-left; shard r owns tiles r, r+N, r+2N, ... and writes
 * them into a "slab": tiles_per_shard * tile * tile pixels, tile-major. Every shard's slab
 * has the same size (padded), so slabs can be all-gathered as-is.
 */
int rt_shard_geometry(const rt_render_params* p, int64_t* tiles_total, int64_t* tiles_per_shard,
                      int64_t* slab_pixels);
/* Render this shard into device buffers on `stream` (hipStream_t, NULL = default).
 * d_slab_rgb8: slab_pixels*3 bytes; d_slab_linear: slab_pixels*3 doubles or NULL.
 * Asynchronous: stream-ordered, returns after the launches are queued. */
int rt_render_shard_async(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p,
                          uint8_t* d_slab_rgb8, double* d_slab_linear, void* stream);
/* Scatter shard_count gathered slabs (concatenated, rank-major) into a H*W*3 device image. */
int rt_assemble_async(rt_ctx* ctx, const rt_render_params* p, const uint8_t* d_slabs_rgb8,
                      uint8_t* d_image_rgb8, void* stream);
/* Same for the optional linear (double) slabs. */
int rt_assemble_linear_async(rt_ctx* ctx, const rt_render_params* p, const double* d_slabs_linear,
                             double* d_image_linear, void* stream);

/*
 * Counting build of the tier-B render (same output, slower): device-measured work for the
 * roofline. out_work[0..7] = {segments traced, BVH box tests, leaf primitive tests,
 * instance/medium tests, light-pdf evaluations, Philox blocks, samples, 4-wide node visits}
 * for this shard; out_work[8..10] = wave time (s_memtime ticks, summed over waves) spent acquiring work and
 * starting samples / traversing / shading; out_work[11..13] (ray-replacement loop only) = live-lane
 * slots of 4-wide node steps, of leaf steps and of outer iterations (lane utilisation = work / slots);
 * out_work[14] = leaf tests that found a hit, out_work[15] = walks redone for an exact tie (worlds
 * with media or frames: samples redone) (replacement loop).
 */
int rt_render_work(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, uint64_t out_work[16]);

/* The same counting render, plus a profile of the binary / mixed walk's steps (replacement loop over
 * worlds with media or frames, and Cornell-like worlds): out_prof[m] = wave time (s_memtime ticks)
 * of the steps whose lanes were at the set m of node kinds, out_prof[32 + m] = their count; kinds:
 * 1 BVH box, 2 4-wide node, 4 leaf (primitive or chain), 8 ConstantMedium, 16 instance frame. */
int rt_render_step_profile(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, uint64_t out_work[16],
                           uint64_t out_prof[64]);

/* Timing of the last render launch on this ctx (HIP events on the launch stream), ms. */
int rt_last_kernel_ms(rt_ctx* ctx, double* out_ms);

/* Which kernel the last tier-B render launch on this ctx ran (kernel selection is per scene and
 * frame: DESIGN.md §3): feature variant (rt_trace.h F_* bits), loop (0 one sample per lane walk,
 * 1 ray replacement over the binary tree, 2 over the 4-wide tree), LDS-staged scene or global
 * memory, leaf table in LDS, waves per SIMD the instantiation targets, grid and block size, dynamic
 * LDS bytes per workgroup, work-items and samples per work-item. */
typedef struct rt_launch_info {
    uint32_t variant;
    int32_t loop;
    int32_t lds_staged;
    int32_t leaf_lds;
    int32_t waves;
    int32_t grid;
    int32_t block;
    int32_t dyn_lds_bytes;
    int64_t work_items;
    int32_t chunk;
    int32_t wide_nodes;  /* 4-wide nodes the launched walk uses: the 4-wide world tree (loop 2), or the
                            mixed walk's trees over re-bounded subtrees (loop 1, media / frame worlds) */
    int32_t chunk_batches; /* launches the frame's chunks were split into (chunk sums bounded per launch) */
    int32_t _pad;
} rt_launch_info;
int rt_last_launch(rt_ctx* ctx, rt_launch_info* out);

/*
 * Debug / parity entry: closest hit of n world rays (7 doubles each: origin, direction, time)
 * in [tmin, tmax]. out: 12 doubles per ray: hit(0/1), t, p xyz, normal xyz, u, v, front_face,
 * material. Media draws use tier-B stream (seed, pixel_id = ray index, sample 0).
 * flags: RT_FLAG_REFERENCE_CULL as for rendering, plus one walk selector: none = the recursive
 * walk (media and frames allowed); RT_DEBUG_RESUMABLE = the render loop's resumable binary
 * walk; RT_DEBUG_WIDE = the resumable walk over the 4-wide fp32-box tree. The last two need a
 * world without ConstantMedium and instance frames (else RT_E_UNSUPPORTED).
 */
#define RT_DEBUG_RESUMABLE 4u
#define RT_DEBUG_WIDE 8u
#define RT_DEBUG_QNODE 16u /* the 4-wide walk over the quantised tree (rt_qnode) and sphere quadruples that the
                              global-memory kernels of spheres-only worlds take */
int rt_debug_closest_hits(rt_ctx* ctx, const double* rays, int n, double tmin, double tmax,
                          uint64_t seed, uint32_t flags, double* out);

/*
 * Debug / parity entry: single hot-path functions on the device (golden vectors per function,
 * tests/golden/make_function_goldens.py). Record i draws from its own tier-B Philox stream
 * (key = seed, pid = i, sample 0). Layouts (doubles per record), in -> out:
 *   RT_PROBE_SCATTER      scatter (src/Lib.hs:822-865; emitted 880-885 for DiffuseLight):
 *                         ray o3 d3 tm, hit t p3 n3 u v front_face material (18) ->
 *                         scattered (0/1), ray o3 d3 tm, att3 (the emission when not scattered),
 *                         pdf, specular, Philox words consumed (14)
 *   RT_PROBE_HTBL_RANDOM  htblRandom on the lights tree (src/Lib.hs:707-724): origin3 -> dir3, words
 *   RT_PROBE_HTBL_PDF     htblPdfValue on the lights tree (src/Lib.hs:673-705): origin3, v3 -> pdf, words
 *   RT_PROBE_TEXTURE      textureValue (src/Lib.hs:496-513): texture id, u, v, p3 -> albedo3
 *   RT_PROBE_GET_RAY      getRay with `cam` (src/Lib.hs:1253-1267): s, t -> ray o3 d3 tm, words
 *   RT_PROBE_BOX          the BVH box test: box min3 max3, ray o3 d3, t_min, t_max (14) -> the default test
 *                         as the walks run it (division-free, rt_trace.h box_hit), the same test with
 *                         divisions, the reference's per-axis boxRayIntersect (src/Lib.hs:798-814) (3; 1 = hit)
 */
/*
 * Debug / parity entry: tier A (RT_RNG_EXACT) over the whole frame, with column `col`'s path segments
 * recorded: 10 doubles per segment {row, sample (in the order rendered), seg (or -(seg + 1) where the
 * path ends), the scattered ray's origin xyz and direction xyz (at the end: the segment's own ray), the
 * column generator's seed after the segment (the uint64 bits)}. *out_n = segments recorded (at most
 * cap). The oracle's oracle_exact_trace records the same, so the first differing record localises a
 * tier-A divergence.
 */
int rt_debug_exact_trace(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, const uint64_t* col_gens,
                         int col, double* out, int cap, int* out_n);

#define RT_PROBE_SCATTER 0
#define RT_PROBE_HTBL_RANDOM 1
#define RT_PROBE_HTBL_PDF 2
#define RT_PROBE_TEXTURE 3
#define RT_PROBE_GET_RAY 4
#define RT_PROBE_BOX 5
int rt_debug_probe(rt_ctx* ctx, const rt_camera* cam, int op, const double* in, int n, uint64_t seed, double* out);

/*
 * Debug / numerics probe: out[i] = op(x[i], y[i]) evaluated on the device.
 * ops: 0 x/y (IEEE), 1 div_exact(x, y) (reciprocal + Markstein), 2 sqrt x, 3 sin x, 4 cos x,
 * 5 atan x, 6 asin x, 7 log x, 8 pow(x, y), 9 GHC atan2(x, y), 10 tan x, 11 the render path's
 * x ** 5 (schlick; double-double, correctly rounded); 12-16 include/rt_libm.h's sin, cos, atan, asin,
 * log x and 17 GHC atan2(x, y) over them (RT_FLAG_SHARED_LIBM).
 */
int rt_debug_math(rt_ctx* ctx, int op, const double* x, const double* y, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* RT_H */
