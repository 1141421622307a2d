/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, called by, or shipped with the
 * product path (ray-tracing_amd/). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it, and only as the checker / CPU baseline.
 *
 * A CPU restatement, in plain C (fp64, glibc libm, built with -ffp-contract=off and no
 * fast-math, as GHC's NCG emits no FMA), of the render path of shaunplee/ray-tracing:
 * runRender -> renderPos -> sampleColor -> getRay -> rayColor -> hit/scatter/pdf/texture.
 * It follows the Haskell recursively and in the same evaluation order; every function cites
 * the src/Lib.hs lines it restates. Scenes arrive flattened (include/rt.h rt_scene_desc);
 * scene construction is restated separately (oracle/scenes_ref.py).
 *
 * Pinning status (see DESIGN.md "Parity"): the reference is Haskell and cannot be built here
 * (no GHC/stack/cabal) and has no tests/golden vectors. The RNG restatement of
 * splitmix-0.1 / random-1.2.0 (stack.yaml:42-44) is UNPINNED against GHC; parity with the
 * reference image is pinned only STATISTICALLY, against the reference-rendered
 * cornellBox1000.png (block means; tests/golden/cornell1000_blocks.npz).
 *
 * libm: glibc's sin/cos/log/atan/asin/pow by default (the reference's). With RT_FLAG_SHARED_LIBM in
 * the render params (tier A parity aid), the portable include/rt_libm.h functions instead, which the
 * device evaluates bit-identically in that mode (a tier-A column is one serial stream, so one ulp of
 * libm difference that later flips a branch changes the rest of the column). The mode is a process-wide
 * switch set for the duration of oracle_render_rows (renders are not run concurrently by the tests).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/rt.h"
#include "../include/rt_libm.h"

#define EPSILON 0.0001 /* src/Lib.hs:76-77 */
static const double PI = 3.141592653589793; /* GHC `pi` for Double */

/* ------------------------------------------------------------------ libm (glibc, or rt_libm.h) */
static int g_shared_libm = 0;
static inline double o_sin(double x) { return g_shared_libm ? rtlm_sin(x) : sin(x); }
static inline double o_cos(double x) { return g_shared_libm ? rtlm_cos(x) : cos(x); }
static inline double o_log(double x) { return g_shared_libm ? rtlm_log(x) : log(x); }
static inline double o_atan(double x) { return g_shared_libm ? rtlm_atan(x) : atan(x); }
static inline double o_asin(double x) { return g_shared_libm ? rtlm_asin(x) : asin(x); }
static inline double o_pow5(double x) { return g_shared_libm ? rtlm_pow5(x) : pow(x, 5); }

/* ------------------------------------------------------------------ Vec3 (src/Lib.hs:200-261) */
typedef struct { double x, y, z; } V3;
static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }   /* |+| */
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }   /* |-| */
static inline V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }   /* |*| */
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 scale(double k, V3 a) { return v3(a.x * k, a.y * k, a.z * k); }    /* Lib.hs:250-251 */
static inline V3 divide(V3 a, double k) { return v3(a.x / k, a.y / k, a.z / k); }   /* Lib.hs:253-254 */
static inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  /* Lib.hs:256-257 */
static inline V3 cross(V3 a, V3 b) {                                                 /* Lib.hs:259-261 */
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double squared_length(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; } /* 244-245 */
static inline double vlength(V3 a) { return sqrt(squared_length(a)); }               /* 241-242 */
static inline V3 unit(V3 a) { return divide(a, vlength(a)); }                        /* 247-248 */
static inline V3 vload(const double* p) { return v3(p[0], p[1], p[2]); }

/* GHC Ord defaults (ghc-prim GHC.Classes): max x y = if x <= y then y else x; min likewise. */
static inline double gmax(double x, double y) { return x <= y ? y : x; }
static inline double gmin(double x, double y) { return x <= y ? x : y; }

/* ------------------------------------------------------------------ RNG */
/* splitmix-0.1 (System.Random.SplitMix) restated; random-1.2.0 `random :: Double`. */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 33)) * 0xff51afd7ed558ccdULL;
    z = (z ^ (z >> 33)) * 0xc4ceb9fe1a85ec53ULL;
    return z ^ (z >> 33);
}
static inline uint64_t mix64v13(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static inline uint64_t mix_gamma(uint64_t z) {
    z = mix64v13(z) | 1ULL;
    int n = __builtin_popcountll(z ^ (z >> 1));
    return n >= 24 ? z : (z ^ 0xaaaaaaaaaaaaaaaaULL);
}
#define GOLDEN_GAMMA 0x9e3779b97f4a7c15ULL

/* Word64 -> Double exactly as random-1.2.0 uniformDouble01M / 2^64, then `random` = 1 - x
 * (randomR (0,1): x*0 + (1-x)*1). (double)w is round-to-nearest like ghc-prim hs_word2double. */
static inline double word_to_draw(uint64_t w) {
    double x = (double)w / 18446744073709551616.0;
    return 1.0 - x;
}

/* Tier B: Philox4x32-10 (Salmon et al. 2011; Random123 constants). */
static inline void philox4x32_10(const uint32_t in[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
    int mode;                 /* RT_RNG_EXACT / RT_RNG_PHILOX */
    uint64_t seed, gamma;     /* exact: SMGen */
    uint32_t key[2];          /* philox */
    uint32_t sample, pid;
    uint32_t pair;            /* next 128-bit block */
    int have_spare;
    uint64_t spare;
    int64_t* draws;           /* optional counter */
} Rng;

static inline uint64_t rng_word(Rng* g) {
    if (g->draws) (*g->draws)++;
    if (g->mode == RT_RNG_EXACT) { /* nextWord64 */
        g->seed += g->gamma;
        return mix64(g->seed);
    }
    if (g->have_spare) { g->have_spare = 0; return g->spare; }
    uint32_t ctr[4] = {g->pair, g->sample, g->pid, 0u}, o[4];
    philox4x32_10(ctr, g->key, o);
    g->pair++;
    g->spare = (uint64_t)o[2] | ((uint64_t)o[3] << 32);
    g->have_spare = 1;
    return (uint64_t)o[0] | ((uint64_t)o[1] << 32);
}
/* randomDoubleM (src/Lib.hs:1119-1125) */
static inline double D(Rng* g) { return word_to_draw(rng_word(g)); }
/* Tier B, a medium occurrence's draw: the first word of the Philox block at counter {words of the sample's
   stream consumed so far (the walk consumes none, so this names the walk), sample, pixel, 2^31 | key}. */
static inline double keyed_draw(const Rng* g, uint32_t key) {
    uint32_t ctr[4] = {2u * g->pair - (uint32_t)g->have_spare, g->sample, g->pid, 0x80000000u | key}, o[4];
    philox4x32_10(ctr, g->key, o);
    return word_to_draw((uint64_t)o[0] | ((uint64_t)o[1] << 32));
}
/* randomDoubleRM (src/Lib.hs:1127-1130) */
static inline double DR(Rng* g, double mn, double mx) { double rd = D(g); return mn + (mx - mn) * rd; }

/* randomInUnitSphere (src/Lib.hs:1160-1168) */
static V3 random_in_unit_sphere(Rng* g) {
    for (;;) {
        double x = D(g), y = D(g), z = D(g);
        V3 p = vsub(scale(2.0, v3(x, y, z)), v3(1.0, 1.0, 1.0));
        if (squared_length(p) < 1.0) return p;
    }
}
/* randomInUnitDisk (src/Lib.hs:1178-1185) */
static V3 random_in_unit_disk(Rng* g) {
    for (;;) {
        double x = D(g), y = D(g);
        V3 p = vsub(scale(2.0, v3(x, y, 0.0)), v3(1.0, 1.0, 0.0));
        if (squared_length(p) < 1.0) return p;
    }
}
/* randomUnitVectorM (src/Lib.hs:1187-1197) */
static V3 random_unit_vector(Rng* g) {
    double aa = D(g);
    double a = aa * 2.0 * PI;
    double zz = D(g);
    double z = (zz * 2.0) - 1.0;
    double r = sqrt(1.0 - z * z);
    return v3(r * o_cos(a), r * o_sin(a), z);
}
/* randomCosineDirection (src/Lib.hs:1206-1217) */
static V3 random_cosine_direction(Rng* g) {
    double r1 = D(g), r2 = D(g);
    double z = sqrt(1.0 - r2);
    double phi = 2.0 * PI * r1;
    double x = o_cos(phi) * sqrt(r2);
    double y = o_sin(phi) * sqrt(r2);
    return v3(x, y, z);
}
/* randomToSphereM (src/Lib.hs:1219-1228) */
static V3 random_to_sphere(Rng* g, double radius, double dist_squared) {
    double r1 = D(g), r2 = D(g);
    double z = 1.0 + r2 * (sqrt(1.0 - radius * radius / dist_squared) - 1.0);
    double phi = 2.0 * PI * r1;
    double s = sqrt(1.0 - z * z);
    return v3(o_cos(phi) * s, o_sin(phi) * s, z);
}

/* ------------------------------------------------------------------ ONB (src/Lib.hs:263-279) */
typedef struct { V3 u, v, w; } ONB;
static ONB onb_from_w(V3 n) {
    ONB o;
    o.w = unit(n);
    V3 a = fabs(o.w.x) > 0.9 ? v3(0.0, 1.0, 0.0) : v3(1.0, 0.0, 0.0);
    o.v = unit(cross(o.w, a));
    o.u = cross(o.w, o.v);
    return o;
}
static V3 onb_local_v(ONB o, V3 a) { /* scale a u |+| scale b v |+| scale c w */
    return vadd(vadd(scale(a.x, o.u), scale(a.y, o.v)), scale(a.z, o.w));
}

/* ------------------------------------------------------------------ GHC atan2 */
/* RealFloat class default (GHC.Float), used by `hit Sphere` (src/Lib.hs:1102). */
static int is_neg_zero(double x) { return x == 0.0 && signbit(x); }
double oracle_ghc_atan2(double y, double x) {
    if (x > 0) return o_atan(y / x);
    if (x == 0 && y > 0) return PI / 2;
    if (x < 0 && y > 0) return PI + o_atan(y / x);
    if ((x <= 0 && y < 0) || (x < 0 && is_neg_zero(y)) || (is_neg_zero(x) && is_neg_zero(y)))
        return -oracle_ghc_atan2(-y, x);
    if (y == 0 && (x < 0 || is_neg_zero(x))) return PI;
    if (x == 0 && y == 0) return y;
    return x + y;
}

/* ------------------------------------------------------------------ scene access */
typedef struct {
    const rt_scene_desc* s;
    const rt_camera* cam;
    int width, height, spp, max_depth;
    int64_t* counters; /* per-thread, optional */
    const uint32_t* medcount; /* medium occurrences under each node (tier-B medium keys), or NULL */
} Ctx;

/* Medium occurrences under each node of the world DAG (children precede parents): a BVH node's are its
   children's, a Translate/Rotate's its child's, a ConstantMedium is one. The walk keys a medium occurrence
   by its preorder rank (hit's `mb`: the occurrences left of it), unless the record carries its key + 1 in
   f[1] (an unfolded array, rt_rebuild_bvh). Caller frees. */
static uint32_t* medium_counts(const rt_scene_desc* d) {
    uint32_t* m = (uint32_t*)calloc((size_t)d->n_nodes, sizeof(uint32_t));
    for (int i = 0; i < d->n_nodes; ++i) {
        const rt_node* n = &d->nodes[i];
        if (n->type == RT_NODE_CONSTANT_MEDIUM) m[i] = 1;
        else if (n->type == RT_NODE_BVH && n->a >= 0 && n->a < i && n->b >= 0 && n->b < i) m[i] = m[n->a] + m[n->b];
        else if ((n->type == RT_NODE_TRANSLATE || n->type == RT_NODE_ROTATE) && n->a >= 0 && n->a < i) m[i] = m[n->a];
    }
    return m;
}

enum { C_WORLD_QUERIES, C_BOX_TESTS, C_SPHERE_TESTS, C_RECT_TESTS, C_OTHER_PRIMS, C_SCATTERS,
       C_DRAWS, C_SAMPLES, C_LIGHT_QUERIES, C_NCOUNTERS };
#define CNT(ctx, k) do { if ((ctx)->counters) (ctx)->counters[k]++; } while (0)

typedef struct { V3 o, d; double tm; } Ray;
typedef struct { double t; V3 p, n; double u, v; int ff; int mat; } Hit;

static inline V3 at(Ray r, double t) { return vadd(r.o, scale(t, r.d)); } /* Lib.hs:317-318 */

/* faceNormal (src/Lib.hs:1111-1117) */
static inline void face_normal(Ray r, V3 outward, int* ff, V3* n) {
    *ff = dot(r.d, outward) < 0;
    *n = *ff ? outward : vneg(outward);
}

/* ------------------------------------------------------------------ textures */
/* noise / perlinInterp / turb (src/Lib.hs:441-494) */
static int64_t hmod(int64_t a, int64_t m) { int64_t r = a % m; return r < 0 ? r + m : r; } /* Haskell `mod` */
static double noise(const rt_perlin* P, double sc, V3 p) {
    V3 q = scale(sc, p);
    double fi = floor(q.x), fj = floor(q.y), fk = floor(q.z);
    int64_t i = (int64_t)fi, j = (int64_t)fj, k = (int64_t)fk;
    double u = q.x - (double)i, v = q.y - (double)j, w = q.z - (double)k;
    double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
    /* foldr over ds = [(di,dj,dk) | di<-[0,1], dj<-[0,1], dk<-[0,1]]: accumulate from the
     * last element (1,1,1) down to (0,0,0). */
    double acc = 0.0;
    for (int idx = 7; idx >= 0; --idx) {
        int di = (idx >> 2) & 1, dj = (idx >> 1) & 1, dk = idx & 1;
        int r = P->perm_x[hmod(i + di, 256)] ^ P->perm_y[hmod(j + dj, 256)] ^ P->perm_z[hmod(k + dk, 256)];
        V3 val = vload(P->ranvec[r]);
        double I = di, J = dj, K = dk;
        acc = acc + ((I * uu + (1 - I) * (1 - uu)) * (J * vv + (1 - J) * (1 - vv)) *
                     (K * ww + (1 - K) * (1 - ww)) * dot(val, v3(u - I, v - J, w - K)));
    }
    return acc;
}
static double turb(const rt_perlin* P, double sc, V3 p, int depth) {
    double acc = 0.0, weight = 1.0;
    V3 tp = p;
    for (int d = 0; d < depth; ++d) {
        acc = acc + weight * noise(P, sc, tp);
        tp = scale(2.0, tp);
        weight = weight * 0.5;
    }
    return fabs(acc);
}
/* textureValue (src/Lib.hs:496-513) */
static V3 texture_value(const Ctx* c, int tid, double u, double v, V3 p) {
    const rt_texture* t = &c->s->textures[tid];
    switch (t->type) {
    case RT_TEX_CONSTANT:
        return v3(t->f[0], t->f[1], t->f[2]);
    case RT_TEX_CHECKER:
        if (o_sin(10 * p.x) * o_sin(10 * p.y) * o_sin(10 * p.z) < 0) return texture_value(c, t->a, u, v, p);
        return texture_value(c, t->b, u, v, p);
    case RT_TEX_PERLIN: {
        double m = 0.5 * (1.0 + o_sin(p.z + 10 * turb(&c->s->perlins[t->a], t->f[0], p, 7)));
        return scale(m, v3(1.0, 1.0, 1.0));
    }
    case RT_TEX_IMAGE: {
        if (t->a < 0) return v3(0, 1, 1);
        const rt_image* im = &c->s->images[t->a];
        double nxd = (double)t->b;
        double ci = u * nxd;
        ci = ci < 0 ? 0 : (ci > nxd - EPSILON ? nxd - EPSILON : ci);
        double nyd = (double)t->c;
        double cj = (1.0 - v) * nyd - EPSILON;
        cj = cj < 0 ? 0 : (cj > nyd - EPSILON ? nyd - EPSILON : cj);
        /* a NaN coordinate would crash JuicyPixels' pixelAt in the reference; clamp to texel 0 */
        int i = ci == ci ? (int)floor(ci) : 0, j = cj == cj ? (int)floor(cj) : 0;
        const uint8_t* px = c->s->image_pool + im->offset + ((int64_t)j * im->width + i) * 3;
        return v3(px[0] / 255.0, px[1] / 255.0, px[2] / 255.0); /* colorToAlbedo Lib.hs:294-297 */
    }
    }
    return v3(0, 0, 0);
}

/* ------------------------------------------------------------------ hit (src/Lib.hs:970-1109) */
/* boxRayIntersect (src/Lib.hs:798-814) */
static int box_ray_intersect(const double* bx, Ray r, double t_min, double t_max) {
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    for (int a = 0; a < 3; ++a) {
        double ta = (bx[a] - o[a]) / d[a];
        double tb = (bx[a + 3] - o[a]) / d[a];
        double t0, t1;
        if (ta < tb) { t0 = ta; t1 = tb; } else { t0 = tb; t1 = ta; }
        double tmin = gmax(t0, t_min);
        double tmax = gmin(t1, t_max);
        if (!(tmax > tmin)) return 0;
    }
    return 1;
}

/* The joint slab test the product adds to boxRayIntersect (ray-tracing_amd/csrc/rt_trace.h box_hit_exact):
 * the largest of the axes' clipped lower bounds below the smallest of their upper bounds. Not the
 * reference's: only probes and tests use it (RT_PROBE_BOX). */
static int box_joint(const double* bx, Ray r, double t_min, double t_max) {
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    double lmax = t_min, hmin = t_max;
    for (int a = 0; a < 3; ++a) {
        const double ta = (bx[a] - o[a]) / d[a], tb = (bx[a + 3] - o[a]) / d[a];
        const double t0 = ta < tb ? ta : tb, t1 = ta < tb ? tb : ta;
        const double lo = gmax(t0, t_min), hi = gmin(t1, t_max);
        if (lo > lmax) lmax = lo;
        if (hi < hmin) hmin = hi;
    }
    return hmin > lmax;
}

/* rectHit (src/Lib.hs:1005-1028); plane 0 XY, 1 XZ, 2 YZ */
static int rect_hit(int plane, double i0, double i1, double j0, double j1, double k, int mat, Ray r,
                    double t_min, double t_max, Hit* h) {
    double oi, oj, ok, di, dj, dk;
    V3 outward;
    if (plane == 0) { oi = r.o.x; oj = r.o.y; ok = r.o.z; di = r.d.x; dj = r.d.y; dk = r.d.z; outward = v3(0, 0, 1); }
    else if (plane == 1) { oi = r.o.x; oj = r.o.z; ok = r.o.y; di = r.d.x; dj = r.d.z; dk = r.d.y; outward = v3(0, 1, 0); }
    else { oi = r.o.y; oj = r.o.z; ok = r.o.x; di = r.d.y; dj = r.d.z; dk = r.d.x; outward = v3(1, 0, 0); }
    double t = (k - ok) / dk;
    if ((t < t_min) || (t > t_max)) return 0;
    double i = oi + t * di, j = oj + t * dj;
    if ((i < i0) || (i > i1) || (j < j0) || (j > j1)) return 0;
    h->t = t;
    h->u = (i - i0) / (i1 - i0);
    h->v = (j - j0) / (j1 - j0);
    h->p = at(r, t);
    face_normal(r, outward, &h->ff, &h->n);
    h->mat = mat;
    return 1;
}

/* hit Sphere (src/Lib.hs:1081-1105) */
static int sphere_hit(V3 sc, double sr, int sm, Ray r, double t_min, double t_max, Hit* h) {
    V3 oc = vsub(r.o, sc);
    double a = dot(r.d, r.d);
    double b = dot(oc, r.d);
    double c = dot(oc, oc) - (sr * sr);
    double disc = b * b - a * c;
    if (!(disc > 0)) return 0;
    double sd = sqrt(disc);
    double temp1 = ((-b) - sd) / a;
    double temp2 = ((-b) + sd) / a;
    double temp;
    if (t_min < temp1 && temp1 < t_max) temp = temp1;
    else if (t_min < temp2 && temp2 < t_max) temp = temp2;
    else return 0;
    h->t = temp;
    h->p = at(r, temp);
    V3 outward = divide(vsub(h->p, sc), sr);
    face_normal(r, outward, &h->ff, &h->n);
    double phi = oracle_ghc_atan2(outward.z, outward.x);
    double theta = o_asin(outward.y);
    h->u = 1.0 - ((phi + PI) / (2 * PI));
    h->v = (theta + (PI / 2)) / PI;
    h->mat = sm;
    return 1;
}

/* rotatePoint / unRotatePoint (src/Lib.hs:763-787) */
static V3 rotate_point(int axis, double s, double c, V3 p) {
    if (axis == 0) return v3(p.x, c * p.y - s * p.z, s * p.y + c * p.z);
    if (axis == 1) return v3(c * p.x + s * p.z, p.y, -s * p.x + c * p.z);
    return v3(c * p.x - s * p.y, s * p.x + c * p.y, p.z);
}
static V3 unrotate_point(int axis, double s, double c, V3 p) {
    if (axis == 0) return v3(p.x, c * p.y + s * p.z, -s * p.y + c * p.z);
    if (axis == 1) return v3(c * p.x - s * p.z, p.y, s * p.x + c * p.z);
    return v3(c * p.x + s * p.y, -s * p.x + c * p.y, p.z);
}

static int hit(const Ctx* c, int id, Ray r, double t_min, double t_max, Rng* g, Hit* h, uint32_t mb) {
    if (id < 0) return 0; /* Unhittable */
    const rt_node* n = &c->s->nodes[id];
    switch (n->type) {
    case RT_NODE_BVH: { /* Lib.hs:971-988 */
        CNT(c, C_BOX_TESTS);
        if (!box_ray_intersect(n->f, r, t_min, t_max)) return 0;
        Hit hl;
        const uint32_t mb_right = mb + (c->medcount ? c->medcount[n->a] : 0);
        if (!hit(c, n->a, r, t_min, t_max, g, &hl, mb)) return hit(c, n->b, r, t_min, t_max, g, h, mb_right);
        Hit hr;
        if (hit(c, n->b, r, t_min, hl.t, g, &hr, mb_right)) *h = hr; else *h = hl;
        return 1;
    }
    case RT_NODE_CUBOID: { /* Lib.hs:989-1004: foldr closerHit, full range for every face */
        const double x0 = n->f[0], y0 = n->f[1], z0 = n->f[2], x1 = n->f[3], y1 = n->f[4], z1 = n->f[5];
        const double rects[6][6] = {{0, x0, x1, y0, y1, z1}, {0, x0, x1, y0, y1, z0},
                                    {1, x0, x1, z0, z1, y1}, {1, x0, x1, z0, z1, y0},
                                    {2, y0, y1, z0, z1, x1}, {2, y0, y1, z0, z1, x0}};
        int have = 0;
        Hit best;
        for (int i = 5; i >= 0; --i) {
            Hit hh;
            CNT(c, C_RECT_TESTS);
            if (rect_hit((int)rects[i][0], rects[i][1], rects[i][2], rects[i][3], rects[i][4], rects[i][5],
                         n->a, r, t_min, t_max, &hh)) {
                if (!have || hh.t < best.t) { best = hh; have = 1; }
            }
        }
        if (have) *h = best;
        return have;
    }
    case RT_NODE_RECT_XY:
    case RT_NODE_RECT_XZ:
    case RT_NODE_RECT_YZ:
        CNT(c, C_RECT_TESTS);
        return rect_hit(n->type - RT_NODE_RECT_XY, n->f[0], n->f[1], n->f[2], n->f[3], n->f[4], n->a, r,
                        t_min, t_max, h);
    case RT_NODE_TRANSLATE: { /* Lib.hs:1029-1037 */
        CNT(c, C_OTHER_PRIMS);
        V3 off = vload(n->f);
        Ray mr = {vsub(r.o, off), r.d, r.tm};
        Hit ch;
        if (!hit(c, n->a, mr, t_min, t_max, g, &ch, mb)) return 0;
        *h = ch;
        face_normal(mr, ch.n, &h->ff, &h->n);
        h->p = vadd(ch.p, off);
        return 1;
    }
    case RT_NODE_ROTATE: { /* Lib.hs:1038-1052 */
        CNT(c, C_OTHER_PRIMS);
        int ax = n->b;
        double s = n->f[0], co = n->f[1];
        Ray rr = {unrotate_point(ax, s, co, r.o), unrotate_point(ax, s, co, r.d), r.tm};
        Hit ch;
        if (!hit(c, n->a, rr, t_min, t_max, g, &ch, mb)) return 0;
        *h = ch;
        h->p = rotate_point(ax, s, co, ch.p);
        face_normal(rr, rotate_point(ax, s, co, ch.n), &h->ff, &h->n);
        return 1;
    }
    case RT_NODE_CONSTANT_MEDIUM: { /* Lib.hs:1053-1080 */
        CNT(c, C_OTHER_PRIMS);
        Hit h1, h2;
        if (!hit(c, n->a, r, -INFINITY, INFINITY, g, &h1, 0)) return 0;
        if (!hit(c, n->a, r, h1.t + EPSILON, INFINITY, g, &h2, 0)) return 0;
        /* Tier B (Philox streams): the draw is keyed by (walk, occurrence) and the candidate computed over
           the boundary's whole inside, then bounded like any leaf (newt <= t_max): the closest hit no longer
           depends on the order media are visited in. Tier A: the reference's own, the
           stream's next draw, made only when the inside meets [t_min, t_max]. */
        const int keyed = g->mode == RT_RNG_PHILOX;
        double rec1tp = gmax(t_min, h1.t);
        double rec2t = keyed ? h2.t : gmin(t_max, h2.t);
        if (rec1tp >= rec2t) return 0;
        double rec1t = rec1tp < 0 ? 0 : rec1tp;
        double ray_length = vlength(r.d);
        double dist_inside = (rec2t - rec1t) * ray_length;
        double rnd = keyed ? keyed_draw(g, n->f[1] >= 1.0 ? (uint32_t)(n->f[1] - 1.0) : mb) : D(g);
        double hit_dist = n->f[0] * o_log(rnd);
        if (hit_dist > dist_inside) return 0;
        double newt = rec1t + (hit_dist / ray_length);
        if (keyed && !(newt <= t_max)) return 0;
        h->t = newt;
        h->p = at(r, newt);
        h->n = v3(1, 0, 0);
        h->u = 0;
        h->v = 0;
        h->ff = 1;
        h->mat = n->b;
        return 1;
    }
    case RT_NODE_SPHERE:
        CNT(c, C_SPHERE_TESTS);
        return sphere_hit(vload(n->f), n->f[3], n->a, r, t_min, t_max, h);
    case RT_NODE_MOVING_SPHERE: { /* Lib.hs:1106-1108 */
        CNT(c, C_SPHERE_TESTS);
        const rt_node* e = n + 1;
        V3 c0 = vload(n->f), c1 = vload(n->f + 3);
        V3 sc = vadd(c0, scale((r.tm - e->f[0]) / e->f[2], vsub(c1, c0)));
        return sphere_hit(sc, e->f[3], n->a, r, t_min, t_max, h);
    }
    default:
        return 0; /* Unhittable */
    }
}

/* ------------------------------------------------------------------ lights (Lib.hs:662-724) */
static int htbl_size(const Ctx* c, int id) { return id < 0 ? 0 : c->s->nodes[id].c; }

/* htblPdfValue (src/Lib.hs:673-705) */
static double htbl_pdf_value(const Ctx* c, int id, V3 origin, V3 v, Rng* g) {
    CNT(c, C_LIGHT_QUERIES);
    Ray r = {origin, v, 0.0};
    Hit hh;
    if (!hit(c, id, r, EPSILON, INFINITY, g, &hh, 0)) return 0.0;
    const rt_node* n = &c->s->nodes[id];
    if (n->type == RT_NODE_RECT_XZ) {
        double x0 = n->f[0], x1 = n->f[1], z0 = n->f[2], z1 = n->f[3];
        double area = (x1 - x0) * (z1 - z0);
        double distance_squared = hh.t * hh.t * squared_length(v);
        double cosine = fabs(dot(v, hh.n) / vlength(v));
        return distance_squared / (cosine * area);
    }
    if (n->type == RT_NODE_SPHERE) {
        V3 center = vload(n->f);
        double radius = n->f[3];
        double cos_theta_max = sqrt(1 - radius * radius / squared_length(vsub(center, origin)));
        double solid_angle = 2 * PI * (1 - cos_theta_max);
        return 1 / solid_angle;
    }
    if (n->type == RT_NODE_BVH) {
        double left_pdf = htbl_pdf_value(c, n->a, origin, v, g) + 0;
        double left_weight = (double)htbl_size(c, n->a) / (double)n->c;
        double right_pdf = htbl_pdf_value(c, n->b, origin, v, g) + 0;
        double right_weight = (double)htbl_size(c, n->b) / (double)n->c;
        return left_weight * left_pdf + right_weight * right_pdf;
    }
    return 0.0;
}

/* htblRandom (src/Lib.hs:707-724) */
static V3 htbl_random(const Ctx* c, int id, V3 o, Rng* g) {
    if (id < 0) return v3(1, 0, 0);
    const rt_node* n = &c->s->nodes[id];
    if (n->type == RT_NODE_RECT_XZ) {
        double rx = DR(g, n->f[0], n->f[1]);
        double rz = DR(g, n->f[2], n->f[3]);
        return vsub(v3(rx, n->f[4], rz), o);
    }
    if (n->type == RT_NODE_SPHERE) {
        V3 dir = vsub(vload(n->f), o);
        double dist_squared = squared_length(dir);
        ONB uvw = onb_from_w(dir);
        V3 rts = random_to_sphere(g, n->f[3], dist_squared);
        return onb_local_v(uvw, rts);
    }
    if (n->type == RT_NODE_BVH) {
        double rd = D(g);
        if (rd < (double)htbl_size(c, n->a) / (double)n->c) return htbl_random(c, n->a, o, g);
        return htbl_random(c, n->b, o, g);
    }
    return v3(1, 0, 0);
}

/* ------------------------------------------------------------------ materials */
static V3 reflect(V3 v, V3 n) { return vsub(v, scale(2.0 * dot(v, n), n)); } /* Lib.hs:887-888 */
static V3 refract(V3 v, V3 n, double eta) {                                 /* Lib.hs:890-896 */
    V3 uv = unit(v);
    double cos_theta = dot(vneg(uv), n);
    V3 par = scale(eta, vadd(uv, scale(cos_theta, n)));
    V3 perp = scale(-sqrt(1.0 - squared_length(par)), n);
    return vadd(par, perp);
}
static double schlick(double cosine, double ref_idx) { /* Lib.hs:899-903 */
    double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
    double r1 = r0 * r0;
    return r1 + (1.0 - r1) * o_pow5(1 - cosine);
}

typedef struct { Ray ray; int specular; V3 att; double pdf; } Scatter;

/* scatter (src/Lib.hs:822-865); returns 0 for Nothing */
static int scatter(const Ctx* c, const rt_material* m, Ray r, const Hit* h, Rng* g, Scatter* s) {
    CNT(c, C_SCATTERS);
    switch (m->type) {
    case RT_MAT_LAMBERTIAN: {
        V3 att = texture_value(c, m->texture, h->u, h->v, h->p);
        ONB uvw = onb_from_w(h->n);
        /* pdfGenerate (MixturePdf (HittablePdf hp lights) (CosinePdf uvw)), Lib.hs:370-372 */
        double rd = D(g);
        V3 pdf_d;
        if (rd < 0.5) pdf_d = htbl_random(c, c->s->lights_root, h->p, g);
        else pdf_d = onb_local_v(uvw, random_cosine_direction(g));
        V3 dir = unit(pdf_d);
        s->ray.o = h->p; s->ray.d = dir; s->ray.tm = r.tm;
        /* pdfValue mixPdf (makeUnitVector pdfD), Lib.hs:379-382, 374-378 */
        double v1 = htbl_pdf_value(c, c->s->lights_root, h->p, dir, g);
        double cosine = dot(unit(dir), uvw.w);
        double v2 = cosine <= 0 ? 0 : cosine / PI;
        s->pdf = 0.5 * (v1 + v2);
        s->specular = 0;
        s->att = att;
        return 1;
    }
    case RT_MAT_METAL: {
        V3 r_unit = random_unit_vector(g);
        V3 reflected = reflect(unit(r.d), h->n);
        s->ray.o = h->p; s->ray.d = vadd(reflected, scale(m->param, r_unit)); s->ray.tm = r.tm;
        s->specular = 1;
        s->att = texture_value(c, m->texture, h->u, h->v, h->p);
        s->pdf = 0.0;
        return 1;
    }
    case RT_MAT_DIELECTRIC: {
        double ref_idx = m->param;
        double eta = h->ff ? 1.0 / ref_idx : ref_idx;
        V3 ud = unit(r.d);
        double cos_theta = gmin(dot(vneg(ud), h->n), 1.0);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        double rd = D(g);
        V3 dir;
        if ((eta * sin_theta > 1.0) || rd < schlick(cos_theta, eta)) dir = reflect(ud, h->n);
        else dir = refract(ud, h->n, eta);
        s->ray.o = h->p; s->ray.d = dir; s->ray.tm = r.tm;
        s->specular = 1;
        s->att = v3(1.0, 1.0, 1.0);
        s->pdf = 1.0;
        return 1;
    }
    case RT_MAT_DIFFUSE_LIGHT:
        return 0;
    case RT_MAT_ISOTROPIC: {
        V3 d = random_in_unit_sphere(g);
        s->ray.o = h->p; s->ray.d = d; s->ray.tm = r.tm;
        s->att = texture_value(c, m->texture, h->u, h->v, h->p);
        s->specular = 0;
        s->pdf = 1.0;
        return 1;
    }
    }
    return 0;
}

/* scatteringPdf (src/Lib.hs:867-878), Lambertian/Isotropic only */
static double scattering_pdf(const Hit* h, Ray scattered) {
    double cosine = dot(h->n, scattered.d);
    return cosine < 0 ? 0 : cosine / PI;
}

/* emitted (src/Lib.hs:880-885) */
static V3 emitted(const Ctx* c, const rt_material* m, const Hit* h) {
    if (m->type == RT_MAT_DIFFUSE_LIGHT && !h->ff) return texture_value(c, m->texture, h->u, h->v, h->p);
    return v3(0, 0, 0);
}

/* Tier-A path trace of one column (oracle_exact_trace; NULL otherwise): 10 doubles per segment. */
static double* g_tr = NULL;
static int g_tr_n = 0, g_tr_cap = 0, g_tr_row = 0, g_tr_j = 0;
static void trace_seg(int seg, int end, Ray r, const Rng* g) {
    if (!g_tr || g_tr_n >= g_tr_cap) return;
    double* o = g_tr + 10 * (size_t)g_tr_n++;
    o[0] = g_tr_row; o[1] = g_tr_j; o[2] = end ? -(seg + 1) : seg;
    o[3] = r.o.x; o[4] = r.o.y; o[5] = r.o.z; o[6] = r.d.x; o[7] = r.d.y; o[8] = r.d.z;
    memcpy(&o[9], &g->seed, 8);
}

/* rayColor (src/Lib.hs:1297-1333), recursion in the continuation's evaluation order:
 * specular: att |*| new; else att |*| (scatteringPdf `scale` (new `divide` pdfVal)). */
static V3 ray_color(const Ctx* c, Ray r, int d, Rng* g) {
    if (d <= 0) { trace_seg(c->max_depth - d, 1, r, g); return v3(0, 0, 0); }
    CNT(c, C_WORLD_QUERIES);
    Hit h;
    if (!hit(c, c->s->world_root, r, EPSILON, INFINITY, g, &h, 0)) {
        trace_seg(c->max_depth - d, 1, r, g);
        return vload(c->s->background);
    }
    const rt_material* m = &c->s->materials[h.mat];
    Scatter s;
    if (!scatter(c, m, r, &h, g, &s)) { trace_seg(c->max_depth - d, 1, r, g); return emitted(c, m, &h); }
    trace_seg(c->max_depth - d, 0, s.ray, g);
    V3 nw = ray_color(c, s.ray, d - 1, g);
    if (s.specular) return vmul(s.att, nw);
    double spdf = scattering_pdf(&h, s.ray);
    return vmul(s.att, scale(spdf, divide(nw, s.pdf)));
}

/* getRay (src/Lib.hs:1253-1267) */
static Ray get_ray(const Ctx* c, double s, double t, Rng* g) {
    const rt_camera* k = c->cam;
    V3 rd = scale(k->lens_radius, random_in_unit_disk(g));
    V3 offset = vadd(scale(rd.x, vload(k->u)), scale(rd.y, vload(k->v)));
    double tm = DR(g, k->t0, k->t1);
    Ray r;
    r.o = vadd(vload(k->origin), offset);
    r.d = vsub(vsub(vadd(vadd(vload(k->llc), scale(s, vload(k->horiz))), scale(t, vload(k->vert))),
                    vload(k->origin)),
               offset);
    r.tm = tm;
    return r;
}

/* clamp / scaleColor (src/Lib.hs:281-288): NaN -> 0 (floor NaN via Int is minBound). */
static uint8_t scale_color(double x) {
    double s = sqrt(x);
    double cl = s < 0.0 ? 0.0 : (s > 0.999 ? 0.999 : s);
    double f = floor(256 * cl);
    if (f != f) return 0;
    return (uint8_t)(int)f;
}

/* ------------------------------------------------------------------ runRender */
/* One pixel, tier A: uniformRandomUVs (Lib.hs:1358-1371, list in REVERSE draw order) then
 * renderPos (Lib.hs:1343-1350: foldM sampleColor in list order, then divide by ns). */
static V3 nan_zero(V3 a);
static V3 render_pixel_exact(const Ctx* c, int x, int y, Rng* g, double* uvbuf, int nanz) {
    int ns = c->spp;
    for (int i = 0; i < ns; ++i) {
        double ru = D(g), rv = D(g);
        uvbuf[2 * i] = ((double)x + ru) / (double)c->width;
        uvbuf[2 * i + 1] = ((double)y + rv) / (double)c->height;
    }
    V3 acc = v3(0, 0, 0);
    for (int i = ns - 1; i >= 0; --i) {
        g_tr_j = ns - 1 - i;
        Ray r = get_ray(c, uvbuf[2 * i], uvbuf[2 * i + 1], g);
        V3 c1 = ray_color(c, r, c->max_depth, g);
        if (nanz) c1 = nan_zero(c1); /* RT_FLAG_NAN_ZERO (tiers A and B: the tier-A/B statistical tests) */
        acc = vadd(acc, c1);
        CNT(c, C_SAMPLES);
    }
    return divide(acc, (double)ns);
}

/* One pixel, tier B: sample s draws from its own Philox stream; samples summed in sample order
   within fixed chunks, chunk sums in chunk order (include/rt.h, rt_sample_chunk). */
/* RT_FLAG_NAN_ZERO (parity diagnostic, include/rt.h): a NaN channel of a sample's colour adds 0 */
static V3 nan_zero(V3 a) { return v3(a.x != a.x ? 0.0 : a.x, a.y != a.y ? 0.0 : a.y, a.z != a.z ? 0.0 : a.z); }

static V3 render_pixel_philox(const Ctx* c, int x, int y, uint32_t pid, uint64_t seed, uint32_t flags,
                              int64_t* draws) {
    V3 acc = v3(0, 0, 0);
    const int ch = rt_sample_chunk((int64_t)c->width * c->height, c->spp);
    for (int k0 = 0; k0 < c->spp; k0 += ch) {
        V3 part = v3(0, 0, 0);
        const int k1 = k0 + ch < c->spp ? k0 + ch : c->spp;
        for (int s = k0; s < k1; ++s) {
            Rng g;
            memset(&g, 0, sizeof g);
            g.mode = RT_RNG_PHILOX;
            g.key[0] = (uint32_t)seed;
            g.key[1] = (uint32_t)(seed >> 32);
            g.sample = (uint32_t)s;
            g.pid = pid;
            g.draws = draws;
            double ru = D(&g), rv = D(&g);
            double u = ((double)x + ru) / (double)c->width;
            double v = ((double)y + rv) / (double)c->height;
            Ray r = get_ray(c, u, v, &g);
            V3 c1 = ray_color(c, r, c->max_depth, &g);
            if (flags & RT_FLAG_NAN_ZERO) c1 = nan_zero(c1);
            part = vadd(part, c1);
            CNT(c, C_SAMPLES);
        }
        acc = vadd(acc, part);
    }
    return divide(acc, (double)c->spp);
}

static void store_pixel(uint8_t* rgb, double* lin, int64_t idx, V3 a) {
    if (rgb) {
        rgb[idx * 3 + 0] = scale_color(a.x);
        rgb[idx * 3 + 1] = scale_color(a.y);
        rgb[idx * 3 + 2] = scale_color(a.z);
    }
    if (lin) { lin[idx * 3 + 0] = a.x; lin[idx * 3 + 1] = a.y; lin[idx * 3 + 2] = a.z; }
}

/*
 * Render output rows [row0, row1) (row 0 = top, y = H-1-row, pixelPositions Lib.hs:1488-1489).
 * Tier A needs row0 == 0 (each column's stream runs through every row above). Buffers hold
 * only the rendered rows: (row1-row0)*W*3. counters (optional) = C_NCOUNTERS int64 totals.
 */
int oracle_render_rows(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_params* p,
                       const uint64_t* col_gens, int row0, int row1, uint8_t* rgb, double* linear,
                       uint64_t* out_gens, int nthreads, int64_t* counters) {
    if (!scene || !cam || !p || p->width <= 0 || p->height <= 0 || p->spp <= 0) return -1;
    if (row0 < 0 || row1 > p->height || row0 > row1) return -1;
    if (p->rng_mode == RT_RNG_EXACT && (row0 != 0 || !col_gens)) return -1;
    if ((p->flags & RT_FLAG_SHARED_LIBM) && p->rng_mode != RT_RNG_EXACT) return -1; /* (as rt_render) */
    const int W = p->width, H = p->height;
    g_shared_libm = (p->flags & RT_FLAG_SHARED_LIBM) != 0;
    uint32_t* mc = medium_counts(scene);
    if (counters) memset(counters, 0, sizeof(int64_t) * C_NCOUNTERS);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    if (p->rng_mode == RT_RNG_EXACT) {
        /* columns are independent streams: parallel over columns, rows serial (Lib.hs:1498-1521) */
#pragma omp parallel
        {
            int64_t cnt[C_NCOUNTERS] = {0};
            double* uvbuf = (double*)malloc(sizeof(double) * 2 * (size_t)p->spp);
            Ctx c = {scene, cam, W, H, p->spp, p->max_depth, counters ? cnt : NULL, mc};
#pragma omp for schedule(dynamic, 1)
            for (int x = 0; x < W; ++x) {
                Rng g;
                memset(&g, 0, sizeof g);
                g.mode = RT_RNG_EXACT;
                g.seed = col_gens[2 * x];
                g.gamma = col_gens[2 * x + 1];
                g.draws = counters ? &cnt[C_DRAWS] : NULL;
                for (int row = 0; row < row1; ++row) {
                    int y = H - 1 - row;
                    V3 a = render_pixel_exact(&c, x, y, &g, uvbuf, (p->flags & RT_FLAG_NAN_ZERO) != 0);
                    store_pixel(rgb, linear, (int64_t)row * W + x, a);
                }
                if (out_gens) { out_gens[2 * x] = g.seed; out_gens[2 * x + 1] = g.gamma; }
            }
            free(uvbuf);
            if (counters) {
#pragma omp critical
                for (int k = 0; k < C_NCOUNTERS; ++k) counters[k] += cnt[k];
            }
        }
    } else {
        const int64_t npx = (int64_t)(row1 - row0) * W;
#pragma omp parallel
        {
            int64_t cnt[C_NCOUNTERS] = {0};
            Ctx c = {scene, cam, W, H, p->spp, p->max_depth, counters ? cnt : NULL, mc};
#pragma omp for schedule(dynamic, 16)
            for (int64_t i = 0; i < npx; ++i) {
                int row = row0 + (int)(i / W), x = (int)(i % W);
                int y = H - 1 - row;
                uint32_t pid = (uint32_t)((int64_t)row * W + x);
                V3 a = render_pixel_philox(&c, x, y, pid, p->seed, p->flags, counters ? &cnt[C_DRAWS] : NULL);
                store_pixel(rgb, linear, i, a);
            }
            if (counters) {
#pragma omp critical
                for (int k = 0; k < C_NCOUNTERS; ++k) counters[k] += cnt[k];
            }
        }
    }
    g_shared_libm = 0;
    free(mc);
    return 0;
}

/* Tier A, one column `col` of the frame, serially, with every path segment recorded: 10 doubles per
   segment {row, sample, seg (or -(seg + 1) where the path ends), ray o xyz, d xyz (the scattered ray; at
   the end the segment's own ray), the generator's seed after the segment (uint64 bits)}. The device's
   rt_debug_exact_trace records the same: the first differing record localises a tier-A divergence. */
int oracle_exact_trace(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_params* p,
                       const uint64_t* col_gens, int col, double* out, int cap, int* out_n) {
    if (!scene || !cam || !p || !col_gens || col < 0 || col >= p->width || !out || cap < 0) return -1;
    g_shared_libm = (p->flags & RT_FLAG_SHARED_LIBM) != 0;
    Ctx c = {scene, cam, p->width, p->height, p->spp, p->max_depth, NULL, NULL};
    double* uvbuf = (double*)malloc(sizeof(double) * 2 * (size_t)p->spp);
    Rng g;
    memset(&g, 0, sizeof g);
    g.mode = RT_RNG_EXACT;
    g.seed = col_gens[2 * col];
    g.gamma = col_gens[2 * col + 1];
    g_tr = out; g_tr_n = 0; g_tr_cap = cap;
    for (int row = 0; row < p->height; ++row) {
        g_tr_row = row;
        (void)render_pixel_exact(&c, col, p->height - 1 - row, &g, uvbuf, (p->flags & RT_FLAG_NAN_ZERO) != 0);
    }
    *out_n = g_tr_n;
    g_tr = NULL;
    g_shared_libm = 0;
    free(uvbuf);
    return 0;
}

/* include/rt_libm.h on the host (tests compare the device's evaluation of the same functions):
   op 12 sin, 13 cos, 14 atan, 15 asin, 16 log, 17 GHC atan2(x, y) over them (rt_debug_math's ids). */
void oracle_shared_libm(int op, const double* x, const double* y, int n, double* out) {
    g_shared_libm = 1;
    for (int i = 0; i < n; ++i) {
        switch (op) {
            case 12: out[i] = rtlm_sin(x[i]); break;
            case 13: out[i] = rtlm_cos(x[i]); break;
            case 14: out[i] = rtlm_atan(x[i]); break;
            case 15: out[i] = rtlm_asin(x[i]); break;
            case 16: out[i] = rtlm_log(x[i]); break;
            default: out[i] = oracle_ghc_atan2(x[i], y[i]); break;
        }
    }
    g_shared_libm = 0;
}

int oracle_render(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_params* p,
                  const uint64_t* col_gens, uint8_t* rgb, double* linear, uint64_t* out_gens, int nthreads) {
    return oracle_render_rows(scene, cam, p, col_gens, 0, p->height, rgb, linear, out_gens, nthreads, NULL);
}

int oracle_num_counters(void) { return C_NCOUNTERS; }

/* Closest hit of n world rays (7 doubles each) — same layout as rt_debug_closest_hits. */
int oracle_closest_hits(const rt_scene_desc* scene, const double* rays, int n, double tmin, double tmax,
                        uint64_t seed, double* out) {
    uint32_t* mc = medium_counts(scene);
    Ctx c = {scene, NULL, 0, 0, 0, 0, NULL, mc};
    for (int i = 0; i < n; ++i) {
        const double* q = rays + 7 * i;
        Ray r = {v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), q[6]};
        Rng g;
        memset(&g, 0, sizeof g);
        g.mode = RT_RNG_PHILOX;
        g.key[0] = (uint32_t)seed;
        g.key[1] = (uint32_t)(seed >> 32);
        g.pid = (uint32_t)i;
        Hit h;
        double* o = out + 12 * i;
        memset(o, 0, sizeof(double) * 12);
        if (hit(&c, scene->world_root, r, tmin, tmax, &g, &h, 0)) {
            o[0] = 1; o[1] = h.t;
            o[2] = h.p.x; o[3] = h.p.y; o[4] = h.p.z;
            o[5] = h.n.x; o[6] = h.n.y; o[7] = h.n.z;
            o[8] = h.u; o[9] = h.v; o[10] = h.ff; o[11] = h.mat;
        }
    }
    free(mc);
    return 0;
}

/* ------------------------------------------------------------------ RNG exports (KAT tests) */
void oracle_mk_smgen(uint64_t s, uint64_t out[2]) { out[0] = mix64(s); out[1] = mix_gamma(s + GOLDEN_GAMMA); }
uint64_t oracle_next_word64(uint64_t gen[2]) { gen[0] += gen[1]; return mix64(gen[0]); }
double oracle_random_double(uint64_t gen[2]) { return word_to_draw(oracle_next_word64(gen)); }
void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { philox4x32_10(ctr, key, out); }
double oracle_word_to_draw(uint64_t w) { return word_to_draw(w); }
uint8_t oracle_scale_color(double x) { return scale_color(x); }

/* ------------------------------------------------------------------ per-function probes
 * Golden vectors for single hot-path functions (tests/golden/make_function_goldens.py).
 * Record i is evaluated with its own tier-B Philox stream (key = seed, pid = i, sample 0), so the
 * device probe (rt_debug_probe) consumes the same numbers. Layouts (doubles per record), in -> out:
 *   0 scatter   (src/Lib.hs:822-865, emitted 880-885):
 *               ray o3 d3 tm, hit t p3 n3 u v ff mat (18) -> scattered, ray o3 d3 tm, att3 (emitted
 *               when Nothing), pdf, specular, words consumed (14)
 *   1 htblRandom   (src/Lib.hs:707-724) on the lights tree: origin3 (3) -> direction3, words (4)
 *   2 htblPdfValue (src/Lib.hs:673-705) on the lights tree: origin3, v3 (6) -> pdf, words (2)
 *   3 textureValue (src/Lib.hs:496-513): texture id, u, v, p3 (6) -> albedo3 (3)
 *   4 getRay       (src/Lib.hs:1253-1267) with `cam`: s, t (2) -> ray o3 d3 tm, words (8)
 *   5 box test     box min3 max3, ray o3 d3, t_min, t_max (14) -> boxRayIntersect (src/Lib.hs:798-814) AND
 *                  the joint slab test (the product's default culling; twice, for its two implementations),
 *                  boxRayIntersect alone (3)
 */
int oracle_probe(const rt_scene_desc* scene, const rt_camera* cam, int op, const double* in, int n, uint64_t seed,
                 double* out) {
    static const int IN[6] = {18, 3, 6, 6, 2, 14}, OUT[6] = {14, 4, 2, 3, 8, 3};
    if (!scene || op < 0 || op > 5 || n < 0 || (op == 4 && !cam)) return -1;
    Ctx c = {scene, cam, 0, 0, 0, 0, NULL, NULL};
    for (int i = 0; i < n; ++i) {
        const double* q = in + (size_t)IN[op] * i;
        double* o = out + (size_t)OUT[op] * i;
        memset(o, 0, sizeof(double) * OUT[op]);
        Rng g;
        memset(&g, 0, sizeof g);
        g.mode = RT_RNG_PHILOX;
        g.key[0] = (uint32_t)seed;
        g.key[1] = (uint32_t)(seed >> 32);
        g.pid = (uint32_t)i;
        switch (op) {
            case 0: {
                Ray r = {v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), q[6]};
                Hit h = {q[7], v3(q[8], q[9], q[10]), v3(q[11], q[12], q[13]), q[14], q[15], (int)q[16], (int)q[17]};
                const rt_material* m = &scene->materials[h.mat];
                Scatter s;
                if (scatter(&c, m, r, &h, &g, &s)) {
                    o[0] = 1;
                    o[1] = s.ray.o.x; o[2] = s.ray.o.y; o[3] = s.ray.o.z;
                    o[4] = s.ray.d.x; o[5] = s.ray.d.y; o[6] = s.ray.d.z; o[7] = s.ray.tm;
                    o[8] = s.att.x; o[9] = s.att.y; o[10] = s.att.z;
                    o[11] = s.pdf; o[12] = s.specular;
                } else {
                    V3 e = emitted(&c, m, &h);
                    o[8] = e.x; o[9] = e.y; o[10] = e.z;
                }
                o[13] = 2.0 * g.pair - g.have_spare;
                break;
            }
            case 1: {
                V3 d = htbl_random(&c, scene->lights_root, v3(q[0], q[1], q[2]), &g);
                o[0] = d.x; o[1] = d.y; o[2] = d.z;
                o[3] = 2.0 * g.pair - g.have_spare;
                break;
            }
            case 2:
                o[0] = scene->lights_root < 0 ? 0.0
                                              : htbl_pdf_value(&c, scene->lights_root, v3(q[0], q[1], q[2]),
                                                               v3(q[3], q[4], q[5]), &g);
                o[1] = 2.0 * g.pair - g.have_spare;
                break;
            case 3: {
                V3 a = texture_value(&c, (int)q[0], q[1], q[2], v3(q[3], q[4], q[5]));
                o[0] = a.x; o[1] = a.y; o[2] = a.z;
                break;
            }
            case 5: {
                const Ray r = {v3(q[6], q[7], q[8]), v3(q[9], q[10], q[11]), 0.0};
                const int per_axis = box_ray_intersect(q, r, q[12], q[13]);
                o[0] = o[1] = per_axis && box_joint(q, r, q[12], q[13]);
                o[2] = per_axis;
                break;
            }
            default: {
                Ray r = get_ray(&c, q[0], q[1], &g);
                o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
                o[3] = r.d.x; o[4] = r.d.y; o[5] = r.d.z; o[6] = r.tm;
                o[7] = 2.0 * g.pair - g.have_spare;
                break;
            }
        }
    }
    return 0;
}
