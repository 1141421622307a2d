// rt_trace.h — intersection, traversal, light sampling, textures and scattering (device).
#pragma once
#ifndef RT_FRAME_BATCH
#define RT_FRAME_BATCH 0
#endif
#include "rt_device.h"

namespace rtd {

// fp32 ray state (Trav::o32 ...) maintained: the 4-wide walk, or the mixed walk's wide subtrees
template <unsigned F>
constexpr bool kRay32 = (F & (F_WIDE | F_MIXW)) != 0;

// Work counters of the counting build (F_COUNT); all zero-cost otherwise.
struct Cnt {
  unsigned box, prim, other, light, wide;
  unsigned islot, lslot, oslot;  // lane slots (live lanes) of wide-node steps, leaf steps, outer iterations
  unsigned phit;                 // leaf tests that found a hit
  unsigned ties;                 // walks redone for an exact tie
  unsigned long long* prof;      // step profile (rt_render_step_profile): wave time and count of the
                                 // walk's steps by the set of node kinds they ran (32 bins each)
};
// node kinds of a walk step (the step profile's bin = the set of kinds its lanes were at)
enum : unsigned { K_BOX = 1u, K_WIDE = 2u, K_LEAF = 4u, K_MEDIUM = 8u, K_FRAME = 16u };

// ------------------------------------------------------------------ textures (Lib.hs:441-513)
__device__ __forceinline__ int hmod256(long long a) {  // Haskell `mod` pointCount
  const long long r = a % 256;
  return (int)(r < 0 ? r + 256 : r);
}
__device__ inline double noise(const rt_perlin* P, double sc, V3 p) {  // Lib.hs:441-461
  const V3 q = scale(sc, p);
  const double fi = floor(q.x), fj = floor(q.y), fk = floor(q.z);
  const long long i = (long long)fi, j = (long long)fj, k = (long long)fk;
  const double u = q.x - (double)i, v = q.y - (double)j, w = q.z - (double)k;
  const double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
  double acc = 0.0;
  // perlinInterp's foldr: corner (1,1,1) is added first, (0,0,0) last (Lib.hs:477-484)
#pragma unroll
  for (int idx = 7; idx >= 0; --idx) {
    const int di = (idx >> 2) & 1, dj = (idx >> 1) & 1, dk = idx & 1;
    const int r = P->perm_x[hmod256(i + di)] ^ P->perm_y[hmod256(j + dj)] ^ P->perm_z[hmod256(k + dk)];
    const V3 val = vload(P->ranvec[r]);
    const double I = di, J = dj, K = dk;
    acc = acc + ((I * uu + (1 - I) * (1 - uu)) * (J * vv + (1 - J) * (1 - vv)) * (K * ww + (1 - K) * (1 - ww)) *
                 dot(val, v3(u - I, v - J, w - K)));
  }
  return acc;
}
__device__ inline double turb(const rt_perlin* P, double sc, V3 p) {  // Lib.hs:486-494, depth 7
  double acc = 0.0, weight = 1.0;
  V3 tp = p;
  for (int d = 0; d < 7; ++d) {
    acc = acc + weight * noise(P, sc, tp);
    tp = scale(2.0, tp);
    weight = weight * 0.5;
  }
  return fabs(acc);
}
// marbleTexture's value (Lib.hs:505-507). Not inlined, like sphere_uv: inlined into a render loop, the
// turbulence's 56 unrolled lattice corners and sin's coefficients raise the whole loop's register
// pressure (the full variant: 352 -> ~290 B/lane of scratch); as a call it costs only Perlin hits.
template <bool SL>
__device__ __noinline__ double marble(const rt_perlin* P, double sc, V3 p) {
  return 0.5 * (1.0 + m_sin<SL>(p.z + 10 * turb(P, sc, p)));
}
// textureValue (Lib.hs:496-510); checker chains are followed iteratively.
template <unsigned F>
__device__ inline V3 texture_value(const Scene& S, int tid, double u, double v, V3 p) {
  const rt_texture* t = &S.texs[tid];
  if constexpr (!(F & F_TEX)) return v3(t->f[0], t->f[1], t->f[2]);
  while (t->type == RT_TEX_CHECKER) {
    const bool odd = m_sin<kSL<F>>(10 * p.x) * m_sin<kSL<F>>(10 * p.y) * m_sin<kSL<F>>(10 * p.z) < 0;
    t = &S.texs[odd ? t->a : t->b];
  }
  if (t->type == RT_TEX_CONSTANT) return v3(t->f[0], t->f[1], t->f[2]);
  if (t->type == RT_TEX_PERLIN) return scale(marble<kSL<F>>(&S.perlins[t->a], t->f[0], p), v3(1.0, 1.0, 1.0));
  // RT_TEX_IMAGE
  if (t->a < 0) return v3(0, 1, 1);
  const rt_image im = S.images[t->a];
  const double nxd = (double)t->b;
  double ci = u * nxd;
  ci = ci < 0 ? 0 : (ci > nxd - kEps ? nxd - kEps : ci);
  const double nyd = (double)t->c;
  double cj = (1.0 - v) * nyd - kEps;
  cj = cj < 0 ? 0 : (cj > nyd - kEps ? nyd - kEps : cj);
  const int i = ci == ci ? (int)floor(ci) : 0, j = cj == cj ? (int)floor(cj) : 0;
  const uint8_t* px = S.pool + im.offset + ((long long)j * im.width + i) * 3;
  return v3(px[0] / 255.0, px[1] / 255.0, px[2] / 255.0);  // colorToAlbedo (Lib.hs:294-297)
}

// ------------------------------------------------------------------ primitives
// Unguarded Markstein quotient and the range it is trusted in (see div_exact in rt_device.h).
__device__ __forceinline__ double div_mk(double a, double b, double y) {
  double q = a * y;
  double r = fma(-q, b, a);
  q = fma(r, y, q);
  r = fma(-q, b, a);
  return fma(r, y, q);
}
// quotient and dividend both in the trusted range (divisors are covered by RayX::safe)
__device__ __forceinline__ bool q_ok(double a, double q) { return in_range(a) & in_range(q); }

// boxRayIntersect (Lib.hs:798-814): per axis, [max t0 t_min, min t1 t_max] must be non-empty,
// with the reference's quotients (bit-exact) and GHC max/min. The reference never intersects the
// three axis intervals; with `joint` the box must ALSO pass the joint slab test (max of the axis
// lower bounds < min of the upper bounds). That accepts a subset of the reference's boxes, so it
// only prunes subtrees; what it prunes cannot hold a hit in [t_min, t_max] except exactly on a box
// face (measure zero; tests/test_gpu_parity.py checks closest hits bit for bit).
__device__ __forceinline__ bool box_hit_exact(const double* f, const RayX& r, double t_min, double t_max, bool joint) {
  bool ok = true;
  double lmax = t_min, hmin = t_max;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double o = comp(r.o, a), d = comp(r.d, a);
    const double ta = (f[a] - o) / d;
    const double tb = (f[a + 3] - o) / d;
    const bool lt = ta < tb;
    const double t0 = lt ? ta : tb, t1 = lt ? tb : ta;
    const double lo = gmax(t0, t_min);
    const double hi = gmin(t1, t_max);
    ok = ok && (hi > lo);
    lmax = lo > lmax ? lo : lmax;
    hmin = hi < hmin ? hi : hmin;
  }
  return ok && (!joint || hmin > lmax);
}

// The default (joint) test decided without divisions. When every quotient is finite and
// non-NaN, (reference per-axis test) AND (joint test) is exactly L < U with
// L = max(t_min, min(ta,tb) over axes) and U = min(t_max, max(ta,tb) over axes), and L and U are
// each one of the exact quotients (or t_min / t_max). For a `safe` ray (|o| <= 2^100, every
// non-zero |d| in [2^-900, 2^900] so y = RN(1/d) is normal) q' = n * y is within 2^-51 |q| + 2^-1074 of
// q = RN(n / d), so L', U' are within 2^-50 (|L'| + |U'|) + 2^-1073 of L, U: outside the band
// U' - L' in [-b, b], b = 2^-48 (|L'| + |U'|) (> 2^-1000 whenever the decision is taken), the
// sign of U' - L' is the sign of U - L. An axis with d = 0 has y = +-inf and n * y is its exact
// quotient (+-inf): with the origin inside that slab (-inf, +inf) it does not constrain L or U, as it
// constrains nothing in the reference's per-axis test (t0 = -inf, t1 = +inf); outside it both are +inf
// (or both -inf), so L = +inf (or U = -inf) — and the reference's test of that axis fails (its tmin is
// +inf, or its tmax -inf). No other product is infinite: the host walks a world with a finite box
// coordinate beyond 2^100 with the per-axis test instead (rt_render.hip far_boxes), so |n| < 2^101 and
// |n * y| < 2^1001 (an overflowed product of a finite quotient must not read as +-inf). NaN
// quotients (n = 0: the origin on a slab plane of a zero axis) or banded cases fall through to the exact
// test. Branch-free except for that (rare) fall-through.
__device__ __forceinline__ bool box_hit(const double* f, const RayX& r, double t_min, double t_max, bool joint) {
  if (!joint) return box_hit_exact(f, r, t_min, t_max, false);
  double L = t_min, U = t_max;
  bool nan = false;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double o = comp(r.o, a), y = comp(r.inv, a);
    const double ta = (f[a] - o) * y, tb = (f[a + 3] - o) * y;
    nan |= (ta != ta) | (tb != tb);
    L = fmax(L, fmin(ta, tb));
    U = fmin(U, fmax(ta, tb));
  }
  const double band = 0x1p-48 * (fabs(L) + fabs(U));
  const bool ok_band = (band > 0x1p-1000) & (band < INFINITY);  // (L and U finite)
  // (a NaN bound — the closest hit so far is a rect hit at t = NaN, which rectHit does not reject: a ray
  // in the plane of a face it runs along — makes the reference's per-axis test fail (gmin(t1, NaN) = NaN),
  // while fmin / fmax above would drop it: decided by the exact test)
  nan |= (t_min != t_min) | (t_max != t_max);
  const bool ok = ray_safe(r) & !nan;
  const bool yes = ok & ok_band & (U - L > band);
  const bool no = ok & ((ok_band & (L - U > band)) | (L == INFINITY) | (U == -INFINITY));
  if (!RT_COLD(!(yes | no))) return yes;
  return box_hit_exact(f, r, t_min, t_max, true);
}

// rectHit's t (Lib.hs:1014-1028); plane 0 XY, 1 XZ, 2 YZ. Rejects only t < tmin or t > tmax
// (t == tmax is a hit; a NaN t passes). Returns the t of a hit.
__device__ __forceinline__ bool rect_t(int plane, double i0, double i1, double j0, double j1, double k,
                                       const RayX& r, double t_min, double t_max, double& tout) {
  const int ii = plane == 2 ? 1 : 0, jj = plane == 0 ? 1 : 2, kk = plane == 0 ? 2 : (plane == 1 ? 1 : 0);
  const double num = k - comp(r.o, kk);
  double t = qdiv(num, comp(r.d, kk), comp(r.inv, kk));
  if ((t < t_min) || (t > t_max)) return false;
  const double i = comp(r.o, ii) + t * comp(r.d, ii);
  const double j = comp(r.o, jj) + t * comp(r.d, jj);
  if ((i < i0) || (i > i1) || (j < j0) || (j > j1)) return false;
  tout = t;
  return true;
}
__device__ __forceinline__ void rect_record(int plane, double i0, double i1, double j0, double j1, int mat,
                                            const Ray& r, double t, Hit& h) {
  const int ii = plane == 2 ? 1 : 0, jj = plane == 0 ? 1 : 2;
  const double i = comp(r.o, ii) + t * comp(r.d, ii);
  const double j = comp(r.o, jj) + t * comp(r.d, jj);
  h.t = t;
  h.u = (i - i0) / (i1 - i0);
  h.v = (j - j0) / (j1 - j0);
  h.p = at(r, t);
  const V3 outward = plane == 0 ? v3(0, 0, 1) : (plane == 1 ? v3(0, 1, 0) : v3(1, 0, 0));
  face_normal(r, outward, h.ff, h.n);
  h.mat = mat;
}
// full rectHit (record included), for the light pdf and cuboid faces
__device__ __forceinline__ bool rect_hit(int plane, double i0, double i1, double j0, double j1, double k, int mat,
                                         const RayX& r, double t_min, double t_max, Hit& h) {
  double t;
  if (!rect_t(plane, i0, i1, j0, j1, k, r, t_min, t_max, t)) return false;
  rect_record(plane, i0, i1, j0, j1, mat, plain(r), t, h);
  return true;
}

// hit Sphere's t (Lib.hs:1081-1095): strict tmin < t < tmax, quotients exact.
// hit Sphere's t (Lib.hs:1081-1095): strict tmin < t < tmax, quotients exact.
__device__ __forceinline__ bool sphere_t(V3 sc, double sr, const RayX& r, double t_min, double t_max, double& tout) {
  const V3 oc = r.o - sc;
  const double a = r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z;  // (Lib.hs:1092)
  const double inva = 1.0 / a;
  const double b = dot(oc, r.d);
  const double c = dot(oc, oc) - (sr * sr);
  const double disc = b * b - a * c;
  if (!(disc > 0)) return false;
  const double sd = sqrt(disc);
  const double n1 = (-b) - sd, n2 = (-b) + sd;
  double temp1 = div_mk(n1, a, inva), temp2 = div_mk(n2, a, inva);
  if (RT_COLD(!(in_range(a) & q_ok(n1, temp1) & q_ok(n2, temp2)))) {
    temp1 = ieee_div(n1, a);
    temp2 = ieee_div(n2, a);
  }
  if (t_min < temp1 && temp1 < t_max) tout = temp1;
  else if (t_min < temp2 && temp2 < t_max) tout = temp2;
  else return false;
  return true;
}
// A ConstantMedium's two boundary queries (Lib.hs:1062-1065) on a sphere boundary in one go: t1 = the
// sphere's t over (-inf, inf), t2 = its t over (t1 + eps, inf). Both queries compute the same quotients;
// this evaluates them once and applies the two range tests of sphere_t.
__device__ __forceinline__ bool sphere_t12(V3 sc, double sr, const RayX& r, double& t1, double& t2) {
  const V3 oc = r.o - sc;
  const double a = r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z;
  const double inva = 1.0 / a;
  const double b = dot(oc, r.d);
  const double c = dot(oc, oc) - (sr * sr);
  const double disc = b * b - a * c;
  if (!(disc > 0)) return false;
  const double sd = sqrt(disc);
  const double n1 = (-b) - sd, n2 = (-b) + sd;
  double temp1 = div_mk(n1, a, inva), temp2 = div_mk(n2, a, inva);
  if (RT_COLD(!(in_range(a) & q_ok(n1, temp1) & q_ok(n2, temp2)))) {
    temp1 = ieee_div(n1, a);
    temp2 = ieee_div(n2, a);
  }
  if (-INFINITY < temp1 && temp1 < INFINITY) t1 = temp1;
  else if (-INFINITY < temp2 && temp2 < INFINITY) t1 = temp2;
  else return false;
  const double lo = t1 + kEps;
  if (lo < temp1 && temp1 < INFINITY) t2 = temp1;
  else if (lo < temp2 && temp2 < INFINITY) t2 = temp2;
  else return false;
  return true;
}
// log for hit ConstantMedium's distance draw (Lib.hs:1074). Not inlined, like sphere_uv: the draw happens
// inside the walk, and OCML's fp64 log coefficients held across the render loop cost the full variant
// 304 -> 240 B/lane of scratch (C4 at 100 spp 323.5 -> 306.6 ms: the spill footprint is what
// crowds the scene out of L2).
__device__ __noinline__ double log_call(double x) { return log(x); }

// A sphere hit's (u, v) from its outward normal (Lib.hs:1100-1104). Not inlined: OCML's fp64 atan and
// asin bring polynomial coefficients that, inlined into a render loop, the compiler materialises once
// for the whole loop and spills (the full variant: 560 -> ~290 B/lane of scratch); as a call they are
// materialised per call, and only image-textured hits make it.
template <bool SL>
__device__ __noinline__ void sphere_uv(V3 outward, double& u, double& v) {
  const double phi = ghc_atan2<SL>(outward.z, outward.x);
  const double theta = m_asin<SL>(outward.y);
  u = 1.0 - ((phi + kPi) / (2 * kPi));
  v = (theta + (kPi / 2)) / kPi;
}

// the rest of hit Sphere (Lib.hs:1096-1105)
template <unsigned F>
__device__ __forceinline__ void sphere_record(const Scene& S, V3 sc, double sr, int sm, const Ray& r, double t,
                                              Hit& h) {
  h.t = t;
  h.p = at(r, t);
  const V3 outward = divide(h.p - sc, sr);
  face_normal(r, outward, h.ff, h.n);
  h.mat = sm;
  if ((F & F_UV) || ((F & F_TEX) && S.mats[sm].needs_uv)) {  // u, v only feed image textures
    sphere_uv<kSL<F>>(outward, h.u, h.v);
  } else {
    h.u = 0.0;
    h.v = 0.0;
  }
}
template <unsigned F>
__device__ __forceinline__ bool sphere_hit(const Scene& S, V3 sc, double sr, int sm, const RayX& r, double t_min,
                                           double t_max, Hit& h) {
  double t;
  if (!sphere_t(sc, sr, r, t_min, t_max, t)) return false;
  sphere_record<F>(S, sc, sr, sm, plain(r), t, h);
  return true;
}

// One face of a cuboid (Lib.hs:599-604): face i -> plane and bounds.
__device__ __forceinline__ void cuboid_face(const rt_node* n, int i, int& plane, double& a0, double& a1, double& b0,
                                            double& b1, double& k) {
  const double x0 = n->f[0], y0 = n->f[1], z0 = n->f[2], x1 = n->f[3], y1 = n->f[4], z1 = n->f[5];
  plane = i >> 1;
  a0 = plane == 2 ? y0 : x0;
  a1 = plane == 2 ? y1 : x1;
  b0 = plane == 0 ? y0 : z0;
  b1 = plane == 0 ? y1 : z1;
  k = (i & 1) ? (plane == 0 ? z0 : (plane == 1 ? y0 : x0)) : (plane == 0 ? z1 : (plane == 1 ? y1 : x1));
}

// A cuboid the ray certainly misses within [t_min, t_max] (round 6): the joint slab interval of its box,
// division-free as box_hit computes it, empty by a margin of 2^-40 of the magnitudes involved (the
// quotients' and the faces' in-plane coordinates' roundings are ~2^-52 of them). Then no face can pass
// rectHit (Lib.hs:1014-1028): at a face's t the ray lies in that face's plane, so another axis's slab must
// exclude it, by more than the face test's rounding of that coordinate. Zero direction components give
// +-inf products, exact (outside a slab it is parallel to: L = +inf or U = -inf, and that face pair's t are
// +-inf, out of range); a NaN product (the origin on such a slab's plane), a NaN bound or a ray box_hit
// cannot bound (ray_safe) decides nothing: the six faces decide. Rays that start on a box they are leaving
// (a bounce off a box top) reach its leaf under the 4-wide test's slack and are the common case here.
// Measured (round 6, A/B only): inlined into the walk it raised the C4 kernel's scratch 176 -> 288 B/lane and
// C4 at 100 spp 146.9 -> 166.0 ms (C3 98.6 -> 99.9); out of line, 304 B/lane. Off.
#ifndef RT_CUBOID_PRETEST
#define RT_CUBOID_PRETEST 0
#endif
__device__ __forceinline__ bool cuboid_missed(const double* f, const RayX& r, double t_min, double t_max) {
  double L = t_min, U = t_max, K = 0.0;
  bool nan = (t_min != t_min) | (t_max != t_max);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double o = comp(r.o, a), y = comp(r.inv, a);
    const double ta = (f[a] - o) * y, tb = (f[a + 3] - o) * y;
    nan |= (ta != ta) | (tb != tb);
    L = fmax(L, fmin(ta, tb));
    U = fmin(U, fmax(ta, tb));
    K = fmax(K, isinf(y) ? 0.0 : fabs(o * y));
  }
  const double band = 0x1p-40 * (fabs(L) + fabs(U) + K);
  const bool ok_band = (band > 0x1p-1000) & (band < INFINITY);
  return ray_safe(r) & !nan & ((ok_band & (L - U > band)) | (L == INFINITY) | (U == -INFINITY));
}

// Leaf primitives (Sphere, MovingSphere, Rect{XY,XZ,YZ}, Cuboid): the t of a hit and, for a
// cuboid, which face (`sub`) won. hit Cuboid (Lib.hs:989-1004) is foldr closerHit over the six
// faces, each with the full [tmin, tmax]: the later face keeps a tie.
template <unsigned F>
__device__ __forceinline__ bool prim_t(const Scene& S, const rt_node* n, const RayX& r, double t_min, double t_max,
                                       double& t, int& sub) {
  const int type = n->type & RT_TYPE_MASK;
  sub = 0;
  if (!(F & (F_RECT | F_MOVING)) || type == RT_NODE_SPHERE) return sphere_t(vload(n->f), n->f[3], r, t_min, t_max, t);
  if ((F & F_MOVING) && type == RT_NODE_MOVING_SPHERE) {  // Lib.hs:1106-1108
    const rt_node* e = n + 1;
    const V3 c0 = vload(n->f), c1 = vload(n->f + 3);
    const V3 sc = c0 + scale((r.tm - e->f[0]) / e->f[2], c1 - c0);
    return sphere_t(sc, e->f[3], r, t_min, t_max, t);
  }
  if constexpr (!(F & F_RECT)) return false;
#if RT_CUBOID_TIMING_PROBE
  // (timing probe only, wrong hits: a plain slab test in place of the six faces — the bound on what a
  // cheaper exact cuboid test could save)
  if (type == RT_NODE_CUBOID) {
    double L = t_min, U = t_max;
    for (int a = 0; a < 3; ++a) {
      const double ta = (n->f[a] - comp(r.o, a)) * comp(r.inv, a), tb = (n->f[a + 3] - comp(r.o, a)) * comp(r.inv, a);
      L = fmax(L, fmin(ta, tb));
      U = fmin(U, fmax(ta, tb));
    }
    t = L;
    return L <= U && L > t_min;
  }
#endif
  if (type == RT_NODE_CUBOID) {
    if (RT_CUBOID_PRETEST && cuboid_missed(n->f, r, t_min, t_max)) return false;
    bool have = false;
    for (int i = 5; i >= 0; --i) {
      int plane;
      double a0, a1, b0, b1, k, tt;
      cuboid_face(n, i, plane, a0, a1, b0, b1, k);
      if (rect_t(plane, a0, a1, b0, b1, k, r, t_min, t_max, tt) && (!have || tt < t)) {
        t = tt;
        sub = i;
        have = true;
      }
    }
    return have;
  }
  if (type >= RT_NODE_RECT_XY && type <= RT_NODE_RECT_YZ)
    return rect_t(type - RT_NODE_RECT_XY, n->f[0], n->f[1], n->f[2], n->f[3], n->f[4], r, t_min, t_max, t);
  return false;
}
template <unsigned F>
__device__ __forceinline__ void prim_record(const Scene& S, const rt_node* n, int sub, const Ray& r, double t, Hit& h) {
  const int type = n->type & RT_TYPE_MASK;
  if (!(F & (F_RECT | F_MOVING)) || type == RT_NODE_SPHERE) {
    sphere_record<F>(S, vload(n->f), n->f[3], n->a, r, t, h);
  } else if ((F & F_MOVING) && type == RT_NODE_MOVING_SPHERE) {
    const rt_node* e = n + 1;
    const V3 c0 = vload(n->f), c1 = vload(n->f + 3);
    const V3 sc = c0 + scale((r.tm - e->f[0]) / e->f[2], c1 - c0);
    sphere_record<F>(S, sc, e->f[3], n->a, r, t, h);
  } else if (type == RT_NODE_CUBOID) {
    int plane;
    double a0, a1, b0, b1, k;
    cuboid_face(n, sub, plane, a0, a1, b0, b1, k);
    rect_record(plane, a0, a1, b0, b1, n->a, r, t, h);
  } else {
    rect_record(type - RT_NODE_RECT_XY, n->f[0], n->f[1], n->f[2], n->f[3], n->a, r, t, h);
  }
}

// One instance transform applied to the ray handed to the child (Lib.hs:1029-1031, 1038-1043).
__device__ __forceinline__ Ray enter_instance(const rt_node* n, const Ray& r) {
  if ((n->type & RT_TYPE_MASK) == RT_NODE_TRANSLATE) return Ray{r.o - vload(n->f), r.d, r.tm};
  const int ax = n->b;
  return Ray{unrotate_point(ax, n->f[0], n->f[1], r.o), unrotate_point(ax, n->f[0], n->f[1], r.d), r.tm};
}
// The instance's rewrite of its child's hit; `rc` is the ray the child saw (Lib.hs:1033-1036, 1046-1052).
__device__ __forceinline__ void exit_instance(const rt_node* n, const Ray& rc, Hit& h) {
  if ((n->type & RT_TYPE_MASK) == RT_NODE_TRANSLATE) {
    face_normal(rc, h.n, h.ff, h.n);
    h.p = h.p + vload(n->f);
  } else {
    const int ax = n->b;
    h.p = rotate_point(ax, n->f[0], n->f[1], h.p);
    const V3 rn = rotate_point(ax, n->f[0], n->f[1], h.n);
    face_normal(rc, rn, h.ff, h.n);
  }
}

// A Translate/Rotate chain that ends in a leaf primitive (or the leaf itself), hit as one unit.
template <unsigned F>
__device__ inline bool chain_hit(const Scene& S, int id, const Ray& ray, double t_min, double t_max, Hit& h) {
  Ray r = ray;
  int cur = id, depth = 0;
  if constexpr ((F & F_INST) != 0) {
    while (true) {
      const int type = S.nodes[cur].type & RT_TYPE_MASK;
      if (type != RT_NODE_TRANSLATE && type != RT_NODE_ROTATE) break;
      r = enter_instance(&S.nodes[cur], r);
      cur = S.nodes[cur].a;
      ++depth;
    }
  }
  double t;
  int sub;
  const rt_node* leaf = &S.nodes[cur];
  if (!prim_t<F>(S, leaf, prep(r), t_min, t_max, t, sub)) return false;
  prim_record<F>(S, leaf, sub, r, t, h);
  for (int lv = depth - 1; lv >= 0; --lv) {  // rewrite from the innermost instance outwards
    Ray rl = ray;
    int nd = id;
    for (int k = 0; k < lv; ++k) {
      rl = enter_instance(&S.nodes[nd], rl);
      nd = S.nodes[nd].a;
    }
    const Ray rc = enter_instance(&S.nodes[nd], rl);
    exit_instance(&S.nodes[nd], rc, h);
  }
  return true;
}

// The t of a chain hit only: Translate/Rotate move and rotate the ray, which keeps its parameter,
// so the chain's t is its primitive's t in the innermost frame (the same operations chain_hit runs).
template <unsigned F>
__device__ inline bool chain_t(const Scene& S, int id, const Ray& ray, double t_min, double t_max, double& t) {
  Ray r = ray;
  int cur = id;
  if constexpr ((F & F_INST) != 0) {
    while (true) {
      const int type = S.nodes[cur].type & RT_TYPE_MASK;
      if (type != RT_NODE_TRANSLATE && type != RT_NODE_ROTATE) break;
      r = enter_instance(&S.nodes[cur], r);
      cur = S.nodes[cur].a;
    }
  }
  int sub;
  return prim_t<F>(S, &S.nodes[cur], prep(r), t_min, t_max, t, sub);
}

// chain_t for a ray whose reciprocals are already known (the walk's RayX): a boundary that is a plain
// primitive is tested with them directly — prep() of the same ray gives the same values, so only
// the recomputation is saved (4 fp64 divisions per query); an instance chain transforms the ray.
template <unsigned F>
__device__ __forceinline__ bool chain_tx(const Scene& S, int id, const RayX& rx, double t_min, double t_max,
                                         double& t) {
  if constexpr ((F & F_INST) != 0) {
    const int type = S.nodes[id].type & RT_TYPE_MASK;
    if (type == RT_NODE_TRANSLATE || type == RT_NODE_ROTATE) return chain_t<F>(S, id, plain(rx), t_min, t_max, t);
  }
  int sub;
  return prim_t<F>(S, &S.nodes[id], rx, t_min, t_max, t, sub);
}

// A medium record's occurrence key (rt_bvh.cpp unfold_media: f[1] = key + 1 on the device copy).
__device__ __forceinline__ uint32_t medium_key(const rt_node* n) { return (uint32_t)(n->f[1] - 1.0); }

// hit ConstantMedium (Lib.hs:1053-1080). The boundary is a primitive chain (host-validated); only
// the two boundary hits' t are used. Tier A (R = RngExactT) follows the reference exactly: the draw is
// the column stream's next, made only when the boundary's inside meets [t_min, t_max]. Tier B (RngPhilox,
// kKeyed) redefines the draw as keyed by the walk and the occurrence, and the candidate as unbounded:
// the closest hit is then the least t over all leaves whatever the order (exact ties aside), so media
// worlds walk re-bounded trees like any other.
template <unsigned F, class R>
__device__ inline bool medium_hit(const Scene& S, const rt_node* n, const RayX& rx, double t_min, double t_max, R& g,
                                  Hit& h) {
  const Ray r = plain(rx);
  double t1, t2;
  if (!chain_tx<F>(S, n->a, rx, -INFINITY, INFINITY, t1)) return false;
  if (!chain_tx<F>(S, n->a, rx, t1 + kEps, INFINITY, t2)) return false;
  const double rec1tp = gmax(t_min, t1);
  // tier B (keyed draws): the candidate is computed over the boundary's whole inside and then bounded
  // like any leaf (newt <= t_max), so it does not depend on the bound in force when the walk gets here
  const double rec2t = R::kKeyed ? t2 : gmin(t_max, t2);
  if (rec1tp >= rec2t) return false;
  const double rec1t = rec1tp < 0 ? 0 : rec1tp;
  const double ray_length = vlen(r.d);
  const double dist_inside = (rec2t - rec1t) * ray_length;
  double rnd;
  if constexpr (R::kKeyed) rnd = g.keyed(medium_key(n));
  else rnd = g.draw();
  const double hit_dist = n->f[0] * m_log<R::kSL>(rnd);
  if (hit_dist > dist_inside) return false;
  const double newt = rec1t + (hit_dist / ray_length);
  if (R::kKeyed && !(newt <= t_max)) return false;
  h.t = newt;
  h.p = at(r, newt);
  h.n = v3(1, 0, 0);
  h.u = 0;
  h.v = 0;
  h.ff = 1;
  h.mat = n->b;
  return true;
}

// ------------------------------------------------------------------ traversal
// Closest hit over the DAG rooted at `root` in [t_min, t_max] (hit, Lib.hs:970-1109).
// Depth-first, left child first, each visit bounded by the closest hit so far: exactly the
// reference's recursion (including media draw order). A plain primitive hit at the top level
// records only (t, node, face); its record is built once at the end from the same ray with the
// same operations. Instances whose subtree is not a primitive chain open a frame (a tagged stack
// entry); the frame's rewrite of the hit is applied when the frame closes if the closest hit was
// found inside it. `stk` is this lane's LDS stack (entries `stride` ints apart).
template <unsigned F, class R>
__device__ __forceinline__ bool traverse(const Scene& S, int root, const Ray& wr, double t_min, double t_max,
                                         Hit& best, R& g, int* stk, bool joint, Cnt& cnt, int stride = RT_BLOCK) {
  const RayX wray = prep(wr);
  RayX ray = wray;
  int level = 0;
  unsigned hitmask = 0;
  double closest = t_max;
  int best_node = -1, best_sub = 0;
  bool best_full = false;  // `best` already holds the record
  int sp = 0;
  int node = root;
  for (;;) {
    const rt_node* n = &S.nodes[node & ~RT_IDTAGS];
    const int tf = n->type;
    const int type = tf & RT_TYPE_MASK;
    if (type == RT_NODE_BVH) {
      if constexpr ((F & F_COUNT) != 0) ++cnt.box;
      if (box_hit(n->f, ray, t_min, closest, joint)) {
        // Rebuilt (media-free) trees: visit the child on the ray's side of the split first;
        // the closest hit is order-independent there. Reference trees stay left-first.
        const int c = n->c;
        const bool flip = (c & RT_BVH_ORDERED) && !(c & RT_BVH_MEDIA_FIRST) && comp(ray.d, c & 3) < 0;
        stk[(sp++) * stride] = flip ? n->a : n->b;
        node = flip ? n->b : n->a;
        continue;
      }
    } else if ((F & F_INST) && (type == RT_NODE_TRANSLATE || type == RT_NODE_ROTATE)) {
      if constexpr ((F & F_COUNT) != 0) ++cnt.other;
      if (tf & RT_CHAIN_PRIM) {
        Hit h;
        if (chain_hit<F>(S, node, plain(ray), t_min, closest, h)) {
          best = h;
          closest = h.t;
          best_node = node;
          best_full = true;
          hitmask = (1u << level) - 1u;
        }
      } else {
        stk[(sp++) * stride] = RT_FRAME | node;
        ray = prep(enter_instance(n, plain(ray)));
        ++level;
        node = n->a;
        continue;
      }
    } else if ((F & F_MEDIA) && type == RT_NODE_CONSTANT_MEDIUM) {
      if constexpr ((F & F_COUNT) != 0) ++cnt.other;
      Hit h;
      if (medium_hit<F>(S, n, ray, t_min, closest, g, h)) {
        best = h;
        closest = h.t;
        best_node = node;
        best_full = true;
        hitmask = (1u << level) - 1u;
      }
    } else {
      if constexpr ((F & F_COUNT) != 0) ++cnt.prim;
      double t;
      int sub;
      if (prim_t<F>(S, n, ray, t_min, closest, t, sub)) {
        closest = t;
        best_node = node;
        best_sub = sub;
        best_full = false;
        if ((F & F_INST) && level > 0) {  // inside a frame: the record is needed in this frame's space
          prim_record<F>(S, n, sub, plain(ray), t, best);
          best_full = true;
          hitmask = (1u << level) - 1u;
        }
      }
    }
    // pop
    for (;;) {
      if (sp == 0) {
        if (best_node < 0) return false;
        if (!best_full) prim_record<F>(S, &S.nodes[best_node], best_sub, wr, closest, best);
        return true;
      }
      const int e = stk[(--sp) * stride];
      if (!(F & F_INST) || !(e & RT_FRAME)) {
        node = e;
        break;
      }
      const rt_node* fn = &S.nodes[e & ~RT_FRAME];
      if ((hitmask >> (level - 1)) & 1u) {
        exit_instance(fn, plain(ray), best);
        hitmask &= ~(1u << (level - 1));
      }
      --level;
      Ray pr = wr;  // rebuild the parent's ray from the world ray through the still-open frames
      for (int k = 0; k < sp; ++k) {
        const int f = stk[k * stride];
        if (f & RT_FRAME) pr = enter_instance(&S.nodes[f & ~RT_FRAME], pr);
      }
      ray = prep(pr);
    }
  }
}

// ------------------------------------------------------------------ resumable traversal
// Per-lane LDS slots of the resumable walk over worlds with instance frames (`stride` ints apart):
// the world ray (restored when the last frame closes), the ids of the open frames, and of the
// frames around the best hit (Trav::best_level of them).
// Side ints per lane for frames nesting `frames` deep: the world ray (14), then the open frames and the
// frames around the best hit. The host sizes the dynamic LDS per scene: C4's two-deep frames take 8 ints
// per lane fewer than RT_MAX_FRAMES would. (The world ray's reciprocals stored as well, 6 more ints, would
// spare prep's divisions when the last frame closes, but take C4's kernel past six blocks per CU: 243.8
// -> 250.1 ms at 100 spp.)
__host__ __device__ constexpr int side_ints_for(int frames) { return 14 + 2 * frames; }
constexpr int kSideInts = side_ints_for(RT_MAX_FRAMES);
// The replacement loop's per-lane LDS ints after the walk stack (philox_loop2's layout, launch_philox's
// sizing — one definition for both): Side slots for the frame kernels on the binary / mixed walk (loop
// 1), then, with RT_LANE_LDS (rt_kernels.h), the 4 lane ints (pixel, row, chunk end, depth) of the
// reference-order kernels (RT_LANE_LDS 1) or of every replacement-loop kernel (2).
#ifndef RT_LANE_LDS
#define RT_LANE_LDS 1
#endif
__host__ __device__ constexpr int side_ints_of(unsigned var, int frames, int loop) {
  return ((var & F_FRAMES) && loop == 1) ? side_ints_for(frames) : 0;
}
__host__ __device__ constexpr bool lane_lds_of(unsigned var, int loop) {
  return loop >= 1 && (RT_LANE_LDS >= 2 || (RT_LANE_LDS == 1 && (var & (F_MEDIA | F_FRAMES)) != 0));
}
struct Side {
  int* p;
  int stride;
  int nf = RT_MAX_FRAMES;  // frame slots (the scene's deepest nesting)
  __device__ __forceinline__ void put_d(int i, double x) {
    const long long b = __double_as_longlong(x);
    p[(2 * i) * stride] = (int)(b & 0xffffffff);
    p[(2 * i + 1) * stride] = (int)(b >> 32);
  }
  __device__ __forceinline__ double get_d(int i) const {
    return __hiloint2double(p[(2 * i + 1) * stride], p[(2 * i) * stride]);
  }
  __device__ __forceinline__ void put_ray(const Ray& r) {
    put_d(0, r.o.x), put_d(1, r.o.y), put_d(2, r.o.z), put_d(3, r.d.x), put_d(4, r.d.y), put_d(5, r.d.z);
    put_d(6, r.tm);
  }
  __device__ __forceinline__ Ray get_ray() const {
    return Ray{v3(get_d(0), get_d(1), get_d(2)), v3(get_d(3), get_d(4), get_d(5)), get_d(6)};
  }
  __device__ __forceinline__ int& frame(int i) { return p[(14 + i) * stride]; }
  __device__ __forceinline__ int& best(int i) { return p[(14 + nf + i) * stride]; }
  __device__ __forceinline__ int best(int i) const { return p[(14 + nf + i) * stride]; }
};
// Trav::best_sub of a chain hit (kSubChain | the primitive's face) and of a ConstantMedium hit
constexpr int kSubChain = 0x100, kSubMedium = -2;
// Trav::best_node of a leaf found by the 4-wide walk: its leaf-table slot | kSlotTag, so that the
// record is built from the (LDS-staged) leaf table rather than the flat node array in HBM
constexpr int kSlotTag = 0x40000000;
// Kernels that walk media / instance-frame worlds in the reference's order (only the full variant
// has F_MEDIA and F_FRAMES): there the walk is mixed — the skeleton above media in the reference's
// semantics, re-bounded media-free subtrees (RT_SUB) with tie detection (rt_bvh.cpp
// rebuild_media_skeleton).
template <unsigned F>
constexpr bool kRefMixed = (F & (F_MEDIA | F_FRAMES)) != 0;

// The same depth-first closest-hit walk as `traverse`, one node per call, with its state kept in
// registers between calls (stack in LDS), for worlds without ConstantMedium and without instance
// frames (instances over primitive chains are leaves here). Lets a wave keep every lane busy:
// lanes whose walk has ended are shaded and restarted while the others keep walking.
struct Trav {
  RayX ray;
  double closest;     // closest hit so far
  int node, sp, best_node, best_sub;
  int pend;           // F_WIDE: a postponed leaf (flat node id), -1 = none
  int level;          // F_INST: open instance frames (their ids in the lane's Side slots)
  int best_level;     // F_INST: frames around the best hit (copied to Side::best)
  bool tie;           // another leaf hit at exactly `closest` whose record may shade differently (tie_same):
                      // the walk is redone with `ref`
  bool ref;           // the reference's own walk: caller's tree, left first, bound = closest
  bool redo;          // a tie redo: reference semantics on every node (no RT_SUB subtrees, left
                      // child first even under RT_BVH_ORDERED nodes), so it never flags a tie
  bool lite;          // a tie redo that only picks among the leaves hit at the tied t (trav_redo):
                      // media are not tested
  // F_WIDE: the ray in fp32 for the conservative child-box test (wide_keys2)
  float o32x, o32y, o32z, i32x, i32y, i32z;
  float slack, tmin32, tmax32;  // slack = +inf: the fp32 distances say nothing, accept every child
};

// The leaf-test bound of a walk that flags exact ties: nextafter(closest, +inf) (+inf stays +inf), so
// that a second leaf hit at exactly `closest` is seen. A reference walk
// of a media-free world (a tie redo) bounds by `closest` itself. Derived, not stored (two registers
// fewer across the walk).
template <unsigned F>
__device__ __forceinline__ double closest_up(const Trav& t);

__device__ __forceinline__ float f32_lower(double x) {  // <= x (or -inf)
  const float f = (float)x;
  return f - fabsf(f) * 0x1p-22f;
}
__device__ __forceinline__ float f32_upper(double x) {  // >= x (or +inf)
  const float f = (float)x;
  return f + fabsf(f) * 0x1p-22f;
}

// The ray in fp32 for the conservative child-box test (wide_keys2), from t.ray: the 4-wide walk's
// rays, and in the mixed walk every ray a frame opens or closes (t.tmax32 is left alone: the bound
// is in t units, which the instance transforms keep).
__device__ __forceinline__ void set_ray32(Trav& t, double t_min) {
  t.o32x = (float)t.ray.o.x;
  t.o32y = (float)t.ray.o.y;
  t.o32z = (float)t.ray.o.z;
  t.i32x = (float)t.ray.inv.x;
  t.i32y = (float)t.ray.inv.y;
  t.i32z = (float)t.ray.inv.z;
  // K = max |o * (1/d)| over the finite axes (the origin's rounding, in t units)
  const float kx = isinf(t.i32x) ? 0.0f : fabsf(t.o32x * t.i32x);
  const float ky = isinf(t.i32y) ? 0.0f : fabsf(t.o32y * t.i32y);
  const float kz = isinf(t.i32z) ? 0.0f : fabsf(t.o32z * t.i32z);
  t.slack = fmaxf(fmaxf(kx, ky), kz) * 0x1p-20f;
  t.tmin32 = f32_lower(t_min);
  // 1/d overflowing fp32 for d != 0 (|d| < 2^-126), a NaN direction, a non-finite origin, or
  // t_min <= 0 (wide_key's scaling needs near > 0): the fp32 distances say nothing. All plane
  // distances become 0 and the slack infinite, so every child is entered (leaves decide).
  const bool bad = (isinf(t.i32x) & (t.ray.d.x != 0.0)) | (isinf(t.i32y) & (t.ray.d.y != 0.0)) |
                   (isinf(t.i32z) & (t.ray.d.z != 0.0)) | isnan(t.i32x) | isnan(t.i32y) | isnan(t.i32z) |
                   !isfinite(t.o32x) | !isfinite(t.o32y) | !isfinite(t.o32z) | isnan(t.slack) |
                   !(t.tmin32 > 0.0f);
  // A ray with a NaN in its origin or direction (the next segment after a rect hit at t = NaN:
  // trav_take) hits nothing in the reference — its root box test fails (a NaN slab quotient) — and
  // here no child is entered (slack -inf): accepting every child instead walked the whole tree for
  // each such segment (a 400-box field alone: 745 4-wide nodes and 2200 leaf tests per sample), and a
  // rect leaf would have taken its t = NaN.
  const bool dead = (t.ray.o.x != t.ray.o.x) | (t.ray.o.y != t.ray.o.y) | (t.ray.o.z != t.ray.o.z) |
                    (t.ray.d.x != t.ray.d.x) | (t.ray.d.y != t.ray.d.y) | (t.ray.d.z != t.ray.d.z);
  t.o32x = bad ? 0.0f : t.o32x;
  t.o32y = bad ? 0.0f : t.o32y;
  t.o32z = bad ? 0.0f : t.o32z;
  t.i32x = bad ? 0.0f : t.i32x;
  t.i32y = bad ? 0.0f : t.i32y;
  t.i32z = bad ? 0.0f : t.i32z;
  t.slack = dead ? -INFINITY : (bad ? INFINITY : t.slack);
}

// The mixed walk refreshes the fp32 origin and reciprocals from the fp64 ray at each wide step instead
// of carrying them across the walk (six registers fewer in the full variant: 240 -> 192 B/lane of
// scratch); `slack` (carried) is +-inf exactly for the rays set_ray32 zeroes.
__device__ __forceinline__ void refresh_ray32(Trav& t) {
  const bool bad = isinf(t.slack);
  t.o32x = bad ? 0.0f : (float)t.ray.o.x;
  t.o32y = bad ? 0.0f : (float)t.ray.o.y;
  t.o32z = bad ? 0.0f : (float)t.ray.o.z;
  t.i32x = bad ? 0.0f : (float)t.ray.inv.x;
  t.i32y = bad ? 0.0f : (float)t.ray.inv.y;
  t.i32z = bad ? 0.0f : (float)t.ray.inv.z;
}

template <unsigned F>
__device__ __forceinline__ void trav_begin(Trav& t, const Ray& r, int root, double t_min, double t_max) {
  t.ray = prep(r);
  t.closest = t_max;
  t.node = root;
  t.sp = 0;
  t.best_node = -1;
  t.best_sub = 0;
  t.pend = -1;
  t.level = 0;
  t.best_level = 0;
  t.tie = false;
  t.ref = false;
  t.redo = false;
  t.lite = false;
  if constexpr ((F & F_WIDE) != 0) t.node = 0;  // wide root
  if constexpr (kRay32<F>) {
    set_ray32(t, t_min);
    t.tmax32 = f32_upper(t_max);
  }
}

template <unsigned F>
__device__ __forceinline__ double closest_up(const Trav& t) {
  const double c = t.closest;
  const long long b = __double_as_longlong(c);
  const double up = isinf(c) ? c : (c > 0 ? __longlong_as_double(b + 1) : (c < 0 ? __longlong_as_double(b - 1) : 0x1p-1074));
  return (!kRefMixed<F> && t.ref) ? t.closest : up;
}

// Redo the walk as the reference does it: the caller's tree, left child first, every accepted hit
// replacing the best under bound = closest. `redo` (a walk redone for an exact tie) applies those
// semantics to every node: a caller's tree may itself hold RT_BVH_ORDERED nodes (rt_rebuild_bvh
// output uploaded again), which in the first walk of a mixed world mark re-bounded subtrees whose
// leaves flag ties — in a redo that would flag the same tie again, forever.
__device__ __forceinline__ void trav_restart_ref(Trav& t, int root, double t_max, bool redo = false) {
  t.node = root;
  t.sp = 0;
  t.closest = t_max;
  t.best_node = -1;
  t.best_sub = 0;
  t.pend = -1;
  t.level = 0;
  t.best_level = 0;
  t.tie = false;
  t.ref = true;
  t.redo = redo;
  t.lite = false;
  t.tmax32 = f32_upper(t_max);  // (mixed walks: the wide subtrees' bound)
}

// A walk that flagged an exact tie at t* = closest is redone as the reference does it, to pick the leaf
// the reference's order picks among those hit at exactly t*. Tier-B media draws are keyed by walk and
// occurrence (RngPhilox::keyed), so a redo repeats them without rewinding anything. The redo starts
// bounded by nextafter(t*) (`lite`): a box test at that bound gives the outcome it gives at any larger
// bound for every box the ray enters by t*, and what it culls holds no leaf hit at t*; the first leaf hit
// at t* is accepted as under the reference's larger bound, and from then on the bound is t* itself, as in
// the reference. A walk whose closest hit is a medium's (a tie there needs a surface at exactly that
// random t) or a rect hit at t = NaN (trav_take) is redone in full.
// (Kernels for media-free worlds, where ties are rare — C2 none, C3 0.015 per sample — redo in full:
// the lighter redo's extra state cost the 4-wave spheres kernel 3.5 %.)
template <unsigned F>
__device__ __forceinline__ void trav_redo(Trav& t, int root, double t_max) {
  if constexpr (!kRefMixed<F>) {
    trav_restart_ref(t, root, t_max, true);
    return;
  }
  if (t.best_sub == kSubMedium || t.lite) {
    trav_restart_ref(t, root, t_max, true);
    return;
  }
  const double c = t.closest;
  const double up = __longlong_as_double(__double_as_longlong(c) + (c > 0 ? 1 : -1));
  trav_restart_ref(t, root, up < t_max ? up : t_max, true);  // (t* == t_max: the reference's own bound)
  t.lite = true;
}

// Leaf of the resumable walk (a primitive, or an instance chain ending in one). Leaves are tested
// under the bound closest_up, so a hit at exactly `closest` is seen: the reference keeps the
// first such leaf in its tree's depth-first order unless a later one accepts t == tmax (rects,
// Lib.hs:1005-1028, vs spheres' strict t < tmax), an order this walk does not follow — such a
// tie is flagged, and the caller redoes the walk as the reference does it (trav_restart_ref).
// Exact ties need two surfaces through one point on the ray (e.g. the book-one glass sphere
// resting on the ground at (0,0,0)); they are rare, so the redo costs nothing measurable.
// `refsem`: the reference's own semantics for this leaf (a ref walk outside any re-bounded
// subtree): its bound is `closest` and every accepted hit replaces, as hit BVHNode prefers the
// right child's hit. Otherwise the bound is closest_up and an exact tie is flagged.
// Which face of which material a plain rect / cuboid leaf's hit is on: plane (0 XY, 1 XZ, 2 YZ) and
// material id; -1 for every other leaf (spheres, moving spheres).
__device__ __forceinline__ int face_sig(const rt_node* n, int sub) {
  const int type = n->type & RT_TYPE_MASK;
  const int plane = type == RT_NODE_CUBOID ? (sub >> 1) : type - RT_NODE_RECT_XY;
  return (type == RT_NODE_CUBOID || (type >= RT_NODE_RECT_XY && type <= RT_NODE_RECT_YZ)) ? plane | (n->a << 2) : -1;
}
// An exact tie needs no redo when the tied leaves' hit records shade identically: two rect faces (plain
// rects or cuboid faces, outside instance frames) on the same plane orientation with the same material,
// whose texture does not read (u, v). Their records then agree in t, p (the same ray at the same t),
// outward normal, hence front_face and normal (faceNormal, Lib.hs:1111-1117), and material; u and v
// differ but reach nothing (textureValue of a (u, v)-free texture). Whichever of them the reference's
// order picks (Lib.hs:971-1004), the rest of the path — its draws and its colour — is the same. (Such
// ties are what the +x light direction of the Lambertian quirk produces along the box field of
// next_week_final: a box's +x face and its neighbour's -x face in one plane)
// Debug kernels (F_UV) compare u, v too: there every tie is redone.
template <unsigned F>
constexpr bool kTieSameOk = (F & F_RECT) != 0 && (F & F_UV) == 0;
template <unsigned F>
__device__ __forceinline__ bool tie_same(const Scene& S, const Trav& t, const rt_node* n, int sub, bool plain) {
  if constexpr (!kTieSameOk<F>) return false;
  int best_level = 0;
  if constexpr ((F & F_FRAMES) != 0) best_level = t.best_level + t.level;
  if (!plain || best_level != 0 || t.best_node < 0 || (t.best_sub & kSubChain) || t.best_sub == kSubMedium) return false;
  const rt_node* b = ((F & (F_WIDE | F_MIXW)) && (t.best_node & kSlotTag)) ? &S.leaves[t.best_node & ~kSlotTag]
                                                                          : &S.nodes[t.best_node];
  const int sig = face_sig(n, sub);
  return sig >= 0 && sig == face_sig(b, t.best_sub) && !S.mats[n->a].needs_uv;
}

template <unsigned F>
__device__ __forceinline__ void trav_take(const Scene& S, Trav& t, double x, int id, int sub, Side& side, bool refsem,
                                          const rt_node* leaf, bool plain) {
  // A rect hit at t = NaN (a ray in the plane of a face it runs along — the Lambertian quirk's +x ray
  // from a point exactly on a box top: rectHit rejects only t < tmin or t > tmax, Lib.hs:1014-1015) is
  // taken like a closer hit, as the reference takes it; the reference keeps it, or replaces it, by its
  // own tree order (every later test against a NaN bound: boxes fail, rects pass). The walk ends here
  // (closest_up(NaN) is 2^-1074, tmax32 0) and is flagged for a full redo in the reference's order
  // (trav_redo): by `tie`, and in walks that mix reference-semantics leaves (kRefMixed), whose later
  // replacement of the NaN clears `tie`, by `lite` too. (No branch
  // of its own: as one, never taken, it cost the Cornell kernel 3 %.)
  const bool nan_t = (F & F_RECT) != 0 && x != x;
  if (refsem || x < t.closest || nan_t) {
    // (a tie at the old closest no longer matters: only leaves hit at the final closest t compete, and
    // the bound the walk carried on with was the same whichever tied leaf won)
    t.tie = nan_t;
    if constexpr ((F & F_RECT) != 0 && kRefMixed<F>) t.lite = t.lite | nan_t;
    t.closest = x;
    t.best_node = id;
    t.best_sub = sub;
    if constexpr ((F & F_FRAMES) != 0) {
      t.best_level = t.level;
      for (int k = 0; k < t.level; ++k) side.best(k) = side.frame(k);
    }
    if constexpr (kRay32<F>) t.tmax32 = nan_t ? 0.0f : f32_upper(x);
  } else if (x == t.closest && id != t.best_node) {  // (the same leaf twice is no tie)
    // (a tie whose records shade identically needs no redo: tie_same)
    if (!tie_same<F>(S, t, leaf, sub, plain)) t.tie = true;
  }
}
// A hoisted medium's tier-B candidate (RT_BVH_MEDIA_FIRST, rt_bvh.cpp): exactly the walk's medium leaf
// (trav_leaf: boundary queries over (-inf, inf) and (t1 + eps, inf), the keyed draw, OCML's log), or -1
// when the ray draws no hit in it (a candidate is >= t_min > 0), or — `bound`, the walk's closest hit when
// the media are taken after it (RT_MEDIA_AFTER) — when the candidate is certainly beyond `bound`, which
// trav_take would not take anyway. That is decided without the fp64 log where an fp32 lower bound of the
// drawn distance already exceeds the room left (below); otherwise the exact expression decides.
// (measured neutral with the media taken in the prelude, C4 at 100 spp 165.1-166.9 vs 165.4-166.4 ms: off)
#ifndef RT_LOG_PREFILTER
#define RT_LOG_PREFILTER 0
#endif
template <unsigned F>
__device__ __forceinline__ double hoisted_medium_t(const rt_node* nodes, int id, RayX rx, double t_min, uint32_t k0,
                                                uint32_t k1, uint32_t walk, uint32_t sample, uint32_t pid,
                                                double bound = INFINITY) {
  Scene S{};
  S.nodes = nodes;
  const rt_node* n = &nodes[id];
  double t1, t2;
  const rt_node* bd = &nodes[n->a];
  if (bd->type == RT_NODE_SPHERE) {  // (one quadratic for both boundary queries)
    if (!sphere_t12(vload(bd->f), bd->f[3], rx, t1, t2)) return -1.0;
  } else {
    if (!chain_tx<F>(S, n->a, rx, -INFINITY, INFINITY, t1)) return -1.0;
    if (!chain_tx<F>(S, n->a, rx, t1 + kEps, INFINITY, t2)) return -1.0;
  }
  const double rec1tp = gmax(t_min, t1);
  if (rec1tp >= t2) return -1.0;
  const double rec1t = rec1tp < 0 ? 0 : rec1tp;
  const double ray_length = vlen(rx.d);
  const double dist_inside = (t2 - rec1t) * ray_length;
  const double rnd = RngPhilox::keyed_at(k0, k1, walk, sample, pid, medium_key(n));
  // The log skipped where it cannot matter (round 6): hit_dist = |f0| * (-log rnd), f0 = -1/density. With
  // r32 >= rnd (fp32, rounded up) -log(r32) <= -log(rnd), and OCML's logf is within 2 ulp (2^-22 relative), so
  // lo = |f0| * (-logf(r32)) * (1 - 2^-20) <= hit_dist. The candidate is used only when hit_dist <= dist_inside
  // and rec1t + hit_dist / ray_length <= bound; lo beyond both (the second with a relative slack of 2^-30 and
  // an absolute one of 2^-40 (|rec1t| + |bound|) ray_length, for the roundings of the quotient and the sum)
  // rejects it exactly as the fp64 expression would. A thin fog's mean free path is far beyond most walks'
  // closest hits (next_week_final's whole-scene fog: 10 000 units against hits ~100 away), so most draws end
  // here.
  if (RT_LOG_PREFILTER) {
    float r32 = (float)rnd;
    r32 = (double)r32 < rnd ? __int_as_float(__float_as_int(r32) + 1) : r32;
    const double lo = fabs(n->f[0]) * (double)(-logf(r32)) * (1.0 - 0x1p-20);
    const double room = fmin(dist_inside, (bound - rec1t) * ray_length * (1.0 + 0x1p-30) +
                                              0x1p-40 * (fabs(rec1t) + fabs(bound)) * ray_length);
    if (lo > room) return -1.0;
  }
  const double hit_dist = n->f[0] * log_call(rnd);  // (not inlined: log_call)
  if (hit_dist > dist_inside) return -1.0;
  return rec1t + (hit_dist / ray_length);
}
// RT_MEDIA_AFTER (round 6, A/B only: measured slower, C4 at 100 spp 158.4 vs 145.4-147.6 ms — without the
// media's bound the walks visit 10 % more nodes, 33.2 vs 30.1 wide nodes per sample): a world's hoisted
// media are taken when the walk over the rest of the
// world has ended (media_after, at the closest hit the walk found) instead of where it starts (the prelude,
// trav_media_first): the candidate is the same number (the keyed draw names the walk by the stream words
// consumed, which no walk changes), the closest hit is the least t either way and a medium candidate at exactly
// a surface's t is flagged as a tie either way (trav_take), but at the end the bound is known, so most draws
// skip the fp64 log (hoisted_medium_t). The walk then starts below the chain (media_rest).
#ifndef RT_MEDIA_AFTER
#define RT_MEDIA_AFTER 0
#endif
template <unsigned F>
__device__ __forceinline__ int media_rest(const Scene& S, int node) {
  if constexpr ((F & F_MEDIA) != 0 && RT_MEDIA_AFTER) {
    for (;;) {
      if (!(node >= 0 && (node & (RT_WNODE | RT_IDTAGS)) == RT_ISBOX)) return node;
      const rt_node* n = &S.nodes[node & ~(RT_SUB | RT_IDTAGS)];
      if (!(n->c & RT_BVH_MEDIA_FIRST)) return node;
      node = n->b | RT_SUB;  // (the rest: below an ordered node, a re-bounded subtree)
    }
  }
  return node;
}
// The hoisted media chain from `node` (S.world): each medium's candidate offered to trav_take like a leaf of a
// re-bounded subtree, without the chain's box tests (they only cull; the medium tests are exact). `after`:
// the walk over the rest has ended (t.closest is its closest hit, t.node is not touched); else the prelude,
// which leaves t.node at the rest.
template <unsigned F, class R>
__device__ __forceinline__ void media_chain(const Scene& S, Trav& t, double t_min, Cnt& cnt, const R& g, Side& side,
                                            int node, bool after) {
  if constexpr ((F & F_MEDIA) != 0 && R::kKeyed) {
    // A ray with a NaN in its origin or direction (the segment after a rect hit at t = NaN) hits nothing
    // in the reference: its root box test fails (a NaN slab quotient, Lib.hs:798-814), so it never
    // reaches a medium. The chain's box tests are skipped here, and a rect or cuboid boundary's t would be
    // NaN, which the medium's range tests pass (a finite candidate): such a ray takes no candidate (ADVICE
    // r5; the rest of the walk rejects it, set_ray32).
    const bool dead = (t.ray.o.x != t.ray.o.x) | (t.ray.o.y != t.ray.o.y) | (t.ray.o.z != t.ray.o.z) |
                      (t.ray.d.x != t.ray.d.x) | (t.ray.d.y != t.ray.d.y) | (t.ray.d.z != t.ray.d.z);
    for (;;) {
      if (!(node >= 0 && (node & (RT_WNODE | RT_IDTAGS)) == RT_ISBOX)) break;
      const rt_node* n = &S.nodes[node & ~(RT_SUB | RT_IDTAGS)];
      if (!(n->c & RT_BVH_MEDIA_FIRST)) break;
      const int m = n->a & ~RT_IDTAGS;
      if constexpr ((F & F_COUNT) != 0) ++cnt.other;
      // (a NaN closest hit — a rect hit at t = NaN, flagged for a redo — takes no medium: x <= NaN is false)
      const double x = dead ? -1.0
                            : hoisted_medium_t<F>(S.nodes, m, t.ray, t_min, g.k0, g.k1, g.consumed(), g.sample, g.pid,
                                                  after ? t.closest : INFINITY);
      if (x >= 0.0 && x <= t.closest) trav_take<F>(S, t, x, m, kSubMedium, side, false, &S.nodes[m], false);
      node = n->b | RT_SUB;
    }
    if (!after) t.node = node;
  }
}
// The walk's prelude (RT_MEDIA_AFTER=0; tier B, worlds with hoisted media): the chain at the top of the world
// taken where lanes start their walks together, so that the walk starts at the rest already bounded by the
// media.
template <unsigned F, class R>
__device__ __forceinline__ void trav_media_first(const Scene& S, Trav& t, double t_min, Cnt& cnt, const R& g,
                                                 Side& side) {
  if constexpr (!RT_MEDIA_AFTER) media_chain<F>(S, t, t_min, cnt, g, side, t.node, false);
}
// RT_MEDIA_AFTER: the chain taken at the end of a first walk (not a tie redo, which walks the caller's tree,
// media included), before the tie check.
template <unsigned F, class R>
__device__ __forceinline__ void media_after(const Scene& S, Trav& t, double t_min, Cnt& cnt, const R& g, Side& side) {
  if constexpr (RT_MEDIA_AFTER) media_chain<F>(S, t, t_min, cnt, g, side, S.world, true);
}
// A leaf: a primitive, an instance chain ending in one (its t and face only: the record is built once,
// in trav_finish), or a ConstantMedium (ref walks only: its one draw happens here, in the reference's
// order and under its bound, Lib.hs:1053-1080). The three kinds share ONE inlined primitive test
// (prim_t): a chain or a medium's boundary chain first carries the ray down to its primitive (the
// transforms keep the ray parameter, chain_t), a medium queries its boundary twice (t1 over
// (-inf, inf), then t2 over (t1 + eps, inf)), so a kernel holds one copy of the primitive code in its
// walk instead of six.
template <unsigned F, class R>
__device__ __forceinline__ void trav_leaf(const Scene& S, Trav& t, const rt_node* n, int id, double t_min, Cnt& cnt,
                                          R& g, Side& side, bool refsem) {
#ifndef RT_COMPACT_SLEAF
#define RT_COMPACT_SLEAF 1
#endif
  if constexpr ((F & F_QNODE) != 0 || ((F & F_SLEAF) != 0 && RT_COMPACT_SLEAF)) {
    if (id & kSlotTag) {  // a leaf-table slot of a spheres-only world: its (center, radius) quadruple
      if constexpr ((F & F_COUNT) != 0) ++cnt.prim;
      const double2* q = reinterpret_cast<const double2*>(S.sleaves + 4 * (size_t)(id & ~kSlotTag));
      const double2 c01 = q[0], c2r = q[1];
      double tt;
      if (!sphere_t(v3(c01.x, c01.y, c2r.x), c2r.y, t.ray, t_min, refsem ? t.closest : closest_up<F>(t), tt)) return;
      if constexpr ((F & F_COUNT) != 0) ++cnt.phit;
      trav_take<F>(S, t, tt, id, 0, side, refsem, n, true);
      return;
    }
  }
  const int type = n->type & RT_TYPE_MASK;
  const bool chain = (F & F_INST) && (type == RT_NODE_TRANSLATE || type == RT_NODE_ROTATE);
  const bool medium = (F & F_MEDIA) && type == RT_NODE_CONSTANT_MEDIUM;  // (always on the skeleton: refsem)
  // (a stream-drawn medium's redo picks among surfaces at the tied t: trav_redo; keyed media are tested)
  if (kRefMixed<F> && !R::kKeyed && medium && t.lite) return;
  if constexpr ((F & F_COUNT) != 0) {
    if (chain || medium) ++cnt.other;
    else ++cnt.prim;
  }
  const rt_node* p = n;
  RayX rx = t.ray;
  if constexpr ((F & (F_INST | F_MEDIA)) != 0) {
    if (chain || medium) {
      // (a chain is walked in the flat node array; a leaf of the 4-wide walk carries its flat id in c)
      int cur = medium ? n->a : ((id & kSlotTag) ? n->c : id);
      if constexpr ((F & F_INST) != 0) {
        int ty = S.nodes[cur].type & RT_TYPE_MASK;
        if (ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE) {
          Ray r = plain(t.ray);
          do {
            r = enter_instance(&S.nodes[cur], r);
            cur = S.nodes[cur].a;
            ty = S.nodes[cur].type & RT_TYPE_MASK;
          } while (ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE);
          rx = prep(r);
        }
      }
      p = &S.nodes[cur];
    }
  }
  double lo = medium ? -INFINITY : t_min;
  const double hi = medium ? INFINITY : (refsem ? t.closest : closest_up<F>(t));
  double tt = 0.0, t1 = 0.0;
  int sub = 0;
  bool ok;
#pragma nounroll
  for (int q = 0;; ++q) {
    ok = prim_t<F>(S, p, rx, lo, hi, tt, sub);
    if (!(medium && ok && q == 0)) break;
    t1 = tt;  // hit ConstantMedium's first boundary query; the second starts just past it
    lo = t1 + kEps;
  }
  if (!ok) return;
  if (!medium) {
    if constexpr ((F & F_COUNT) != 0) cnt.phit += !chain;
    trav_take<F>(S, t, tt, id, chain ? (kSubChain | sub) : sub, side, refsem, p, !chain);
    return;
  }
  if constexpr ((F & F_MEDIA) != 0) {  // the rest of hit ConstantMedium (Lib.hs:1062-1080; medium_hit)
    const Ray r = plain(t.ray);
    const double rec1tp = gmax(t_min, t1);
    const double rec2t = R::kKeyed ? tt : gmin(t.closest, tt);
    if (rec1tp >= rec2t) return;
    const double rec1t = rec1tp < 0 ? 0 : rec1tp;
    const double ray_length = vlen(r.d);
    const double dist_inside = (rec2t - rec1t) * ray_length;
    double rnd;
    if constexpr (R::kKeyed) rnd = g.keyed(medium_key(n));
    else rnd = g.draw();
    const double hit_dist = n->f[0] * log_call(rnd);
    if (hit_dist > dist_inside) return;
    const double x = rec1t + (hit_dist / ray_length);
    if constexpr (R::kKeyed) {
      // bounded like any leaf: accepted at x <= closest (a medium in a re-bounded subtree at exactly
      // closest is an exact tie, redone in the reference's order)
      if (!(x <= t.closest)) return;
      trav_take<F>(S, t, x, id, kSubMedium, side, refsem, n, false);
    } else {
      trav_take<F>(S, t, x, id, kSubMedium, side, true, n, false);
    }
  }
}

// Conservative fp32 slab test of the child boxes (two at a time in packed fp32). Each plane
// distance (plane - o32) * i32 is within eps*(K + 3|t|) of the exact distance to the fp32 box
// (eps = 2^-24, K = max |o * (1/d)| over finite axes; the fp32 box contains the fp64 one). With
// near >= tmin > 0, the test near*(1 - 2^-21) <= far*(1 + 2^-21) + 2^-20*K accepts every ray
// whose exact slab interval over the box meets [tmin, tmax]: for far >= 0 the relative margin
// covers 3eps(|near| + |far|) and the slack 2eps*K; a computed far < 0 with an exact far >= tmin
// means far <= eps*K, which the slack covers. A zero direction component gives i32 = +-inf: its
// distances are +-inf (origin outside the slab: near = +inf or far = -inf, rejected; inside:
// no constraint), or NaN exactly when the origin lies on the plane, which fmaxf/fminf (IEEE
// maxNum/minNum) drop — the plane then does not constrain, as for a ray inside the slab.
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void wide_keys2(const Trav& t, f32x2 nx, f32x2 ny, f32x2 nz, f32x2 fx, f32x2 fy, f32x2 fz,
                                           float& k0, float& k1) {
  const f32x2 ox = {t.o32x, t.o32x}, oy = {t.o32y, t.o32y}, oz = {t.o32z, t.o32z};
  const f32x2 ix = {t.i32x, t.i32x}, iy = {t.i32y, t.i32y}, iz = {t.i32z, t.i32z};
  const f32x2 tnx = (nx - ox) * ix, tny = (ny - oy) * iy, tnz = (nz - oz) * iz;
  const f32x2 tfx = (fx - ox) * ix, tfy = (fy - oy) * iy, tfz = (fz - oz) * iz;
  const float n0 = fmaxf(fmaxf(tnx.x, tny.x), fmaxf(tnz.x, t.tmin32));
  const float n1 = fmaxf(fmaxf(tnx.y, tny.y), fmaxf(tnz.y, t.tmin32));
  const float f0 = fminf(fminf(tfx.x, tfy.x), fminf(tfz.x, t.tmax32));
  const float f1 = fminf(fminf(tfx.y, tfy.y), fminf(tfz.y, t.tmax32));
  const bool h0 = n0 * (1.0f - 0x1p-21f) <= fmaf(f0, 1.0f + 0x1p-21f, t.slack);
  const bool h1 = n1 * (1.0f - 0x1p-21f) <= fmaf(f1, 1.0f + 0x1p-21f, t.slack);
  k0 = h0 ? fminf(n0, 3.0e38f) : INFINITY;
  k1 = h1 ? fminf(n1, 3.0e38f) : INFINITY;
}

__device__ __forceinline__ void cswap(float& ka, int& ca, float& kb, int& cb) {
  const bool s = kb < ka;
  const float k = s ? kb : ka;
  const int c = s ? cb : ca;
  kb = s ? ka : kb;
  cb = s ? ca : cb;
  ka = k;
  ca = c;
}

// The four planes of one axis of a quantised node (rt_qnode): origin + q * scale, exact in fp32.
__device__ __forceinline__ float4 qplanes(uint32_t q, float s, float o) {
  return float4{fmaf((float)(q & 255u), s, o), fmaf((float)((q >> 8) & 255u), s, o),
                fmaf((float)((q >> 16) & 255u), s, o), fmaf((float)(q >> 24), s, o)};
}

// One wide node (index `w`): test the four child boxes, enter the nearest accepted child, stack the
// others (farthest deepest). F_QNODE: the node is read in its quantised form (64 bytes) and its planes
// decoded; the test over them is the same.
template <unsigned F = 0, class STK>
__device__ __forceinline__ bool wide_node(const Scene& S, Trav& t, STK* stk, int stride, int w, bool all = false) {
  float4 nx, ny, nz, fx, fy, fz;
  int4 ch;
  if constexpr ((F & F_QNODE) != 0) {
    const uint4* qb = reinterpret_cast<const uint4*>(&S.qnodes[w]);
    const uint4 a = qb[0], b = qb[1], c = qb[2];
    const uint4 d = qb[3];
    ch = int4{(int)d.x, (int)d.y, (int)d.z, (int)d.w};
    const float ox = __uint_as_float(a.x), oy = __uint_as_float(a.y), oz = __uint_as_float(a.z);
    const float sx = __uint_as_float(a.w), sy = __uint_as_float(b.x), sz = __uint_as_float(b.y);
    // (qlo x, y, z = b.z, b.w, c.x; qhi x, y, z = c.y, c.z, c.w; a ray towards -axis: hi is the near plane)
    const bool mx = signbit(t.i32x), my = signbit(t.i32y), mz = signbit(t.i32z);
    nx = qplanes(mx ? c.y : b.z, sx, ox);
    fx = qplanes(mx ? b.z : c.y, sx, ox);
    ny = qplanes(my ? c.z : b.w, sy, oy);
    fy = qplanes(my ? b.w : c.z, sy, oy);
    nz = qplanes(mz ? c.w : c.x, sz, oz);
    fz = qplanes(mz ? c.x : c.w, sz, oz);
  } else {
    const float* base = reinterpret_cast<const float*>(&S.wnodes[w]);
    // (a ray running towards -axis a has the box's hi as its near plane on that axis)
    const int ox = signbit(t.i32x) ? 12 : 0, oy = signbit(t.i32y) ? 16 : 4, oz = signbit(t.i32z) ? 20 : 8;
    nx = *reinterpret_cast<const float4*>(base + ox);
    ny = *reinterpret_cast<const float4*>(base + oy);
    nz = *reinterpret_cast<const float4*>(base + oz);
    fx = *reinterpret_cast<const float4*>(base + (ox ^ 12));
    fy = *reinterpret_cast<const float4*>(base + (oy < 12 ? oy + 12 : oy - 12));
    fz = *reinterpret_cast<const float4*>(base + (oz < 12 ? oz + 12 : oz - 12));
    ch = *reinterpret_cast<const int4*>(base + 24);
  }
  float k0, k1, k2, k3;
  wide_keys2(t, f32x2{nx.x, nx.y}, f32x2{ny.x, ny.y}, f32x2{nz.x, nz.y}, f32x2{fx.x, fx.y}, f32x2{fy.x, fy.y},
             f32x2{fz.x, fz.y}, k0, k1);
  wide_keys2(t, f32x2{nx.z, nx.w}, f32x2{ny.z, ny.w}, f32x2{nz.z, nz.w}, f32x2{fx.z, fx.w}, f32x2{fy.z, fy.w},
             f32x2{fz.z, fz.w}, k2, k3);
  int c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
  const int n_hit = (k0 < INFINITY) + (k1 < INFINITY) + (k2 < INFINITY) + (k3 < INFINITY);
  cswap(k0, c0, k1, c1);
  cswap(k2, c2, k3, c3);
  cswap(k0, c0, k2, c2);
  cswap(k1, c1, k3, c3);
  cswap(k1, c1, k2, c2);
  if ((F & F_W8) && all) {
    // (F_W8's farther half: every accepted child stacked, farthest deepest, four slots written — the
    // stacks have 4 entries of headroom under F_W8)
    const int a0 = n_hit > 3 ? c3 : (n_hit > 2 ? c2 : (n_hit > 1 ? c1 : c0));
    const int a1 = n_hit > 3 ? c2 : (n_hit > 2 ? c1 : c0);
    const int a2 = n_hit > 3 ? c1 : c0;
    stk[t.sp * stride] = a0;
    stk[(t.sp + 1) * stride] = a1;
    stk[(t.sp + 2) * stride] = a2;
    stk[(t.sp + 3) * stride] = c0;
    t.sp += n_hit;
    return n_hit != 0;
  }
  // Stack the accepted children after c0 without branches, farthest deepest: three slots are always
  // written (slots at or above the new sp are dead; the stacks have 3 entries of headroom for this).
  const int e0 = n_hit > 3 ? c3 : (n_hit > 2 ? c2 : c1);
  const int e1 = n_hit > 3 ? c2 : c1;
  stk[t.sp * stride] = e0;
  stk[(t.sp + 1) * stride] = e1;
  stk[(t.sp + 2) * stride] = c1;
  t.sp += n_hit > 1 ? n_hit - 1 : 0;
  t.node = c0;
  return n_hit != 0;
}

// F_W8 (A/B; measured 1.8x slower on C5: the kernel spills and the 8-wide stack bound costs occupancy,
// DESIGN.md §0 row 6): node p is the record pair (2p, 2p + 1), its children ordered along the axis in the first
// record's pad[0] (rt_bvh.cpp build_wide8_bvh). The half farther along the ray on that axis is tested first
// and every child it accepts stacked; then the nearer half's nearest accepted child is entered and its
// others stacked above — or, with none, the walk pops (the farther half's nearest, if any).
template <unsigned F, class STK>
__device__ __forceinline__ bool wide_node8(const Scene& S, Trav& t, STK* stk, int stride, int p) {
  const int ax = S.wnodes[2 * p].pad[0];
  const bool neg = signbit(ax == 0 ? t.i32x : (ax == 1 ? t.i32y : t.i32z));
  // (one inlined copy of the node test for both halves: a uniform loop)
  bool in = false;
#pragma nounroll
  for (int h = 0; h < 2; ++h) in = wide_node<F>(S, t, stk, stride, 2 * p + ((h == 0) == neg ? 0 : 1), h == 0);
  return in;
}
// Trav::node values of a walk with a postponed leaf (Trav::pend): nothing left but that leaf (kNone); or
// the next stack entry closes an instance frame, which must wait until the leaf — found inside that frame,
// in its ray's coordinates — is tested (kHold, the mixed walk).
constexpr int kNone = (int)0x80000000;
constexpr int kHold = (int)0x80000001;

// Leaf postponement in the mixed walk (media / frame worlds over 4-wide trees, F_MIXW; RT_MIXW_POSTPONE=1,
// A/B only): see walk_until. Measured slower (C4 at 100 spp, same box: 150.5 / 152.7 ms without, 164.4 /
// 166.1 with; leaf-step thresholds 1 / 8 / 16 of 64: 170-174 / 166 / 188 ms), so off by default.
#ifndef RT_MIXW_POSTPONE
#define RT_MIXW_POSTPONE 0
#endif
template <unsigned F>
constexpr bool kMixPostpone = RT_MIXW_POSTPONE && (F & F_MIXW) != 0 && (F & F_WIDE) == 0;

// Pop the next node of a binary (or mixed) walk; false once the walk is over. Frames that close
// rebuild the parent's ray from the world ray, once for a run of them. (Mixed walks: leaf slots are
// negative, so only a non-negative entry can be a frame marker.) `hold` (a postponed leaf is waiting,
// kMixPostpone): a frame marker is not popped — the walk waits at it (kHold) — and an empty stack leaves
// the walk on (kNone) for its leaf.
template <unsigned F, class STK>
__device__ __forceinline__ bool trav_pop_mixed(const Scene& S, Trav& t, const STK* stk, int stride, Side& side,
                                               double t_min = kEps, bool hold = false) {
  bool reb = false;
  for (;;) {
    const bool end = t.sp == 0;
    const int e = end ? 0 : stk[(--t.sp) * stride];
    const bool frame = (F & F_FRAMES) && ((F & F_MIXW) ? (e >= 0 && (e & RT_FRAME)) : (e & RT_FRAME));
    if (kMixPostpone<F> && hold && (end || frame)) {  // (reb is false: no frame closes while a leaf waits)
      t.sp += end ? 0 : 1;
      t.node = end ? kNone : kHold;
      return true;
    }
    if (end || !frame) {
      if ((F & F_FRAMES) && reb) {  // (also at the end: a tie redo walks on from it)
        // the parent's ray, once for the run of closed frames: the world ray rebuilt through the frames
        // still open. (Storing the world ray's reciprocals as well would save prep's divisions, but six
        // more LDS ints per lane cost C4's kernel a block per CU: 12 -> 10 waves, 249 -> 288 ms.)
        Ray pr = side.get_ray();
        for (int k = 0; k < t.level; ++k) pr = enter_instance(&S.nodes[side.frame(k)], pr);
        t.ray = prep(pr);
        if constexpr ((F & F_MIXW) != 0) set_ray32(t, t_min);
      }
      t.node = e;
      return !end;
    }
    --t.level;  // a frame closes
    reb = true;
  }
}

// Visit one node; false once the walk is over. The binary walk also opens instance frames
// (Translate/Rotate over a BVH, Lib.hs:1029-1052): a tagged stack entry, the frame's id in the
// lane's Side slots, and the child's ray in Trav::ray; when the entry is popped the parent's ray is
// rebuilt from the world ray through the frames still open (the same operations as on entry).
template <unsigned F, class R, class STK>
__device__ __forceinline__ bool trav_step(const Scene& S, Trav& t, double t_min, STK* stk, int stride, bool joint,
                                          Cnt& cnt, R& g, Side& side) {
  bool wide = false;
  if constexpr ((F & F_WIDE) != 0) wide = !t.ref;
  if (wide) {
    if (t.node >= 0) {
      if constexpr ((F & F_COUNT) != 0) ++cnt.wide;
      if ((F & F_W8) ? wide_node8<F>(S, t, stk, stride, t.node) : wide_node<F>(S, t, stk, stride, t.node)) return true;
    } else {
      const rt_node* n = &S.leaves[~t.node];
      trav_leaf<F>(S, t, n, ~t.node | kSlotTag, t_min, cnt, g, side, false);
    }
    if (t.sp == 0) return false;
    t.node = stk[(--t.sp) * stride];
    return true;
  }
  // Mixed walks with wide subtrees (F_MIXW): a node is a flat id (| RT_SUB), a wide node
  // (RT_WNODE | index) or a leaf-table slot handed out by a wide node (~slot, negative); all of them
  // lie in re-bounded subtrees except flat ids without RT_SUB.
  bool leaf_slot = false, to_wide = false;
  if constexpr ((F & F_MIXW) != 0) {
    to_wide = t.node >= 0 && (t.node & RT_WNODE);
    leaf_slot = t.node < 0;
  }
  if (!to_wide) {
  // (mixed walks: the RT_SUB tag of the node id says whether it lies below an RT_BVH_ORDERED node)
  int id = leaf_slot ? (~(t.node | RT_ISMED) | kSlotTag) : (t.node & ~(RT_SUB | RT_IDTAGS));
  int tag = leaf_slot ? RT_SUB : (kRefMixed<F> ? (t.node & RT_SUB) : 0);
  bool refsem = t.ref && !tag;
  const rt_node* n = leaf_slot ? &S.leaves[~(t.node | RT_ISMED)] : &S.nodes[id];
  const int tf = n->type;
  const int type = tf & RT_TYPE_MASK;
  if (type == RT_NODE_BVH) {  // (never a leaf slot)
   // A lane whose box test passes and whose next node is again a BVH node (RT_ISBOX) tests that one in
   // the same step, up to kFuse boxes: the boxes of a path without a leaf between them are tested under
   // the same bound in the same order, only in fewer walk steps (C4's skeleton: the fog's three
   // ancestors; C4 at 100 spp 253 -> 248 ms, C3 322 -> 318 ms). Not in the 4-wide kernels, whose binary
   // steps are tie redos only (+16 B/lane of scratch there).
   constexpr int kFuse = (F & F_WIDE) ? 0 : 8;
   for (int fuse = 0;; ++fuse) {
    if (fuse) {
      id = t.node & ~(RT_SUB | RT_IDTAGS);
      tag = kRefMixed<F> ? (t.node & RT_SUB) : 0;
      refsem = t.ref && !tag;
      n = &S.nodes[id];
    }
    // (RT_SAMEBOX: the parent's box, just passed under this bound)
    const bool same = kRefMixed<F> && (t.node & RT_IDTAGS) == RT_SAMEBOX;
    if constexpr ((F & F_COUNT) != 0) cnt.box += !same;
    if (same || box_hit(n->f, t.ray, t_min, refsem ? t.closest : closest_up<F>(t), joint)) {
      const int c = n->c;
      const bool ord = (c & RT_BVH_ORDERED) && !t.redo;
      if constexpr ((F & F_MIXW) != 0) {
        if (ord && (c & RT_WROOT)) {  // a re-bounded subtree with a 4-wide tree: walk that instead, from its
          t.node = RT_WNODE | ((c >> 2) & RT_WROOT_MASK);  // root node in this same step (below)
          to_wide = true;
          break;
        }
      }
      const bool flip = ord && !(c & RT_BVH_MEDIA_FIRST) && comp(t.ray.d, c & 3) < 0;  // (hoisted media first)
      const int ctag = (kRefMixed<F> && ord) ? RT_SUB : tag;
      stk[(t.sp++) * stride] = (flip ? n->a : n->b) | ctag;
      t.node = (flip ? n->b : n->a) | ctag;
      if ((t.node & RT_ISBOX) && fuse < kFuse) continue;
      return true;
    }
    break;
   }
  } else if ((F & F_FRAMES) && (type == RT_NODE_TRANSLATE || type == RT_NODE_ROTATE) && !(tf & RT_CHAIN_PRIM)) {
    if (t.level == 0) side.put_ray(plain(t.ray));
    // consecutive instances over a BVH (e.g. translate (rotate bvh)) open their frames in one step,
    // with one prep() for the innermost ray (the outer frames' rays are not tested against anything)
    Ray cr = plain(t.ray);
    int cur = leaf_slot ? n->c : id, ct = tf;
    if ((F & F_MIXW) && leaf_slot && (tf & RT_FRAME_FUSED)) {
      // the chain from the leaf-table copy (rt_prepare.cpp fuse_frame), read whole in one batch of four
      // 16-byte loads (field by field, the branches on its contents made the loads wait one by one)
      rt_node rec;
      {
        const uint4* q = reinterpret_cast<const uint4*>(n);
        const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        uint4* r = reinterpret_cast<uint4*>(&rec);
        r[0] = q0, r[1] = q1, r[2] = q2, r[3] = q3;
      }
      cur = rec.c;
      if constexpr ((F & F_COUNT) != 0) ++cnt.other;
      side.frame(t.level++) = cur;
      stk[(t.sp++) * stride] = RT_FRAME | cur;
      cr = enter_instance(&rec, cr);
      if (tf & RT_FRAME_FUSED2) {
        if constexpr ((F & F_COUNT) != 0) ++cnt.other;
        side.frame(t.level++) = rec.a;
        stk[(t.sp++) * stride] = RT_FRAME | rec.a;
        const int ax = (tf >> RT_FRAME_AX2_SHIFT) & 3;
        cr = Ray{unrotate_point(ax, rec.f[3], rec.f[4], cr.o), unrotate_point(ax, rec.f[3], rec.f[4], cr.d), cr.tm};
      }
      const int inner = (int)rec.f[5];
      t.ray = prep(cr);
      set_ray32(t, t_min);
      t.node = (inner & RT_WNODE) ? inner : (inner | tag);  // (a 4-wide root carries no tag)
      return true;
    } else {
      do {
        if constexpr ((F & F_COUNT) != 0) ++cnt.other;
        side.frame(t.level++) = cur;
        stk[(t.sp++) * stride] = RT_FRAME | cur;
        cr = enter_instance(&S.nodes[cur], cr);
        cur = S.nodes[cur].a;
        ct = S.nodes[cur].type;
      } while (((ct & RT_TYPE_MASK) == RT_NODE_TRANSLATE || (ct & RT_TYPE_MASK) == RT_NODE_ROTATE) &&
               !(ct & RT_CHAIN_PRIM));
    }
    t.ray = prep(cr);
    if constexpr ((F & F_MIXW) != 0) set_ray32(t, t_min);
    t.node = cur | tag;
    return true;
  } else {
    trav_leaf<F>(S, t, n, id, t_min, cnt, g, side, refsem);
  }
  if (!to_wide) return trav_pop_mixed<F>(S, t, stk, stride, side, t_min, t.pend >= 0);
  }
  if constexpr ((F & F_MIXW) != 0) {  // a 4-wide node (RT_WNODE | index)
    if constexpr ((F & F_COUNT) != 0) ++cnt.wide;
    refresh_ray32(t);
    if (wide_node<F>(S, t, stk, stride, t.node & ~RT_WNODE)) return true;
  }
  return trav_pop_mixed<F>(S, t, stk, stride, side, kEps, t.pend >= 0);
}

// ---- the 4-wide walk with postponed leaves (Aila & Laine's while-while, one postponed slot)
// A lane keeps stepping wide nodes while it holds one postponed leaf (`pend`); the wave switches to
// a leaf step, in which every lane holding a leaf tests it, once (almost) no walking lane is still
// searching for its first leaf. So wide-node steps and fp64 leaf tests do not share a divergent
// step. Culling is looser while a leaf waits (its hit does not yet bound the walk); the closest
// hit and the tie flag do not depend on the order leaves are tested in (trav_take).

template <class STK>
__device__ __forceinline__ int trav_pop(Trav& t, const STK* stk, int stride) {
  return t.sp ? stk[(--t.sp) * stride] : kNone;
}
// A second postponed leaf per lane (RT_LEAF_Q=1, round 6, A/B): kept in the lane's LDS word just below its
// stack (stk[-stride], -1 = empty; the kernels reserve it), filled only while `pend` holds one, so the walk
// is over exactly when node and pend are. A lane then walks on past its second leaf instead of waiting for
// the next leaf step. Measured slower (same images): C2 136.0 -> 138.5 ms, C5 at 64 spp 658 -> 670 ms; =2
// (both leaves tested in one leaf step) 149.5 / 690 ms. Off.
#ifndef RT_LEAF_Q
#define RT_LEAF_Q 0
#endif
// node -> pend when node is a leaf and the slot is free (else the queue word), then continue with the
// next stack entry
template <class STK>
__device__ __forceinline__ void trav_postpone(Trav& t, STK* stk, int stride) {
  if (t.node < 0 && t.node != kNone) {
    if (t.pend < 0) {
      t.pend = ~t.node;
      t.node = trav_pop(t, stk, stride);
    } else if (RT_LEAF_Q && stk[-stride] < 0) {
      stk[-stride] = (STK)~t.node;
      t.node = trav_pop(t, stk, stride);
    }
  }
}
template <unsigned F, class STK>
__device__ __forceinline__ void wide_inner(const Scene& S, Trav& t, STK* stk, int stride, Cnt& cnt) {
  if constexpr ((F & F_COUNT) != 0) ++cnt.wide;
  bool in;
  if constexpr ((F & F_W8) != 0) in = wide_node8<F>(S, t, stk, stride, t.node);
  else in = wide_node<F>(S, t, stk, stride, t.node);
  if (!in) t.node = trav_pop(t, stk, stride);
  trav_postpone(t, stk, stride);
}
template <unsigned F, class R, class STK>
__device__ __forceinline__ void wide_leaf(const Scene& S, Trav& t, double t_min, STK* stk, int stride, Cnt& cnt, R& g,
                                          Side& side) {
  // (RT_LEAF_Q=2: a lane holding two leaves tests both in one leaf step, one trav_leaf call site)
#pragma nounroll
  for (int k = 0; k < (RT_LEAF_Q == 2 ? 2 : 1) && t.pend >= 0; ++k) {
    const rt_node* n = &S.leaves[t.pend];  // (pend holds the leaf table slot)
    trav_leaf<F>(S, t, n, t.pend | kSlotTag, t_min, cnt, g, side, false);
    if (RT_LEAF_Q) {
      t.pend = stk[-stride];
      stk[-stride] = (STK)-1;
    } else {
      t.pend = -1;
    }
  }
  trav_postpone(t, stk, stride);
}

// Step the wave's walking lanes until at most `stop` of them still walk (`walking` goes false when
// a lane's walk is over). Binary walks: one node per lane per step; while more than `leaf_stop` of
// the walking lanes are at BVH nodes, a step runs only those (lanes at leaves, instances and media
// wait), so that one step runs the box test alone instead of every node kind its lanes are at
// (leaf_stop >= the live lanes: every step runs every lane). 4-wide walks: wide-node steps until at
// most `leaf_stop` walking lanes still look for their first leaf, then one leaf step.
template <unsigned F, class R, class STK>
__device__ __forceinline__ void walk_until(const Scene& S, Trav& t, bool& walking, double t_min, STK* stk, int stride,
                                           bool joint, int stop, int leaf_stop, Cnt& cnt, R& g, Side& side,
                                           int med_batch = 0) {
  if constexpr (kMixPostpone<F>) {
    // The mixed walk with postponed leaves (round 6; the 4-wide walk's scheme, Aila & Laine's while-while
    // with one slot): a lane that reaches a leaf-table slot of a 4-wide tree (a primitive, a chain, or an
    // instance frame to open) parks it in `pend` and walks on; the wave runs a leaf step — every lane holding
    // a leaf tests it (or opens its frame) — once at most leaf_stop of its walking lanes can still step
    // nodes. So wide / box steps and the leaf kinds' code do not share divergent steps (round 5's profile:
    // steps mixing wide nodes with leaves and frames were 17 % of C4's steps and 53 % of its time). The
    // closest hit is the least t over the leaves in any order (tier B: keyed media, re-bounded subtrees;
    // exact ties are flagged and redone in the reference's order), culling is only looser while a leaf
    // waits. A waiting leaf is tested in the coordinates it was found in: a lane holding one does not close
    // an instance frame (kHold), and a parked frame opens in the leaf step above the lane's next node.
    // Tie redos (t.redo) walk the caller's tree node by node, as before.
    for (;;) {
      if (__popcll(__ballot(walking)) <= stop) break;
      const bool holding = walking && !t.redo && t.pend >= 0 && t.node < 0;  // (at a second leaf, kHold, kNone)
      const bool seeking = walking && !holding;
      unsigned kinds = 0;
      unsigned long long t0 = 0;
      const bool inner = __popcll(__ballot(seeking)) > leaf_stop || __ballot(holding) == 0;
      if constexpr ((F & F_COUNT) != 0) {
        ++(inner ? cnt.islot : cnt.lslot);
        kinds = inner ? K_WIDE : K_LEAF;
        t0 = stamp();
      }
      // inner step: the seeking lanes' nodes (a lane at a leaf slot only parks it, below); leaf step: the
      // holding lanes' parked leaves — a leaf's test, or its frame opened — with the lane's next node (a
      // second leaf slot) put back on the stack, unless the walk waits at a frame marker (kHold) or is done
      // (kNone). One trav_step call site for both (a second inlined copy cost registers).
      bool go;
      if (inner) {
        go = seeking && (t.redo || t.node >= 0);
      } else {
        go = holding;
        if (holding) {
          const int saved = t.node;
          if (saved != kNone && saved != kHold) stk[(t.sp++) * stride] = saved;
          t.node = ~t.pend;
          t.pend = -1;
        }
      }
      if (go) walking = trav_step<F>(S, t, t_min, stk, stride, joint, cnt, g, side) || t.pend >= 0;
      // a leaf slot reached (by this step, or waiting since the last) with the slot free: park it, walk on
      if (walking && !t.redo && t.pend < 0 && t.node < 0 && t.node != kNone && t.node != kHold) {
        t.pend = ~t.node;
        // (trav_pop_mixed with `hold`: the next entry, or wait at a frame marker, or nothing left)
        const int e = t.sp ? stk[(t.sp - 1) * stride] : 0;
        const bool fr = e >= 0 && (e & RT_FRAME);
        t.node = t.sp == 0 ? kNone : (fr ? kHold : e);
        t.sp -= (t.sp == 0 || fr) ? 0 : 1;
      }
      if constexpr ((F & F_COUNT) != 0) {
        const unsigned long long t1 = stamp();
        if (cnt.prof && __lane_id() == (unsigned)(__ffsll((long long)__ballot(true)) - 1)) {
          atomicAdd(&cnt.prof[kinds], t1 - t0);
          atomicAdd(&cnt.prof[32 + kinds], 1ull);
        }
      }
    }
    return;
  }
  if constexpr ((F & F_WIDE) == 0) {
    for (;;) {
      const int n_walk = __popcll(__ballot(walking));
      if (n_walk <= stop) break;
      // (box-first steps only in the full variant's kernels, whose steps mix node kinds; elsewhere the
      // node-kind read and ballots would be overhead: C3 357 ms either way)
      // (the counting build follows the production schedule: its step counts describe the timed kernel)
      constexpr bool kBoxFirst = kRefMixed<F>;
      // (BVH nodes and wide nodes carry their kind in the id: RT_ISBOX, RT_WNODE; a wide node's leaf is
      // negative; the counting build also reads the other kinds)
      const bool box_id = walking && t.node >= 0 && (t.node & (RT_ISBOX | RT_WNODE));
      const bool at_box = kBoxFirst && box_id;
      int ty = -1;
      if constexpr ((F & F_COUNT) != 0) {
        if (walking) {
          if ((F & F_MIXW) && t.node < 0) ty = S.leaves[~(t.node | RT_ISMED)].type & RT_TYPE_MASK;
          else if (box_id) ty = RT_NODE_BVH;
          else ty = S.nodes[t.node & ~(RT_SUB | RT_IDTAGS)].type & RT_TYPE_MASK;
        }
      }
      bool go = walking;
      if constexpr (kBoxFirst) {
        const int n_box = __popcll(__ballot(at_box));
        if (leaf_stop < n_walk && n_box > leaf_stop) {
          go = walking && at_box;
        } else if ((F & F_MEDIA) && med_batch > 0) {
          // lanes at a medium (two boundary queries, a draw, a log) wait until med_batch of them are there
          // or nothing else walks, so that fewer steps carry the medium code
          const bool at_med = walking && t.node >= 0 && (t.node & (RT_WNODE | RT_IDTAGS)) == RT_ISMED;
          const int n_med = __popcll(__ballot(at_med));
          if constexpr (RT_FRAME_BATCH && (F & F_MIXW) && (F & F_FRAMES)) {
            // (likewise lanes at an instance frame found by a 4-wide node: its leaf slot lacks bit 26)
            const bool at_frm = walking && t.node < 0 && !(t.node & RT_ISMED);
            const int n_frm = __popcll(__ballot(at_frm));
            const bool hold = (n_med < med_batch && at_med) || (n_frm < med_batch && at_frm);
            go = walking && !hold;
            if (__ballot(go) == 0) go = walking;  // (every walking lane held: all go)
          } else {
            if (n_med < med_batch && n_med < n_walk) go = walking && !at_med;
          }
        }
      }
      if constexpr ((F & F_COUNT) != 0) {  // counting build: wave steps, and the node kinds each one runs
        ++cnt.islot;                        // (every lane counts a step: / 64 per wave)
        const bool inst = ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE;
        const bool box = ty == RT_NODE_BVH;
        cnt.lslot += (__ballot(go && box) != 0) + (__ballot(go && inst) != 0) +
                     (__ballot(go && ty == RT_NODE_CONSTANT_MEDIUM) != 0) +
                     (__ballot(go && !box && !inst && ty != RT_NODE_CONSTANT_MEDIUM) != 0);
      }
      unsigned kinds = 0;
      unsigned long long t0 = 0;
      if constexpr ((F & F_COUNT) != 0) {
        const bool wide = walking && t.node >= 0 && (t.node & RT_WNODE);
        const bool inst = ty == RT_NODE_TRANSLATE || ty == RT_NODE_ROTATE;
        bool frame = false;
        if (inst) {
          const int nid = t.node < 0 ? -1 : (t.node & ~(RT_SUB | RT_IDTAGS));
          const int tf = t.node < 0 ? S.leaves[~(t.node | RT_ISMED)].type : S.nodes[nid].type;
          frame = !(tf & RT_CHAIN_PRIM);
        }
        kinds = (__ballot(go && ty == RT_NODE_BVH && !wide) ? K_BOX : 0u) | (__ballot(go && wide) ? K_WIDE : 0u) |
                (__ballot(go && ty == RT_NODE_CONSTANT_MEDIUM) ? K_MEDIUM : 0u) | (__ballot(go && frame) ? K_FRAME : 0u) |
                (__ballot(go && ty >= 0 && ty != RT_NODE_BVH && ty != RT_NODE_CONSTANT_MEDIUM && !frame) ? K_LEAF : 0u);
        t0 = stamp();
      }
      if (go) walking = trav_step<F>(S, t, t_min, stk, stride, joint, cnt, g, side);
      if constexpr ((F & F_COUNT) != 0) {
        const unsigned long long t1 = stamp();
        if (cnt.prof && __lane_id() == (unsigned)(__ffsll((long long)__ballot(true)) - 1)) {
          atomicAdd(&cnt.prof[kinds], t1 - t0);
          atomicAdd(&cnt.prof[32 + kinds], 1ull);
        }
      }
    }
  } else {
    for (;;) {
      if (__popcll(__ballot(walking)) <= stop) break;
      // lanes that need wide-node steps before they can test a leaf (tie redo walks: binary steps)
      const bool seeking = walking && (t.ref || (t.pend < 0 && t.node >= 0));
      const bool holding = walking && !t.ref && t.pend >= 0;
      // (every walking lane is seeking or holding, so one of the two steps always makes progress)
      unsigned kinds = 0;
      unsigned long long t0 = 0;
      if constexpr ((F & F_COUNT) != 0) t0 = stamp();
      if (__popcll(__ballot(seeking)) > leaf_stop || __ballot(holding) == 0) {
        if constexpr ((F & F_COUNT) != 0) {
          ++cnt.islot;
          kinds = __ballot(walking && t.ref) ? K_BOX | K_WIDE : K_WIDE;
        }
        if (walking && t.ref) {
          walking = trav_step<F>(S, t, t_min, stk, stride, joint, cnt, g, side);
        } else if (walking && t.node >= 0) {
          wide_inner<F>(S, t, stk, stride, cnt);
          walking = t.node != kNone || t.pend >= 0;
        }
      } else {
        if constexpr ((F & F_COUNT) != 0) {
          ++cnt.lslot;
          kinds = K_LEAF;
        }
        if (holding) {
          wide_leaf<F>(S, t, t_min, stk, stride, cnt, g, side);
          walking = t.node != kNone || t.pend >= 0;
        }
      }
      if constexpr ((F & F_COUNT) != 0) {  // (step profile: wide steps, tie-redo steps, leaf steps)
        const unsigned long long t1 = stamp();
        if (cnt.prof && __lane_id() == (unsigned)(__ffsll((long long)__ballot(true)) - 1)) {
          atomicAdd(&cnt.prof[kinds], t1 - t0);
          atomicAdd(&cnt.prof[32 + kinds], 1ull);
        }
      }
    }
  }
}

// The closest hit's record, built once from the same ray with the same operations (a chain hit's
// primitive in the chain's innermost frame, with the t and face the walk found; a medium's record is
// its t, the point on the ray, normal (1,0,0), u = v = 0, front face, Lib.hs:1074-1080). A hit inside
// instance frames is recorded in the innermost frame's ray, then each frame's rewrite is applied from
// the innermost outwards with the ray its child saw (as `traverse` does when frames close); a chain's
// instances likewise (chain_hit). `r` is the world ray. Callers check `tie` first and re-walk with
// trav_restart_ref (ties between shading-identical records need none: tie_same). One inlined copy of the record code (prim_record) per kernel.
template <unsigned F>
__device__ __forceinline__ bool trav_finish(const Scene& S, const Trav& t, const Ray& r, double t_min, Hit& h,
                                            const Side& side) {
  if (t.best_node < 0) return false;
  // (a leaf of the 4-wide walk: its record from the leaf table)
  const bool slot = (F & (F_WIDE | F_MIXW)) && (t.best_node & kSlotTag);
  const rt_node* n = slot ? &S.leaves[t.best_node & ~kSlotTag] : &S.nodes[t.best_node];
  int levels = 0;  // frames around the hit, then the chain's instances
  if constexpr ((F & F_FRAMES) != 0) levels = t.best_level;
  Ray fr = r;  // the ray in the hit primitive's (or medium's) frame
  int sub = t.best_sub;
  const rt_node* leaf = n;
  int chain_id = -1, chain_len = 0;
  if constexpr ((F & F_FRAMES) != 0)
    for (int k = 0; k < levels; ++k) fr = enter_instance(&S.nodes[side.best(k)], fr);
  bool med = false;
  if constexpr ((F & F_MEDIA) != 0) med = sub == kSubMedium;
  if (med) {
    h.t = t.closest;
    h.p = at(fr, t.closest);
    h.n = v3(1, 0, 0);
    h.u = 0;
    h.v = 0;
    h.ff = 1;
    h.mat = n->b;  // (n: the leaf-table copy for a 4-wide walk's slot, whose id carries kSlotTag)
  }
  if constexpr ((F & F_INST) != 0) {
    if (!med && (sub & kSubChain)) {
      sub &= ~kSubChain;
      chain_id = slot ? n->c : t.best_node;
      int cur = chain_id;
      while ((S.nodes[cur].type & RT_TYPE_MASK) == RT_NODE_TRANSLATE || (S.nodes[cur].type & RT_TYPE_MASK) == RT_NODE_ROTATE) {
        fr = enter_instance(&S.nodes[cur], fr);
        cur = S.nodes[cur].a;
        ++chain_len;
      }
      leaf = &S.nodes[cur];
    }
  }
  if (!med) prim_record<F>(S, leaf, sub, fr, t.closest, h);
  // rewrites from the innermost instance outwards: the chain's (innermost), then the frames'
  for (int lv = levels + chain_len - 1; lv >= 0; --lv) {
    Ray rl = r;  // the ray instance lv's child saw
    const rt_node* inst = nullptr;
    int cur = chain_id;
    for (int k = 0; k <= lv; ++k) {
      if ((F & F_FRAMES) && k < levels) {
        inst = &S.nodes[side.best(k)];
      } else {
        inst = &S.nodes[cur];
        cur = inst->a;
      }
      rl = enter_instance(inst, rl);
    }
    exit_instance(inst, rl, h);
  }
  return true;
}

// ------------------------------------------------------------------ lights (Lib.hs:662-724)
// htblPdfValue (Lib.hs:673-705). For a BVHNode the reference gates on hit(node) and then sums
// the children's pdfs, each re-hit on its own. With no media in the lights tree (validated) a
// child that is not hit contributes exactly +0, so gating on the node's box test alone gives
// the same value: pdf(BVH) = box ? wl*(pdf(l)+0) + wr*(pdf(r)+0) : 0. Depth <= RT_LIGHT_DEPTH.
template <unsigned F, int D>
__device__ __forceinline__ double htbl_pdf_value(const Scene& S, int id, V3 origin, V3 v, const RayX& r) {
  id &= ~RT_IDTAGS;
  const rt_node* n = &S.nodes[id];
  const int type = n->type & RT_TYPE_MASK;
  Hit hh;
  if (type == RT_NODE_RECT_XZ) {
    if (!rect_hit(1, n->f[0], n->f[1], n->f[2], n->f[3], n->f[4], n->a, r, kEps, INFINITY, hh)) return 0.0;
    const double area = (n->f[1] - n->f[0]) * (n->f[3] - n->f[2]);
    const double distance_squared = hh.t * hh.t * sqlen(v);
    const double cosine = fabs(dot(v, hh.n) / vlen(v));
    return distance_squared / (cosine * area);
  }
  if (type == RT_NODE_SPHERE) {
    double t;
    if (!sphere_t(vload(n->f), n->f[3], r, kEps, INFINITY, t)) return 0.0;
    const double radius = n->f[3];
    const double cos_theta_max = sqrt(1 - radius * radius / sqlen(vload(n->f) - origin));
    const double solid_angle = 2 * kPi * (1 - cos_theta_max);
    return 1 / solid_angle;
  }
  if constexpr (D > 0) {
    if (type == RT_NODE_BVH) {
      if (!box_hit(n->f, r, kEps, INFINITY, false)) return 0.0;
      const double left_pdf = htbl_pdf_value<F, D - 1>(S, n->a, origin, v, r) + 0;
      const double left_w = (double)S.nodes[n->a & ~RT_IDTAGS].c / (double)n->c;
      const double right_pdf = htbl_pdf_value<F, D - 1>(S, n->b, origin, v, r) + 0;
      const double right_w = (double)S.nodes[n->b & ~RT_IDTAGS].c / (double)n->c;
      return left_w * left_pdf + right_w * right_pdf;
    }
  }
  return 0.0;
}

// htblRandom (Lib.hs:707-724)
template <class R>
__device__ inline V3 htbl_random(const Scene& S, int id, V3 o, R& g) {
  if (id >= 0) id &= ~RT_IDTAGS;
  while (id >= 0 && (S.nodes[id].type & RT_TYPE_MASK) == RT_NODE_BVH) {
    const rt_node* n = &S.nodes[id];
    const double rd = g.draw();
    id = (rd < (double)S.nodes[n->a & ~RT_IDTAGS].c / (double)n->c ? n->a : n->b) & ~RT_IDTAGS;
  }
  if (id < 0) return v3(1, 0, 0);
  const rt_node* n = &S.nodes[id];
  const int type = n->type & RT_TYPE_MASK;
  if (type == RT_NODE_RECT_XZ) {
    const double rx = draw_r(g, n->f[0], n->f[1]);
    const double rz = draw_r(g, n->f[2], n->f[3]);
    return v3(rx, n->f[4], rz) - o;
  }
  if (type == RT_NODE_SPHERE) {
    const V3 dir = vload(n->f) - o;
    const double dist_squared = sqlen(dir);
    const ONB uvw = onb_from_w(dir);
    const V3 rts = random_to_sphere(g, n->f[3], dist_squared);
    return onb_local(uvw, rts);
  }
  return v3(1, 0, 0);
}

// ------------------------------------------------------------------ materials (Lib.hs:822-903)
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return v - scale(2.0 * dot(v, n), n); }
__device__ __forceinline__ V3 refract(V3 v, V3 n, double eta) {
  const V3 uv = unit(v);
  const double cos_theta = dot(vneg(uv), n);
  const V3 par = scale(eta, uv + scale(cos_theta, n));
  const V3 perp = scale(-sqrt(1.0 - sqlen(par)), n);
  return par + perp;
}
// x ** 5 for schlick (Lib.hs:903, libm pow on the reference's side). x^2, x^4 and x^5 are carried
// as unevaluated sums hi + lo (each product's rounding error recovered exactly by an FMA), so the
// one final rounding is correct except within ~2^-100 relative of a rounding midpoint: the result
// is the correctly rounded x^5 (glibc's pow is within 0.52 ulp of it; OCML's pow(x, 5) matched
// glibc in 76 % of cases). No polynomial constants either: the compiler hoisted OCML pow's into
// registers for the whole kernel and spilled them. Zeros, NaN, infinities and magnitudes outside
// [2^-200, 2^200] (x = 1 - cos theta lies in [0, 2]) take the plain product. (Shared with the oracle's
// RT_FLAG_SHARED_LIBM mode: include/rt_libm.h.)
__device__ __forceinline__ double pow5(double x) { return rtlm_pow5(x); }
__device__ __forceinline__ double schlick(double cosine, double ref_idx) {
  const double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  const double r1 = r0 * r0;
  return r1 + (1.0 - r1) * pow5(1 - cosine);
}

// textureValue of a shaded hit's material, evaluated once per shaded hit so that a kernel holds one
// inlined copy of the texture code (Perlin turbulence is ~1.7 k instructions): every material but
// Dielectric reads its texture (Lib.hs:822-885), DiffuseLight only on back faces (`emitted`: front
// faces are black). Texture values draw no random numbers, so where they are evaluated changes
// nothing else.
// Kernels without non-constant textures (no F_TEX) read the constant where it is used instead (one
// load; hoisting it would only keep three more doubles live across the shading code).
template <unsigned F>
__device__ __forceinline__ V3 hit_texture(const Scene& S, const DMat& m, const Hit& h) {
  if constexpr ((F & F_TEX) == 0) return v3(0, 0, 0);
  const bool need = m.type != RT_MAT_DIELECTRIC && !(m.type == RT_MAT_DIFFUSE_LIGHT && h.ff);
  return need ? texture_value<F>(S, m.tex, h.u, h.v, h.p) : v3(0, 0, 0);
}
// The material's texture value at the hit: hit_texture's (F_TEX kernels) or the constant, read here.
template <unsigned F>
__device__ __forceinline__ V3 mat_texture(const Scene& S, const DMat& m, const Hit& h, V3 tx) {
  if constexpr ((F & F_TEX) != 0) return tx;
  return texture_value<F>(S, m.tex, h.u, h.v, h.p);
}

struct Scatter {
  Ray ray;
  V3 att;
  double pdf;
  int specular;
};

// scatter for every material except DiffuseLight (which the caller turns into `emitted`).
// The branches are fused where the materials compute the same thing, so that a wave holding
// several materials runs the expensive parts once: Lambertian's cosine sample
// (random_cosine_direction, Lib.hs:1206-1217) and Metal's fuzz vector (random_unit_vector,
// Lib.hs:1187-1197) both draw two numbers and take the cosine and sine of 2*pi*(first draw) —
// `2.0 * pi * r1` and `aa * 2.0 * pi` round identically, doubling being exact — and one square
// root; Metal and Dielectric both start from `unit(r.d)`. Each lane's draws keep the reference's
// order (Lambertian: coin, then its branch's draws). `tx` is the material's textureValue at the hit
// (hit_texture), evaluated once by the caller.
template <unsigned F, class R>
__device__ __forceinline__ void scatter(const Scene& S, const DMat& m, const Ray& r, const Hit& h, R& g, Scatter& s,
                                        V3 tx) {
  s.ray.o = h.p;
  s.ray.tm = r.tm;
  g.reserve(3);  // Lambertian draws 1 or 3 (more when sampling a lights BVH), Metal 2, Dielectric 1
  const bool lamb = m.type == RT_MAT_LAMBERTIAN, metal = m.type == RT_MAT_METAL;
  const bool diel = m.type == RT_MAT_DIELECTRIC;
  if (!(lamb || metal || diel)) {  // RT_MAT_ISOTROPIC, Lib.hs:861-865
    s.ray.d = random_in_unit_sphere(g);
    s.att = mat_texture<F>(S, m, h, tx);
    s.pdf = 1.0;
    s.specular = 0;
    return;
  }
  ONB uvw{};
  double coin = 1.0;
  if (lamb) {  // Lib.hs:823-836, mixture of light and cosine pdfs: the coin comes first
    uvw = onb_from_w(h.n);
    coin = g.draw();
  }
  const bool light = lamb && coin < 0.5;
  V3 v = v3(1, 0, 0);  // the cosine-weighted sample (Lambertian) or the unit vector (Metal)
  if (metal || (lamb && !light)) {
    const double a = g.draw(), b = g.draw();
    const double ang = 2.0 * kPi * a;
    const double cs = m_cos<R::kSL>(ang), sn = m_sin<R::kSL>(ang);
    const double z = (b * 2.0) - 1.0;                      // Metal: z = 2 zz - 1
    const double q = sqrt(metal ? 1.0 - z * z : 1.0 - b);  // Metal: r; Lambertian: z
    const double sr2 = sqrt(b);
    if (metal) v = v3(q * cs, q * sn, z);
    else v = onb_local(uvw, v3(cs * sr2, sn * sr2, q));
  }
  V3 ud = v3(0, 0, 0);
  if (metal || diel) ud = unit(r.d);
  if (lamb) {
    s.att = mat_texture<F>(S, m, h, tx);
    V3 pdf_d = v;
    if constexpr ((F & F_LIGHTS) != 0)
      if (light) pdf_d = htbl_random(S, S.lights, h.p, g);
    const V3 dir = unit(pdf_d);
    s.ray.d = dir;
    double v1 = 0.0;
    if constexpr ((F & F_LIGHTS) != 0)
      if (S.lights >= 0) v1 = htbl_pdf_value<F, RT_LIGHT_DEPTH>(S, S.lights, h.p, dir, prep(Ray{h.p, dir, 0.0}));
    const double cosine = dot(unit(dir), uvw.w);
    const double v2 = cosine <= 0 ? 0 : cosine / kPi;
    s.pdf = 0.5 * (v1 + v2);
    s.specular = 0;
  } else if (metal) {  // Lib.hs:837-841
    const V3 reflected = reflect(ud, h.n);
    s.ray.d = reflected + scale(m.param, v);
    s.att = mat_texture<F>(S, m, h, tx);
    s.pdf = 0.0;
    s.specular = 1;
  } else {  // Dielectric, Lib.hs:842-859
    const double eta = h.ff ? 1.0 / m.param : m.param;
    const double cos_theta = gmin(dot(vneg(ud), h.n), 1.0);
    const double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
    const double rd = g.draw();
    if ((eta * sin_theta > 1.0) || rd < schlick(cos_theta, eta)) s.ray.d = reflect(ud, h.n);
    else s.ray.d = refract(ud, h.n, eta);
    s.att = v3(1.0, 1.0, 1.0);
    s.pdf = 1.0;
    s.specular = 1;
  }
}

}  // namespace rtd
