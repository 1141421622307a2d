// rt_device.h — device-side geometry, RNG and shading for the gfx950 path tracer.
//
// Everything here is fp64 and compiled with -ffp-contract=off: the reference is Haskell on
// GHC 8.8's x86-64 NCG (no FMA), and its semantics are followed operation by operation
// (evaluation order of `infixl 7` vector ops, GHC's NaN-propagating min/max, strict/lenient
// interval tests per primitive). Every function cites the src/Lib.hs lines it follows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt.h"
#include "rt_layout.h"
#include "rt_libm.h"
#include "rt_wide.h"


namespace rtd {

constexpr double kEps = 0.0001;            // src/Lib.hs:76-77
constexpr double kPi = 3.141592653589793;  // GHC pi

struct V3 {
  double x, y, z;
};
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 scale(double k, V3 a) { return v3(a.x * k, a.y * k, a.z * k); }
__device__ __forceinline__ V3 divide(V3 a, double k) { return v3(a.x / k, a.y / k, a.z / k); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double sqlen(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ double vlen(V3 a) { return sqrt(sqlen(a)); }
__device__ __forceinline__ V3 unit(V3 a) { return divide(a, vlen(a)); }
__device__ __forceinline__ V3 vload(const double* p) { return v3(p[0], p[1], p[2]); }
__device__ __forceinline__ double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// GHC Ord defaults: max x y = if x <= y then y else x; min x y = if x <= y then x else y.
__device__ __forceinline__ double gmax(double x, double y) { return x <= y ? y : x; }
__device__ __forceinline__ double gmin(double x, double y) { return x <= y ? x : y; }

struct Ray {
  V3 o, d;
  double tm;
};

// The transcendentals of the path: OCML, or (SL, tier A with RT_FLAG_SHARED_LIBM) the portable ones of
// include/rt_libm.h that the oracle evaluates too, bit for bit.
template <bool SL>
__device__ __forceinline__ double m_sin(double x) {
  if constexpr (SL) return rtlm_sin(x);
  else return sin(x);
}
template <bool SL>
__device__ __forceinline__ double m_cos(double x) {
  if constexpr (SL) return rtlm_cos(x);
  else return cos(x);
}
template <bool SL>
__device__ __forceinline__ double m_log(double x) {
  if constexpr (SL) return rtlm_log(x);
  else return log(x);
}
template <bool SL>
__device__ __forceinline__ double m_atan(double x) {
  if constexpr (SL) return rtlm_atan(x);
  else return atan(x);
}
template <bool SL>
__device__ __forceinline__ double m_asin(double x) {
  if constexpr (SL) return rtlm_asin(x);
  else return asin(x);
}
template <unsigned F>
constexpr bool kSL = (F & F_SLIBM) != 0;

// Correctly rounded a / b from y = RN(1/b): two Markstein residual corrections (each residual
// a - b*q is exact under FMA when nothing under- or overflows), then a range guard that falls back
// to the IEEE division unless |a|, |b| and |q| all lie in [2^-900, 2^900] (zero, tiny, huge and
// non-finite operands included). Bit-identical to `a / b` (tests/test_gpu_math.py).
// A branch to a rare fallback (RT_COLD_BRANCHES=1, round 6, A/B): marked unlikely, so that block placement
// moves the fallback out of the hot code's instruction-cache lines. Measured (round 6, same images): C5 -1.2 %;
// with the opaque Philox key (below) C2 -0.4 %, C3 -1.1 %, C4 ~-1 % (alone, C2 +0.4 %: +8 B/lane of scratch).
#ifndef RT_COLD_BRANCHES
#define RT_COLD_BRANCHES 1
#endif
#if RT_COLD_BRANCHES
#define RT_COLD(c) __builtin_expect(!!(c), 0)
#else
#define RT_COLD(c) (c)
#endif
// The IEEE division of the rare operands. RT_DIV_CALL=1 puts it out of line, one copy per kernel instead of
// one per inlined quotient (the C4 kernel inlines 157 IEEE divisions, ~1.9 k of its 14.1 k instructions, and
// its 83.5 KB of code miss the instruction cache: 102 M misses per launch, profiles/r6_pmc_c4.json); the call
// raised its scratch 176 -> 192 B/lane (round 6), so it stays inline.
#ifndef RT_DIV_CALL
#define RT_DIV_CALL 0
#endif
#if RT_DIV_CALL
__device__ __noinline__ double ieee_div(double a, double b) { return a / b; }
#else
__device__ __forceinline__ double ieee_div(double a, double b) { return a / b; }
#endif
__device__ __forceinline__ bool in_range(double x) {
  const double ax = fabs(x);
  return (ax >= 0x1p-900) & (ax <= 0x1p900);
}
__device__ __forceinline__ double div_exact(double a, double b, double y) {
  double q = a * y;
  double r = fma(-q, b, a);
  q = fma(r, y, q);
  r = fma(-q, b, a);
  q = fma(r, y, q);
  if (RT_COLD(!(in_range(a) && in_range(b) && in_range(q)))) q = ieee_div(a, b);
  return q;
}

// A ray plus the per-ray reciprocals the exact divisions use. A zero component (the +x light direction
// of the Lambertian quirk, DESIGN.md §4.4, is (1, 0, 0)) has inv = +-inf, and a * inv is then exactly the
// IEEE a / +-0 (qdiv). Nothing else is carried (round 4: the sphere quadratic's d.d and its reciprocal,
// and the `safe` flag, are recomputed where they are used — five registers fewer in every walk's live
// state: C2's 4-wave kernel 124 -> 108 B/lane of scratch, C4's 192 -> 176).
struct RayX {
  V3 o, d;
  double tm;
  V3 inv;      // RN(1 / d)
};
__device__ __forceinline__ bool div_ok(double b) { return in_range(b); }
__device__ __forceinline__ RayX prep(const Ray& r) {
  RayX x;
  x.o = r.o;
  x.d = r.d;
  x.tm = r.tm;
  x.inv = V3{1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z};
  return x;
}
__device__ __forceinline__ Ray plain(const RayX& x) { return Ray{x.o, x.d, x.tm}; }
// The division-free box test's condition (box_hit): a finite origin (|o| <= 2^100) and every direction
// component either zero or in [2^-900, 2^900]. With the world's finite box coordinates within 2^100 (else
// the host walks it with the per-axis test, rt_render.hip far_boxes) no slab product (f - o) * RN(1/d)
// then overflows (|f - o| < 2^101, |RN(1/d)| <= 2^900): an infinite product is a zero axis's exact quotient.
__device__ __forceinline__ bool ray_safe(const RayX& r) {
  return ((r.d.x == 0.0) | div_ok(r.d.x)) & ((r.d.y == 0.0) | div_ok(r.d.y)) & ((r.d.z == 0.0) | div_ok(r.d.z)) &
         (fabs(r.o.x) <= 0x1p100) & (fabs(r.o.y) <= 0x1p100) & (fabs(r.o.z) <= 0x1p100);
}
// a / d exactly, given y = RN(1/d): a zero divisor gives a * y (= the IEEE a / +-0: +-inf with the
// sign of a xor d, NaN for a = 0 or NaN), operands and quotient in [2^-900, 2^900] the Markstein
// quotient (div_exact), anything else the IEEE division (a rare, divergent branch).
__device__ __forceinline__ double qdiv(double a, double d, double y) {
  double q = a * y;
  double r = fma(-q, d, a);
  q = fma(r, y, q);
  r = fma(-q, d, a);
  q = fma(r, y, q);
  const bool zero = d == 0.0;
  q = zero ? a * y : q;
  if (RT_COLD(!(zero | (in_range(a) & in_range(d) & in_range(q))))) q = ieee_div(a, d);
  return q;
}
struct Hit {
  double t;
  V3 p, n;
  double u, v;
  int ff;
  int mat;
};
__device__ __forceinline__ V3 at(const Ray& r, double t) { return r.o + scale(t, r.d); }  // Lib.hs:317-318

struct Scene {
  const rt_node* nodes;
  const rt_wnode* wnodes;  // 4-wide world tree (F_WIDE kernels); null when not built
  const rt_node* leaves;   // its leaf table: referenced leaves (c = flat node id), LDS or global
  const rt_qnode* qnodes;  // spheres-only worlds: the 4-wide tree quantised (F_QNODE kernels), or null
  const double* sleaves;   // and its leaf table's spheres: center xyz, radius per slot
  const DMat* mats;
  const rt_texture* texs;
  const rt_perlin* perlins;
  const rt_image* images;
  const uint8_t* pool;
  int world;
  int world_ref;  // the caller's (makeBVH) world root: exact ties are resolved on this tree
  int lights;
  int ref_walk;   // media or instance frames: the replacement loop walks the caller's tree in the
                  // reference's own order (media draw order, Lib.hs:971-988,1053-1080)
  int frames;     // deepest nesting of instance frames in the world trees (the lanes' Side slots)
  double bg[3];
};

// Wave-level timestamp for the counting build's phase split (MI355X_MICROARCH.md / HIP guide
// "In-kernel stamps": one asm statement with its own lgkmcnt wait, fenced by sched barriers).
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// ------------------------------------------------------------------ RNG
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 33)) * 0xff51afd7ed558ccdULL;
  z = (z ^ (z >> 33)) * 0xc4ceb9fe1a85ec53ULL;
  return z ^ (z >> 33);
}
// random-1.2.0 `random :: Double` = 1 - word64/2^64 (src/Random.hs:23-25)
__device__ __forceinline__ double word_to_draw(uint64_t w) {
  return 1.0 - (double)w / 18446744073709551616.0;
}

// Tier A: the reference's SplitMix64 stream (nextWord64). SL: the draws' transcendentals (random unit
// vectors, cosine directions, sphere samples, media distances) from rt_libm.h.
template <bool SL = false>
struct RngExactT {
  static constexpr bool kSL = SL;
  static constexpr bool kKeyed = false;  // media draw from the stream, in the walk's order (the reference's)
  uint64_t seed, gamma;
  __device__ __forceinline__ void reserve(int) {}
  __device__ __forceinline__ double draw() {
    seed += gamma;
    return word_to_draw(mix64(seed));
  }
};
using RngExact = RngExactT<false>;

// Tier B: Philox4x32-10, key = seed, counter = {pair, sample, pixel, 0}; two draws per block.
// RT_PHILOX_OPAQUE_KEY=1 (round 6, A/B): the key is made opaque at each block (an empty asm on its scalar
// registers), so that the 20 round keys are derived where a block is computed instead of being hoisted to the
// kernel's entry and held (spilled to VGPR lanes and read back with v_readlane) across the whole loop.
// Set by the spheres (C1, C2), Cornell (C3) and full-dark (C4) units; not by C5's (+0.5 % there): DESIGN.md §3.1.
#ifndef RT_PHILOX_OPAQUE_KEY
#define RT_PHILOX_OPAQUE_KEY 0
#endif
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  if (RT_PHILOX_OPAQUE_KEY) asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 multiply per word (v_mad_u64_u32) instead of separate mul_hi / mul_lo
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// The stream's words pass through a 4-word FIFO. `reserve(k)` tops it up to k words, one Philox
// block per loop trip, at a point where the whole wave runs the same code; `draw` then only shifts
// the FIFO. (Blocks computed inside every divergent draw site would each cost the wave a full
// Philox evaluation.) The sequence of words is the stream's, whatever the reserve points.
struct RngPhilox {
  static constexpr bool kSL = false;
  // media draw keyed by (walk, occurrence): keyed() below, not from the stream
  static constexpr bool kKeyed = true;
  uint32_t k0, k1, pid, sample, pair;
  uint32_t n;  // buffered words
  uint64_t w0, w1, w2, w3;
  __device__ __forceinline__ void init(uint64_t seed, uint32_t p, uint32_t s) {
    k0 = (uint32_t)seed;
    k1 = (uint32_t)(seed >> 32);
    pid = p;
    sample = s;
    pair = 0;
    n = 0;
  }
  __device__ __forceinline__ void block(uint64_t& x, uint64_t& y) {
    uint32_t c[4] = {pair, sample, pid, 0u};
    philox(c, k0, k1);
    ++pair;
    x = (uint64_t)c[0] | ((uint64_t)c[1] << 32);
    y = (uint64_t)c[2] | ((uint64_t)c[3] << 32);
  }
  __device__ __forceinline__ void reserve(int k) {  // k <= 3 (the FIFO then holds at most 4 words)
    while ((int)n < k) {
      uint64_t x, y;
      block(x, y);
      if (n == 0) {
        w0 = x;
        w1 = y;
      } else if (n == 1) {
        w1 = x;
        w2 = y;
      } else {
        w2 = x;
        w3 = y;
      }
      n += 2;
    }
  }
  // Words of this stream consumed so far (word i is word i % 2 of block i / 2).
  __device__ __forceinline__ uint32_t consumed() const { return 2u * pair - n; }
  // A medium occurrence's draw (tier B): the first word of the Philox block at counter {words of this
  // sample's stream consumed so far, sample, pixel, 2^31 | key}, key = the occurrence's key (rt_bvh.cpp
  // unfold_media). A walk consumes no stream words, so the counter names the walk (the path's position in
  // its stream) and the key the occurrence: the draw does not depend on the order media are visited in.
  // Word 3 >= 2^31 keeps these blocks apart from the stream's (word 3 = 0).
  __device__ __forceinline__ double keyed(uint32_t key) const { return keyed_at(k0, k1, consumed(), sample, pid, key); }
  static __device__ __forceinline__ double keyed_at(uint32_t k0, uint32_t k1, uint32_t walk, uint32_t sample,
                                                    uint32_t pid, uint32_t key) {
    uint32_t c[4] = {walk, sample, pid, 0x80000000u | key};
    philox(c, k0, k1);
    return word_to_draw((uint64_t)c[0] | ((uint64_t)c[1] << 32));
  }
  __device__ __forceinline__ double draw() {
    if (n == 0) block(w0, w1), n = 2;  // not reserved: compute here
    const uint64_t w = w0;
    w0 = w1;
    w1 = w2;
    w2 = w3;
    --n;
    return word_to_draw(w);
  }
};

template <class R>
__device__ __forceinline__ double draw_r(R& g, double mn, double mx) {  // randomDoubleRM
  const double rd = g.draw();
  return mn + (mx - mn) * rd;
}
template <class R>
__device__ __forceinline__ V3 random_in_unit_sphere(R& g) {  // Lib.hs:1160-1168
  for (;;) {
    g.reserve(3);
    const double x = g.draw(), y = g.draw(), z = g.draw();
    const V3 p = scale(2.0, v3(x, y, z)) - v3(1.0, 1.0, 1.0);
    if (sqlen(p) < 1.0) return p;
  }
}
template <class R>
__device__ __forceinline__ V3 random_in_unit_disk(R& g) {  // Lib.hs:1178-1185
  for (;;) {
    g.reserve(2);
    const double x = g.draw(), y = g.draw();
    const V3 p = scale(2.0, v3(x, y, 0.0)) - v3(1.0, 1.0, 0.0);
    if (sqlen(p) < 1.0) return p;
  }
}
template <class R>
__device__ __forceinline__ V3 random_unit_vector(R& g) {  // Lib.hs:1187-1197
  const double aa = g.draw();
  const double a = aa * 2.0 * kPi;
  const double zz = g.draw();
  const double z = (zz * 2.0) - 1.0;
  const double r = sqrt(1.0 - z * z);
  return v3(r * m_cos<R::kSL>(a), r * m_sin<R::kSL>(a), z);
}
template <class R>
__device__ __forceinline__ V3 random_cosine_direction(R& g) {  // Lib.hs:1206-1217
  const double r1 = g.draw(), r2 = g.draw();
  const double z = sqrt(1.0 - r2);
  const double phi = 2.0 * kPi * r1;
  const double sr2 = sqrt(r2);
  return v3(m_cos<R::kSL>(phi) * sr2, m_sin<R::kSL>(phi) * sr2, z);
}
template <class R>
__device__ __forceinline__ V3 random_to_sphere(R& g, double radius, double dist_squared) {  // Lib.hs:1219-1228
  const double r1 = g.draw(), r2 = g.draw();
  const double z = 1.0 + r2 * (sqrt(1.0 - radius * radius / dist_squared) - 1.0);
  const double phi = 2.0 * kPi * r1;
  const double s = sqrt(1.0 - z * z);
  return v3(m_cos<R::kSL>(phi) * s, m_sin<R::kSL>(phi) * s, z);
}

// ------------------------------------------------------------------ ONB (Lib.hs:263-279)
struct ONB {
  V3 u, v, w;
};
__device__ __forceinline__ ONB onb_from_w(V3 n) {
  ONB o;
  o.w = unit(n);
  const V3 a = fabs(o.w.x) > 0.9 ? v3(0.0, 1.0, 0.0) : v3(1.0, 0.0, 0.0);
  o.v = unit(cross(o.w, a));
  o.u = cross(o.w, o.v);
  return o;
}
__device__ __forceinline__ V3 onb_local(const ONB& o, V3 a) {
  return (scale(a.x, o.u) + scale(a.y, o.v)) + scale(a.z, o.w);
}

// GHC's RealFloat-default atan2 (GHC.Float), used by `hit Sphere` for u (Lib.hs:1102).
__device__ __forceinline__ bool neg_zero(double x) { return x == 0.0 && signbit(x); }
template <bool SL = false>
__device__ inline double ghc_atan2(double y, double x) {
  double sgn = 1.0;
  // -atan2 (-y) x branch, applied at most once (it maps y < 0 to y > 0 / y = +0)
  if ((x <= 0 && y < 0) || (x < 0 && neg_zero(y)) || (neg_zero(x) && neg_zero(y))) {
    sgn = -1.0;
    y = -y;
  }
  double r;
  if (x > 0) r = m_atan<SL>(y / x);
  else if (x == 0 && y > 0) r = kPi / 2;
  else if (x < 0 && y > 0) r = kPi + m_atan<SL>(y / x);
  else if (y == 0 && (x < 0 || neg_zero(x))) r = kPi;
  else if (x == 0 && y == 0) r = y;
  else r = x + y;
  return sgn * r;
}

// faceNormal (Lib.hs:1111-1117)
__device__ __forceinline__ void face_normal(const Ray& r, V3 outward, int& ff, V3& n) {
  ff = dot(r.d, outward) < 0;
  n = ff ? outward : vneg(outward);
}

// rotatePoint / unRotatePoint (Lib.hs:763-787)
__device__ __forceinline__ V3 rotate_point(int axis, double s, double c, V3 p) {
  if (axis == 0) return v3(p.x, c * p.y - s * p.z, s * p.y + c * p.z);
  if (axis == 1) return v3(c * p.x + s * p.z, p.y, -s * p.x + c * p.z);
  return v3(c * p.x - s * p.y, s * p.x + c * p.y, p.z);
}
__device__ __forceinline__ V3 unrotate_point(int axis, double s, double c, V3 p) {
  if (axis == 0) return v3(p.x, c * p.y + s * p.z, -s * p.y + c * p.z);
  if (axis == 1) return v3(c * p.x - s * p.z, p.y, s * p.x + c * p.z);
  return v3(c * p.x + s * p.y, -s * p.x + c * p.y, p.z);
}

}  // namespace rtd
