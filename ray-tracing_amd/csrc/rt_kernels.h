// rt_kernels.h — the render kernels as templates (device code), shared by the kernel translation
// units: rt_k_spheres.hip, rt_k_cornell.hip and rt_k_full.hip each instantiate one scene
// variant's render kernels (so the variants compile in parallel), rt_render.hip the small kernels
// and the host half of the C ABI. Kernel design: DESIGN.md §3.
#pragma once
#ifndef RT_LANE_LDS
#define RT_LANE_LDS 1
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "rt.h"
#include "rt_device.h"
#include "rt_internal.h"
#include "rt_trace.h"

using namespace rtd;

namespace {

// Unsigned 32-bit division by an invariant divisor d >= 1 (Granlund & Montgomery): with
// l = ceil(log2 d) and m = floor(2^32 (2^l - d) / d) + 1, n / d = (t + ((n - t) >> s1)) >> s2 for
// every 32-bit n, t = umulhi(m, n), s1 = min(l, 1), s2 = max(l - 1, 0). One multiply and a few
// shifts instead of the software division a `/` on the device becomes.
struct UDiv {
  uint32_t m;
  int s1, s2;
};
inline UDiv make_udiv(uint32_t d) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return UDiv{(uint32_t)m, l < 1 ? l : 1, l > 1 ? l - 1 : 0};
}
__device__ __forceinline__ uint32_t udiv(uint32_t n, UDiv d) {
  const uint32_t t = __umulhi(d.m, n);
  return (t + ((n - t) >> d.s1)) >> d.s2;
}

struct RenderArgs {
  Scene S;
  rt_camera cam;
  int W, H, spp, max_depth;
  uint32_t flags;
  int tile, tiles_x, tiles_total, shard_rank, shard_count;
  long long work_total;  // claimable units of this launch (< 2^32): work-items before tail_start, then one
                         // unit per sample of each work-item from tail_start on (kTail kernels)
  long long slab;        // slab pixels of this shard
  int chunk, chunks;     // tier B: samples per chunk (rt_sample_chunk) and chunks per pixel in this launch
  int chunk_base;        // the launch's first chunk (a frame may render its chunks in batches)
  int combine;           // combine_chunks: 1 = add to the running sums in `acc`, 2 = the last batch (store)
  double* acc;           // running per-pixel sums between chunk batches, [slab pixel][3]
  UDiv div_tp, div_tile, div_tiles_x, div_bpr;  // by tile*tile, tile*tile*chunks, tiles_x, tile/8
  double* partial;       // tier B: chunk sums, [chunk][slab pixel][3]
  uint64_t seed;
  unsigned long long* counter;
  unsigned long long* work;  // counting build: [segments, box, prim, other, light, blocks, samples]
  unsigned long long* prof;  // counting build, optional: the walk's step profile (Cnt::prof)
  int trav_stop;             // replacement loop: keep stepping while > trav_stop/64 of live lanes walk
  int batch;                 // replacement loop: most work-items a wave claims per atomic
  float batch_per_item;      // ...tapering to rem * batch_per_item as `rem` items remain (>= need)
  int batch_floor;           // ...but never below this many (RTAMD_BATCH_FLOOR; 0: the lanes' need)
  int leaf_stop;             // 4-wide walk: leaf step once <= leaf_stop/64 of live lanes seek a leaf
  int box_first;             // binary walk: box-only steps while > box_first/64 of live lanes are at BVH
                             // nodes (64: never)
  uint32_t rev_tiles;        // RTAMD_TILE_REV: the slab's tiles run last to first (this count; 0: in order)
  uint8_t* out_rgb;  // tier B: slab; tier A: image
  double* out_lin;
  uint64_t* gens;  // tier A: per-column (seed, gamma), updated in place
  int med_batch;   // binary walk of media worlds: lanes at a medium wait until this many are there (or
                   // nothing else walks); 0: never wait
  double* trace;   // tier A, rt_debug_exact_trace: column trace_col's path segments (10 doubles each)
  int* trace_n;
  int trace_col, trace_cap;
  // (last, so that the fields before keep their kernel-argument offsets in the kernels that do not read
  // these: moved in the middle, they cost the spheres and Cornell kernels 0.7 %)
  long long items_total; // work-items of this launch: slab pixels x sample chunks
  long long tail_start;  // the work-items from here on are dealt one sample per unit (kTail: the frame's
                         // tail, so that no lane starts a whole chunk of long paths as the GPU runs dry),
                         // their colours stored in tail_buf and summed in sample order by tail_combine
  double* tail_buf;      // [unit][3]
  UDiv div_chunk;        // by chunk
};

// Slab pixel index -> image pixel (tile-major, 8x8 blocks inside a tile). Slab indices are < 2^32
// (launch_philox checks).
__device__ __forceinline__ bool work_pixel(const RenderArgs& A, uint32_t w, int& px, int& row) {
  const uint32_t tp = (uint32_t)(A.tile * A.tile);
  const uint32_t lt = udiv(w, A.div_tp);
  const uint32_t within = w - lt * tp;
  const long long gt = (long long)A.shard_rank + (long long)lt * A.shard_count;
  if (gt >= A.tiles_total) return false;
  const uint32_t ty = udiv((uint32_t)gt, A.div_tiles_x), tx = (uint32_t)gt - ty * (uint32_t)A.tiles_x;
  const uint32_t blk = within >> 6, l = within & 63;
  const uint32_t by = udiv(blk, A.div_bpr), bx = blk - by * (uint32_t)(A.tile >> 3);
  px = (int)(tx * A.tile + bx * 8 + (l & 7));
  row = (int)(ty * A.tile + by * 8 + (l >> 3));
  return px < A.W && row < A.H;
}

// Tier-B work-item -> (slab pixel, sample chunk). Items run tile by tile, chunk by chunk inside a
// tile, so a wave's 64 consecutive items are one 8x8 pixel block at one chunk (coherent rays).
// Returns false for pixels outside the image; else the sample range [s0, s1) and the chunk
// sum's slot in `partial`.
__device__ __forceinline__ bool work_item(const RenderArgs& A, uint32_t wi, int& px, int& row, int& s0, int& s1,
                                          long long& slot) {
  const uint32_t tp = (uint32_t)(A.tile * A.tile);
  const uint32_t lw = udiv(wi, A.div_tile);  // by tp * chunks
  const uint32_t rem = wi - lw * tp * (uint32_t)A.chunks;
  const uint32_t lt = A.rev_tiles ? A.rev_tiles - 1 - lw : lw;
  const uint32_t k = udiv(rem, A.div_tp);
  const uint32_t idx = lt * tp + (rem - k * tp);
  if (!work_pixel(A, idx, px, row)) return false;
  s0 = (A.chunk_base + (int)k) * A.chunk;
  s1 = min(A.spp, s0 + A.chunk);
  slot = (long long)k * A.slab + idx;
  return s0 < s1;
}
__device__ __forceinline__ void store_partial_at(double* base, long long slot, V3 sum) {
  double* q = base + slot * 3;
  q[0] = sum.x;
  q[1] = sum.y;
  q[2] = sum.z;
}
__device__ __forceinline__ void store_partial(const RenderArgs& A, long long slot, V3 sum) {
  store_partial_at(A.partial, slot, sum);
}
// Sample-granular tails: in the full variants' kernels only (media / frame worlds, C4), whose work-items
// (8 samples of paths up to 50 segments through fog) are long and uneven — a frame's last claims left
// C4 a ~19 ms tail per launch. (In the spheres kernel the extra state cost more than its ~2 ms tail:
// DESIGN.md §3.1.)
template <unsigned F>
constexpr bool kTail = (F & F_FRAMES) != 0;
// A claimable unit: a work-item, or (from tail_start on) one sample of one. A tail unit's slot is
// kTailSlot + its index (its colour goes to tail_buf); false for pixels outside the image and for units
// past the work-item's last sample.
constexpr long long kTailSlot = 1ll << 40;
__device__ __forceinline__ bool work_unit(const RenderArgs& A, uint32_t wi, int& px, int& row, int& s0, int& s1,
                                          long long& slot) {
  if ((long long)wi < A.tail_start) return work_item(A, wi, px, row, s0, s1, slot);
  const uint32_t u = wi - (uint32_t)A.tail_start;
  const uint32_t q = udiv(u, A.div_chunk);
  const uint32_t k = u - q * (uint32_t)A.chunk;
  if (!work_item(A, (uint32_t)A.tail_start + q, px, row, s0, s1, slot)) return false;
  s0 += (int)k;
  if (s0 >= s1) return false;
  s1 = s0 + 1;
  slot = kTailSlot + u;
  return true;
}

// getRay (Lib.hs:1253-1267): the disk and time draws always happen.
template <class R>
__device__ __forceinline__ Ray get_ray(const rt_camera& k, double s, double t, R& g) {
  const V3 rd = scale(k.lens_radius, random_in_unit_disk(g));
  const V3 offset = scale(rd.x, vload(k.u)) + scale(rd.y, vload(k.v));
  g.reserve(1);
  const double tm = draw_r(g, k.t0, k.t1);
  Ray r;
  r.o = vload(k.origin) + offset;
  r.d = (((vload(k.llc) + scale(s, vload(k.horiz))) + scale(t, vload(k.vert))) - vload(k.origin)) - offset;
  r.tm = tm;
  return r;
}

// scaleColor (Lib.hs:287-288): NaN -> 0, +inf -> 255.
__device__ __forceinline__ uint8_t scale_color(double x) {
  const double s = sqrt(x);
  const double cl = s < 0.0 ? 0.0 : (s > 0.999 ? 0.999 : s);
  const double f = floor(256 * cl);
  return f == f ? (uint8_t)(int)f : (uint8_t)0;
}

// RT_FLAG_NAN_ZERO (parity diagnostic, rt.h): a NaN channel of a sample's colour adds 0
__device__ __forceinline__ V3 nan_zero(V3 a) {
  return v3(a.x != a.x ? 0.0 : a.x, a.y != a.y ? 0.0 : a.y, a.z != a.z ? 0.0 : a.z);
}

__device__ __forceinline__ void store_pixel(const RenderArgs& A, long long idx, V3 avg) {
  A.out_rgb[idx * 3 + 0] = scale_color(avg.x);
  A.out_rgb[idx * 3 + 1] = scale_color(avg.y);
  A.out_rgb[idx * 3 + 2] = scale_color(avg.z);
  if (A.out_lin) {
    A.out_lin[idx * 3 + 0] = avg.x;
    A.out_lin[idx * 3 + 1] = avg.y;
    A.out_lin[idx * 3 + 2] = avg.z;
  }
}

// The rest of a segment once its closest hit is known (rayColor, Lib.hs:1309-1333): background,
// emission, or a scatter. Returns true when the path ends (contribution in `contrib`).
template <unsigned F, class R>
__device__ __forceinline__ bool shade_hit(const Scene& S, bool got, const Hit& h, Ray& ray, V3& thr, int& depth, R& g,
                                          V3& contrib, Cnt& cnt) {
  if (!got) {
    contrib = vmul(thr, v3(S.bg[0], S.bg[1], S.bg[2]));
    return true;
  }
  const DMat m = S.mats[h.mat];
  const V3 tx = hit_texture<F>(S, m, h);  // (the kernel's one copy of the texture code)
  if (m.type == RT_MAT_DIFFUSE_LIGHT) {
    contrib = vmul(thr, h.ff ? v3(0, 0, 0) : mat_texture<F>(S, m, h, tx));
    return true;
  }
  Scatter s;
  if constexpr ((F & F_COUNT) != 0) cnt.light += (m.type == RT_MAT_LAMBERTIAN && S.lights >= 0);
  scatter<F>(S, m, ray, h, g, s, tx);
  if (s.specular) {
    thr = vmul(thr, s.att);
  } else {
    const double c = dot(h.n, s.ray.d);
    const double spdf = c < 0 ? 0 : c / kPi;
    const double k = spdf / s.pdf;
    thr = vmul(thr, scale(k, s.att));
  }
  ray = s.ray;
  --depth;
  return false;
}

// One path segment: closest hit, then emission/background or a scatter. Returns true when the
// path ends, with its contribution in `contrib` (rayColor, Lib.hs:1298-1333).
template <unsigned F, class R>
__device__ __forceinline__ bool segment(const RenderArgs& A, const Scene& S, Ray& ray, V3& thr, int& depth, R& g,
                                        int* stk, V3& contrib, Cnt& cnt, int stride = RT_BLOCK,
                                        unsigned long long* t_trav = nullptr) {
  if (depth <= 0) {  // d <= 0 -> black
    contrib = vmul(thr, v3(0.0, 0.0, 0.0));
    return true;
  }
  Hit h;
  // (worlds walked in the reference's order: the recursive walk takes the caller's tree as is)
  const bool got = traverse<F>(S, S.ref_walk ? S.world_ref : S.world, ray, kEps, INFINITY, h, g, stk,
                               !(A.flags & RT_FLAG_REFERENCE_CULL), cnt, stride);
  if constexpr ((F & F_COUNT) != 0) *t_trav = stamp();
  return shade_hit<F>(S, got, h, ray, thr, depth, g, contrib, cnt);
}

// ---------------------------------------------------------------- tier B: Philox per (pixel, sample)
// Wave-reduce a per-lane counter and add it once per wave.
__device__ __forceinline__ void wave_add(unsigned long long* dst, unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
  if ((threadIdx.x & 63) == 0) atomicAdd(dst, v);
}

// The persistent tier-B loop, shared by the global-memory and LDS-staged kernels.
template <unsigned F>
__device__ __forceinline__ void philox_loop(const RenderArgs& A, const Scene& S, int* stk, int stride) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lanes_below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  long long w = -1;  // the current chunk's slot in A.partial
  bool done = false, path = false;
  int px = 0, row = 0, s = 0, s_end = 0, depth = 0;
  Ray ray;
  V3 thr = v3(0, 0, 0), sum = v3(0, 0, 0);
  RngPhilox g;
  g.init(A.seed, 0, 0);
  Cnt cnt{};
  unsigned long long segs = 0, blocks = 0, samples = 0;
  unsigned long long ph_acq = 0, ph_trav = 0, ph_shade = 0, s0 = 0, s1 = 0, s2 = 0;

  for (;;) {
    if constexpr ((F & F_COUNT) != 0) s0 = stamp();
    // acquire pixels for idle lanes: one atomic per wave per round
    for (;;) {
      const bool need = (w < 0) && !done;
      const unsigned long long mask = __ballot(need);
      if (!mask) break;
      const int leader = __ffsll((long long)mask) - 1;
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(A.counter, (unsigned long long)__popcll(mask));
      base = __shfl(base, leader);
      if (need) {
        const long long wi = (long long)(base + __popcll(mask & lanes_below));
        if (wi >= A.work_total) {
          done = true;
        } else if (work_item(A, (uint32_t)wi, px, row, s, s_end, w)) {
          sum = v3(0, 0, 0);
          path = false;
        } else {
          w = -1;
        }
      }
    }
    if (w < 0) break;  // no pixel left for this lane (done); the others keep going
    if (!path) {  // start sample s: uniformRandomUVs' pair, then getRay
      const uint32_t pid = (uint32_t)((long long)row * A.W + px);
      g.init(A.seed, pid, (uint32_t)s);
      g.reserve(3);  // the UV pair and the first disk try
      const double ru = g.draw(), rv = g.draw();
      const int y = A.H - 1 - row;
      const double u = ((double)px + ru) / (double)A.W;
      const double v = ((double)y + rv) / (double)A.H;
      ray = get_ray(A.cam, u, v, g);
      thr = v3(1.0, 1.0, 1.0);
      depth = A.max_depth;
      path = true;
    }
    V3 contrib;
    if constexpr ((F & F_COUNT) != 0) {
      segs += depth > 0;
      s1 = stamp();
      s2 = s1;
    }
    const bool ended = segment<F>(A, S, ray, thr, depth, g, stk, contrib, cnt, stride, &s2);
    if constexpr ((F & F_COUNT) != 0) {
      const unsigned long long s3 = stamp();
      ph_acq += s1 - s0;
      ph_trav += s2 - s1;
      ph_shade += s3 - s2;
    }
    if (ended) {
      if constexpr ((F & F_COUNT) != 0) {
        blocks += g.pair;
        ++samples;
      }
      if (A.flags & RT_FLAG_NAN_ZERO) contrib = nan_zero(contrib);
      sum = sum + contrib;
      path = false;
      ++s;
      const bool all_nan = (A.flags & RT_FLAG_NAN_CULL) && sum.x != sum.x && sum.y != sum.y && sum.z != sum.z;
      if (s == s_end || all_nan) {
        store_partial(A, w, sum);
        w = -1;
      }
    }
  }
  if constexpr ((F & F_COUNT) != 0) {  // lanes re-converge after the loop: one add per wave
    wave_add(&A.work[0], segs);
    wave_add(&A.work[1], cnt.box);
    wave_add(&A.work[2], cnt.prim);
    wave_add(&A.work[3], cnt.other);
    wave_add(&A.work[4], cnt.light);
    wave_add(&A.work[5], blocks);
    wave_add(&A.work[6], samples);
    if ((threadIdx.x & 63) == 0) {  // wave-uniform phase times (s_memtime ticks)
      atomicAdd(&A.work[8], ph_acq);
      atomicAdd(&A.work[9], ph_trav);
      atomicAdd(&A.work[10], ph_shade);
    }
  }
}

template <unsigned F, int WAVES>
__global__ void __launch_bounds__(RT_BLOCK, WAVES) render_philox(RenderArgs A) {
  __shared__ int stk_mem[RT_STACK * RT_BLOCK];
  philox_loop<F>(A, A.S, &stk_mem[threadIdx.x], RT_BLOCK);
}

// LDS-staged variant: one workgroup of WAVES*4 waves per CU; the whole node array is copied
// into LDS once, ahead of the traversal stack, so every node fetch of the traversal's
// dependent chain is an LDS read (~64 cycles) instead of an L2 hit (~200-500 cycles).
template <unsigned F, int WAVES>
__global__ void __launch_bounds__(WAVES * 256, WAVES) render_philox_lds(RenderArgs A, int n_nodes, int stack_entries) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  rt_node* nodes = reinterpret_cast<rt_node*>(lds);
  {
    const uint4* src = reinterpret_cast<const uint4*>(A.S.nodes);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    const int n16 = n_nodes * (int)(sizeof(rt_node) / 16);
    for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  Scene S = A.S;
  S.nodes = nodes;
  int* stk = reinterpret_cast<int*>(lds + (size_t)n_nodes * sizeof(rt_node)) + threadIdx.x;
  (void)stack_entries;
  philox_loop<F>(A, S, stk, WAVES * 256);
}


// Tier-B loop with ray replacement (media-free worlds without instance frames): traversal state
// persists in registers across iterations; each iteration first shades the lanes whose walk has
// ended and starts their next segment (or sample, or pixel), then steps every walking lane one
// node at a time until at most trav_stop/64 of the live lanes are still walking. Lanes never
// wait for the slowest walk of their wave, and shading runs for many lanes at once.
// The replacement loop's per-segment throughput and per-chunk sum: in registers, or (kStateLds: the compact
// LDS-staged spheres kernel, RT_STATE_LDS) in the lane's LDS slots, so that they are not live across the
// walk — the 4-wave kernel spilled them to scratch.
// RT_STATE_LDS: 1 throughput and sum, 2 the throughput only, 0 neither. The compact form's parts are
// separable for A/B runs: RT_COMPACT_STACK16 (16-bit stacks), RT_COMPACT_SLEAF (32-byte sphere leaves).
#ifndef RT_STATE_LDS
#define RT_STATE_LDS 1
#endif
#ifndef RT_COMPACT_STACK16
#define RT_COMPACT_STACK16 1
#endif
#ifndef RT_COMPACT_SLEAF
#define RT_COMPACT_SLEAF 1
#endif
template <unsigned F>
constexpr bool kStateLds = RT_STATE_LDS != 0 && (F & F_SLEAF) != 0;
template <unsigned F>
constexpr bool kSumLds = RT_STATE_LDS == 1 && (F & F_SLEAF) != 0;
// LDS bytes per lane the compact form keeps its state in
constexpr int kStateLdsBytes = RT_STATE_LDS == 1 ? 48 : (RT_STATE_LDS == 2 ? 24 : 0);
template <bool LDS>
struct LaneV3 {
  V3 r;
  double* p;
  int stride;
  __device__ __forceinline__ V3 get() const {
    if constexpr (LDS) return v3(p[0], p[stride], p[2 * stride]);
    return r;
  }
  __device__ __forceinline__ void set(V3 v) {
    if constexpr (LDS) {
      p[0] = v.x;
      p[stride] = v.y;
      p[2 * stride] = v.z;
    } else {
      r = v;
    }
  }
};

template <unsigned F, class STK>
__device__ __forceinline__ void philox_loop2(const RenderArgs& A, const Scene& S, STK* stk, int stride, int* side_p,
                                             volatile uint32_t* wq, double* st = nullptr) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lanes_below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const bool joint = !(A.flags & RT_FLAG_REFERENCE_CULL);

  long long w = -1;  // the current chunk's slot in A.partial
  bool done = false, walking = false, ready = false;
  // wq[0..1]: the wave's claimed, not yet handed out work-items [next, end), in LDS (lanes that
  // are walking skip the acquisition code, so a per-lane copy would go stale); indices are < 2^32
  // (launch_philox checks)
  if (lane == 0) {
    wq[0] = 0u;
    wq[1] = 0u;
  }
  // (the ints only acquisition and shading touch — pixel, row, the chunk's end sample, the path depth —
  // live in LDS after the stacks and Side slots, out of the walk loop's VGPRs; RT_LANE_LDS: 1 the
  // reference-order kernels, 2 every replacement-loop kernel)
  constexpr int kLoop = (F & F_WIDE) ? 2 : 1;
  constexpr bool kLaneLds = lane_lds_of(F, kLoop);
  int l_px = 0, l_row = 0, l_s_end = 0, l_depth = 0;
  int* ex = side_p + side_ints_of(F, S.frames, kLoop) * stride;  // (the host sizes the LDS with the same helpers)
  int& px = kLaneLds ? ex[0] : l_px;
  int& row = kLaneLds ? ex[stride] : l_row;
  int& s_end = kLaneLds ? ex[2 * stride] : l_s_end;
  int& depth = kLaneLds ? ex[3 * stride] : l_depth;
  px = 0, row = 0, s_end = 0, depth = 0;
  int s = 0;
  // (st: the lane's 6 LDS doubles, `stride` apart: throughput xyz, then the chunk's sum xyz)
  LaneV3<kStateLds<F>> thr{v3(0, 0, 0), st, stride};
  LaneV3<kSumLds<F>> sum{v3(0, 0, 0), st + 3 * (kSumLds<F> ? stride : 0), stride};
  // (RT_LEAF_Q: the 4-wide walk's queue word sits below the lane's stack, rt_trace.h trav_postpone)
  if constexpr (RT_LEAF_Q && (F & F_WIDE) != 0) {
    stk[0] = (STK)-1;
    stk += stride;
  }
  RngPhilox g;
  g.init(A.seed, 0, 0);
  Trav t;  // the segment's ray lives only here between segments (no second copy is carried)
  Side side{side_p, stride, S.frames};
  Cnt cnt{};
  if constexpr ((F & F_COUNT) != 0) cnt.prof = A.prof;
  unsigned long long segs = 0, blocks = 0, samples = 0, ph_setup = 0, ph_trav = 0, ph_shade = 0;

  // sample s is over: add its colour; the chunk is done after its last sample
  auto end_sample = [&](V3 contrib) __attribute__((always_inline)) {
    if constexpr ((F & F_COUNT) != 0) {
      blocks += g.pair;
      ++samples;
    }
    if (A.flags & RT_FLAG_NAN_ZERO) contrib = nan_zero(contrib);
    const V3 sm = sum.get() + contrib;
    sum.set(sm);
    ++s;
    const bool all_nan = (A.flags & RT_FLAG_NAN_CULL) && sm.x != sm.x && sm.y != sm.y && sm.z != sm.z;
    if (s == s_end || all_nan) {
      // (a tail unit: its one sample's colour, summed in order with its chunk's others by tail_combine)
      if (kTail<F> && w >= kTailSlot) store_partial_at(A.tail_buf, w - kTailSlot, contrib);
      else store_partial(A, w, sm);
      w = -1;
    }
  };
  auto all_nan3 = [](V3 a) __attribute__((always_inline)) { return a.x != a.x && a.y != a.y && a.z != a.z; };

  for (;;) {
    unsigned long long s0 = 0;
    if constexpr ((F & F_COUNT) != 0) {
      s0 = stamp();
      ++cnt.oslot;
    }
    // ---- shade finished walks, then set up the next walk for every lane that is not walking
    // exact tie, or a NaN-t rect hit in a re-bounded subtree (trav_take: `lite` in a first walk): redo
    // this walk as the reference does (once) — unless the path's throughput is NaN in every channel
    // already: its colour is NaN whichever leaf the reference's order picks (NaN * anything, including
    // the background's 0, is NaN), and a tier-B sample's draws reach no other sample. (NaN-t hits come
    // from the Lambertian quirk's +x ray in a box top's plane, whose pdf is 0 / 0: DESIGN.md §4.3.)
    // hoisted media, taken at the end of a first walk (RT_MEDIA_AFTER; rt_trace.h media_after)
    if constexpr ((F & F_MEDIA) != 0)
      if (ready && !t.redo) media_after<F>(S, t, kEps, cnt, g, side);
    if (ready && (t.tie || (kRefMixed<F> && t.lite)) && !t.redo && !all_nan3(thr.get())) {
      ready = false;
      if constexpr ((F & F_COUNT) != 0) ++cnt.ties;
      trav_redo<F>(t, S.world_ref, INFINITY);
      // (the redo's binary box tests need 1/d: recomputed here, the same values, so that the 4-wide
      // walk need not carry Trav::ray.inv)
      if constexpr ((F & F_WIDE) != 0) t.ray = prep(plain(t.ray));
      walking = true;
    }
    // the next walk's ray: a scattered ray (next segment) or a camera ray (next sample), parked in
    // t.ray (free once the walk's hit is recorded); both kinds of lane start their walk together
    // below, so the walk set-up runs once per wave
    bool start = false;
    if (ready) {
      ready = false;
      Hit h;
      Ray ray = plain(t.ray);  // (every frame has closed: the world ray again)
      const bool got = trav_finish<F>(S, t, ray, kEps, h, side);
      V3 contrib;
      V3 th = thr.get();
      if (shade_hit<F>(S, got, h, ray, th, depth, g, contrib, cnt)) {
        end_sample(contrib);
      } else if (depth <= 0) {  // rayColor's d <= 0 -> black (thr * 0 keeps a NaN throughput NaN)
        end_sample(vmul(th, v3(0.0, 0.0, 0.0)));
      } else {  // next segment of the same path
        thr.set(th);
        t.ray.o = ray.o;
        t.ray.d = ray.d;
        t.ray.tm = ray.tm;
        start = true;
        if constexpr ((F & F_COUNT) != 0) ++segs;
      }
    }
    unsigned long long s0b = 0;
    if constexpr ((F & F_COUNT) != 0) s0b = stamp();
    while (!walking && !start) {
      // acquire work-items for idle lanes: from the wave's claimed range first; when it runs short,
      // one atomic claims a batch of A.batch more (exactly the lanes' need once the counter is near
      // the end, so that no wave hoards the frame's last items)
      for (;;) {
        const bool need = (w < 0) && !done;
        const unsigned long long mask = __ballot(need);
        if (!mask) break;
        const uint32_t n_need = (uint32_t)__popcll(mask);
        const uint32_t q_next = wq[0], q_end = wq[1];
        const uint32_t avail = q_end - q_next;
        uint32_t base2 = q_next, end2 = q_end;  // items past `avail` come from a new claim
        if (avail < n_need) {
          const int leader = __ffsll((long long)mask) - 1;
          unsigned long long claim = 0;
          if (lane == leader) {
            // batch: A.batch items, fewer as the frame runs out (the wave's last claim end tells it
            // roughly how many remain), so that no wave hoards the tail; never less than the need
            const uint32_t want = n_need - avail;
            const long long rem = A.work_total - (long long)q_end;
            const uint32_t b = rem <= 0 ? 0u : max((uint32_t)A.batch_floor,
                                                   (uint32_t)fminf((float)A.batch, (float)rem * A.batch_per_item));
            const uint32_t got = want < b ? b : want;
            const unsigned long long c0 = atomicAdd(A.counter, (unsigned long long)got);
            // (claims past 2^32 only happen once every item is handed out: clamp, the lanes see
            // `done`); the claim and its size travel together in one broadcast
            claim = (c0 < 0xffff0000ull ? c0 : 0xffff0000ull) | ((unsigned long long)got << 32);
          }
          const unsigned long long c1 = __shfl(claim, leader);
          base2 = (uint32_t)c1;
          end2 = base2 + (uint32_t)(c1 >> 32);
        }
        const uint32_t rank = (uint32_t)__popcll(mask & lanes_below);
        if (need) {
          const long long wi = (long long)(rank < avail ? q_next + rank : base2 + (rank - avail));
          if (wi >= A.work_total) {
            done = true;
          } else if (kTail<F> ? work_unit(A, (uint32_t)wi, px, row, s, s_end, w)
                              : work_item(A, (uint32_t)wi, px, row, s, s_end, w)) {
            sum.set(v3(0, 0, 0));
          } else {
            w = -1;
          }
        }
        const int leader = __ffsll((long long)mask) - 1;
        if (lane == leader) {
          wq[0] = avail < n_need ? base2 + (n_need - avail) : q_next + n_need;
          wq[1] = end2;
        }
      }
      if (w < 0) break;  // no work left for this lane
      // start sample s: uniformRandomUVs' pair, then getRay
      const uint32_t pid = (uint32_t)((long long)row * A.W + px);
      g.init(A.seed, pid, (uint32_t)s);
      g.reserve(3);  // the UV pair and the first disk try
      const double ru = g.draw(), rv = g.draw();
      const int y = A.H - 1 - row;
      const double u = ((double)px + ru) / (double)A.W;
      const double v = ((double)y + rv) / (double)A.H;
      const Ray cray = get_ray(A.cam, u, v, g);
      t.ray.o = cray.o;
      t.ray.d = cray.d;
      t.ray.tm = cray.tm;
      thr.set(v3(1.0, 1.0, 1.0));
      depth = A.max_depth;
      if (depth <= 0) {
        end_sample(vmul(v3(1.0, 1.0, 1.0), v3(0.0, 0.0, 0.0)));
        continue;
      }
      start = true;
      if constexpr ((F & F_COUNT) != 0) ++segs;
    }
    if (start) {
      trav_begin<F>(t, plain(t.ray), S.world, kEps, INFINITY);
      // worlds with media or frames: the reference's order over the re-bounded skeleton
      if (S.ref_walk) trav_restart_ref(t, S.world, INFINITY);
      trav_media_first<F>(S, t, kEps, cnt, g, side);  // (hoisted media: RT_BVH_MEDIA_FIRST, RT_MEDIA_AFTER=0)
      t.node = media_rest<F>(S, t.node);               // (RT_MEDIA_AFTER: they are taken when the walk ends)
      walking = true;
    }
    if (!walking) break;  // this lane is finished; the rest of the wave carries on without it
    unsigned long long s1 = 0;
    if constexpr ((F & F_COUNT) != 0) s1 = stamp();
    // ---- walk until few lanes are still walking
    const int live = __popcll(__ballot(true));
    const int stop = (live * A.trav_stop) >> 6;
    const int ls = (F & F_WIDE) ? A.leaf_stop : A.box_first;
    walk_until<F>(S, t, walking, kEps, stk, stride, joint, stop, (live * ls) >> 6, cnt, g, side, A.med_batch);
    ready = !walking;
    if constexpr ((F & F_COUNT) != 0) {
      const unsigned long long s2 = stamp();
      ph_shade += s0b - s0;
      ph_setup += s1 - s0b;
      ph_trav += s2 - s1;
    }
  }
  if constexpr ((F & F_COUNT) != 0) {
    wave_add(&A.work[0], segs);
    wave_add(&A.work[1], cnt.box);
    wave_add(&A.work[2], cnt.prim);
    wave_add(&A.work[3], cnt.other);
    wave_add(&A.work[4], cnt.light);
    wave_add(&A.work[5], blocks);
    wave_add(&A.work[6], samples);
    wave_add(&A.work[7], cnt.wide);
    wave_add(&A.work[11], cnt.islot);
    wave_add(&A.work[12], cnt.lslot);
    wave_add(&A.work[13], cnt.oslot);
    wave_add(&A.work[14], cnt.phit);
    wave_add(&A.work[15], cnt.ties);
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&A.work[8], ph_setup);
      atomicAdd(&A.work[9], ph_trav);
      atomicAdd(&A.work[10], ph_shade);
    }
  }
}

// LDS ints per lane of a kernel: the traversal stack, then (instance frames possible) Side slots
template <unsigned F>
constexpr int lane_ints() {
  return ((F & F_W8) ? 2 * RT_WSTACK : ((F & (F_WIDE | F_MIXW)) ? RT_WSTACK : RT_STACK)) + ((F & F_FRAMES) ? kSideInts : 0);
}

// Global-memory replacement loop: the lane stacks (and Side slots) in dynamic LDS sized by the host
// for the world's stack bound (`stack_entries` per lane), not for the RT_STACK / RT_WSTACK maxima:
// the LDS per workgroup then does not cap the occupancy (C4: 54 -> 40 ints per lane, 2.5 -> 3 waves
// per SIMD).
template <unsigned F, int WAVES>
__global__ void __launch_bounds__(RT_BLOCK, WAVES) render_philox2(RenderArgs A, int stack_entries) {
  extern __shared__ __attribute__((aligned(16))) int stk_mem[];
  __shared__ uint32_t wave_q[RT_BLOCK / 64][2];
  philox_loop2<F>(A, A.S, &stk_mem[threadIdx.x], RT_BLOCK, &stk_mem[stack_entries * RT_BLOCK + threadIdx.x],
                  wave_q[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)]);
}

// LDS-staged replacement loop: the traversal's node array (the wide records for F_WIDE, else the
// flat nodes) and the per-lane stacks live in the CU's LDS; leaves are read from global memory
// under F_WIDE.
// LEAF_LDS: the 4-wide walk's leaf table is staged too (n_leaves > 0); as its own instantiation,
// so that the leaf reads compile to ds_read (a pointer that is LDS or global at run time would
// make them flat loads, which wait on both the vector-memory and LDS counters).
template <unsigned F, int WAVES, bool LEAF_LDS = false>
__global__ void __launch_bounds__(WAVES * 256, WAVES)
    render_philox2_lds(RenderArgs A, int n_nodes, int stack_entries, int n_leaves) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ uint32_t wave_q[WAVES * 4][2];  // (static: kStaticLds bytes ahead of the dynamic LDS)
  constexpr int rec = (F & F_WIDE) ? (int)sizeof(rt_wnode) : (int)sizeof(rt_node);
  // The compact form (F_SLEAF, round 6; spheres-only worlds): the leaf table staged as the leaves' 32-byte
  // sphere quadruples (Scene::sleaves; the 64-byte records stay in global memory for trav_finish, once per
  // segment), 16-bit lane stacks (the staged tree's node ids, leaf slots and — in tie redos — the flat ids
  // of a world whose tree fits the LDS all fit 15 bits, and an F_WIDE kernel masks a flat id's kind tags off
  // anyway), and the lanes' throughput and chunk sums in LDS (kStateLds): VERDICT r5 item 3.
  constexpr bool kCompact = (F & F_SLEAF) != 0;
  constexpr bool kSleaf = kCompact && RT_COMPACT_SLEAF;
  constexpr int lrec = kSleaf ? 32 : (int)sizeof(rt_node);
  using STK = typename std::conditional<kCompact && RT_COMPACT_STACK16, short, int>::type;
  {
    const uint4* src = (F & F_WIDE) ? reinterpret_cast<const uint4*>(A.S.wnodes)
                                    : reinterpret_cast<const uint4*>(A.S.nodes);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    const int n16 = n_nodes * (rec / 16);
    for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
    // F_WIDE: the leaf table too, when it fits (n_leaves > 0)
    const uint4* lsrc = kSleaf ? reinterpret_cast<const uint4*>(A.S.sleaves) : reinterpret_cast<const uint4*>(A.S.leaves);
    uint4* ldst = reinterpret_cast<uint4*>(lds + (size_t)n_nodes * rec);
    const int l16 = n_leaves * (lrec / 16);
    for (int i = threadIdx.x; i < l16; i += blockDim.x) ldst[i] = lsrc[i];
  }
  __syncthreads();
  Scene S = A.S;
  if constexpr ((F & F_WIDE) != 0) S.wnodes = reinterpret_cast<const rt_wnode*>(lds);
  else S.nodes = reinterpret_cast<const rt_node*>(lds);
  if constexpr (kSleaf) S.sleaves = reinterpret_cast<const double*>(lds + (size_t)n_nodes * rec);
  else if constexpr (LEAF_LDS) S.leaves = reinterpret_cast<const rt_node*>(lds + (size_t)n_nodes * rec);
  else n_leaves = 0;
  constexpr int lanes = WAVES * 256;
  unsigned char* lane_base = lds + (size_t)n_nodes * rec + (size_t)n_leaves * lrec;
  STK* stk = reinterpret_cast<STK*>(lane_base) + threadIdx.x;
  // (per lane: stack_entries stack entries, then side_ints_of Side slots, then lane_lds_of's 4 lane ints —
  // launch_philox sizes the dynamic LDS with the same helpers — and for kStateLds 6 doubles after them)
  int* side_p = reinterpret_cast<int*>(lane_base + (size_t)stack_entries * lanes * sizeof(STK)) + threadIdx.x;
  double* st = nullptr;
  if constexpr (kStateLds<F>) {
    const int side_total = side_ints_of(F, S.frames, 2) + (lane_lds_of(F, 2) ? 4 : 0);
    st = reinterpret_cast<double*>(lane_base + (size_t)stack_entries * lanes * sizeof(STK) +
                                   (size_t)side_total * lanes * sizeof(int)) + threadIdx.x;
  }
  philox_loop2<F>(A, S, stk, lanes, side_p, wave_q[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], st);
}

// The tail's work-items (work_unit): each chunk's sample colours added in sample order from 0, as the
// lane that renders a whole chunk adds them (end_sample), into the chunk's slot.
__global__ void __launch_bounds__(256) tail_combine(RenderArgs A) {
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  if (j >= A.items_total - A.tail_start) return;
  int px, row, s0, s1;
  long long slot;
  if (!work_item(A, (uint32_t)(A.tail_start + j), px, row, s0, s1, slot)) return;
  const double* q = A.tail_buf + j * A.chunk * 3;
  V3 sum = v3(0, 0, 0);
  for (int k = 0; k < s1 - s0; ++k) sum = sum + v3(q[3 * k], q[3 * k + 1], q[3 * k + 2]);
  store_partial(A, slot, sum);
}

// Tier B: a slab pixel's chunk sums added in chunk order, then averaged and stored (rt.h); with chunk
// batches, each batch's chunks are added to the running sum of the batches before it.
__global__ void __launch_bounds__(256) combine_chunks(RenderArgs A) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= A.slab) return;
  int px, row;
  if (!work_pixel(A, (uint32_t)idx, px, row)) return;  // outside the image: never assembled
  V3 acc = (A.combine & 1) ? vload(A.acc + idx * 3) : v3(0, 0, 0);
  for (int k = 0; k < A.chunks; ++k) {
    const double* q = A.partial + ((long long)k * A.slab + idx) * 3;
    acc = acc + v3(q[0], q[1], q[2]);
  }
  if (A.combine & 2) {
    store_pixel(A, idx, divide(acc, (double)A.spp));
  } else {  // a batch of chunks before the last: keep the running sum
    A.acc[idx * 3 + 0] = acc.x;
    A.acc[idx * 3 + 1] = acc.y;
    A.acc[idx * 3 + 2] = acc.z;
  }
}

// ---------------------------------------------------------------- tier A: the reference's stream
// One lane per image column; rows top to bottom; each pixel draws its 2*ns UVs first and uses
// them in reverse draw order (uniformRandomUVs' foldr, Lib.hs:1358-1371) — the UV pairs are
// recomputed from the pixel's starting state (SplitMix is seed + k*gamma), no list is stored.
// Columns per wave of the tier-A kernel (lanes 0..k-1 of each wave; 64: every lane).
#ifndef RT_EXACT_COLS_PER_WAVE
#define RT_EXACT_COLS_PER_WAVE 1
#endif
constexpr int kExactColsPerWave = RT_EXACT_COLS_PER_WAVE;
// LDS (round 5): the whole node array staged in the block's LDS when it fits (n_nodes records; the
// launch sizes the dynamic LDS). Tier A runs one lane per column, so few waves hold the GPU and each
// dependent node read's latency is the lane's own time: from L2 it cost the Cornell box ~10x the
// 16-thread CPU oracle's time.
template <unsigned F, bool LDS = false>
__global__ void __launch_bounds__(RT_BLOCK) render_exact(RenderArgs A, int n_nodes) {
  __shared__ int stk_mem[RT_STACK * RT_BLOCK];
  int* stk = &stk_mem[threadIdx.x];
  // Tier A reproduces the reference's stream exactly, exact ties included: walk the caller's tree.
  Scene S = A.S;
  S.world = S.world_ref;
  if constexpr (LDS) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_nodes[];
    const uint4* src = reinterpret_cast<const uint4*>(A.S.nodes);
    uint4* dst = reinterpret_cast<uint4*>(lds_nodes);
    const int n16 = n_nodes * (int)(sizeof(rt_node) / 16);
    for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    S.nodes = reinterpret_cast<const rt_node*>(lds_nodes);
  }
  // One column per wave, on its lane 0: a column is one serial chain of draws (the stream threads every
  // row, sample and bounce), so a wave of 64 columns ran every sample at its slowest lane's path length
  // and through every lane's branches; alone, a lane runs only its own (RT_EXACT_COLS_PER_WAVE).
  const int x = blockIdx.x * (RT_BLOCK / 64) * kExactColsPerWave + (int)(threadIdx.x >> 6) * kExactColsPerWave +
                (int)(threadIdx.x & 63);
  if ((int)(threadIdx.x & 63) >= kExactColsPerWave || x >= A.W) return;
  RngExactT<kSL<F>> g{A.gens[2 * x], A.gens[2 * x + 1]};
  const bool traced = A.trace && x == A.trace_col;
  int tn = 0;
  const int ns = A.spp;
  for (int row = 0; row < A.H; ++row) {
    const int y = A.H - 1 - row;
    const uint64_t seed0 = g.seed;
    g.seed += (uint64_t)(2 * (long long)ns) * g.gamma;
    V3 sum = v3(0, 0, 0);
    for (int j = 0; j < ns; ++j) {
      const int i = ns - 1 - j;
      const double ru = word_to_draw(mix64(seed0 + (uint64_t)(2 * i + 1) * g.gamma));
      const double rv = word_to_draw(mix64(seed0 + (uint64_t)(2 * i + 2) * g.gamma));
      const double u = ((double)x + ru) / (double)A.W;
      const double v = ((double)y + rv) / (double)A.H;
      Ray ray = get_ray(A.cam, u, v, g);
      V3 thr = v3(1.0, 1.0, 1.0), contrib;
      int depth = A.max_depth;
      Cnt cnt{};
      for (int seg = 0;; ++seg) {
        const bool end = segment<F>(A, S, ray, thr, depth, g, stk, contrib, cnt);
        if (traced && tn < A.trace_cap) {  // (rt_debug_exact_trace: the oracle's oracle_exact_trace layout)
          double* o = A.trace + 10 * (long long)tn++;
          o[0] = row, o[1] = j, o[2] = end ? -(seg + 1) : seg;
          o[3] = ray.o.x, o[4] = ray.o.y, o[5] = ray.o.z, o[6] = ray.d.x, o[7] = ray.d.y, o[8] = ray.d.z;
          o[9] = __longlong_as_double((long long)g.seed);
        }
        if (end) break;
      }
      if (A.flags & RT_FLAG_NAN_ZERO) contrib = nan_zero(contrib);
      sum = sum + contrib;
    }
    store_pixel(A, (long long)row * A.W + x, divide(sum, (double)ns));
  }
  A.gens[2 * x] = g.seed;
  if (traced) *A.trace_n = tn;
}

// ---------------------------------------------------------------- slab -> image
template <class T>
__global__ void assemble(const T* slabs, T* image, int W, int H, int tile, int tiles_x, int shards,
                         long long slab_pixels) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)W * H) return;
  const int row = (int)(i / W), px = (int)(i % W);
  const int gt = (row / tile) * tiles_x + (px / tile);
  const int shard = gt % shards;
  const long long lt = gt / shards;
  const int bpr = tile >> 3;
  const int bx = (px % tile) >> 3, by = (row % tile) >> 3;
  const int within = (by * bpr + bx) * 64 + (row & 7) * 8 + (px & 7);
  const long long src = (long long)shard * slab_pixels + lt * tile * tile + within;
  image[i * 3 + 0] = slabs[src * 3 + 0];
  image[i * 3 + 1] = slabs[src * 3 + 1];
  image[i * 3 + 2] = slabs[src * 3 + 2];
}

// ---------------------------------------------------------------- debug: closest hits
template <unsigned F>
__global__ void __launch_bounds__(RT_BLOCK) closest_hits(Scene S, const double* rays, int n, double tmin,
                                                         double tmax, uint64_t seed, int joint, int walk, double* out) {
  __shared__ int stk_mem[(lane_ints<F>() + 1) * RT_BLOCK];
  int* stk = &stk_mem[threadIdx.x];
  Side side{&stk_mem[(((F & F_W8) ? 2 * RT_WSTACK : ((F & (F_WIDE | F_MIXW)) ? RT_WSTACK : RT_STACK)) + 1) * RT_BLOCK +
                     threadIdx.x],
            RT_BLOCK};
  if constexpr (RT_LEAF_Q && (F & F_WIDE) != 0) {  // (the leaf queue word below the stack)
    stk[0] = -1;
    stk += RT_BLOCK;
  }
  const int i = blockIdx.x * RT_BLOCK + threadIdx.x;
  if (i >= n) return;
  const double* q = rays + 7 * (long long)i;
  const Ray r{v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), q[6]};
  RngPhilox g;
  g.init(seed, (uint32_t)i, 0);
  Hit h;
  double* o = out + 12 * (long long)i;
  Cnt cnt{};
  bool got;
  if (walk == 0) {
    got = traverse<F>(S, S.ref_walk ? S.world_ref : S.world, r, tmin, tmax, h, g, stk, joint != 0, cnt);
  } else {  // the render loop's resumable walk (binary, or 4-wide under F_WIDE)
    Trav t;
    trav_begin<F>(t, r, S.world, tmin, tmax);
    if (S.ref_walk) trav_restart_ref(t, S.world, tmax);  // (the re-bounded skeleton, mixed walk)
    trav_media_first<F>(S, t, tmin, cnt, g, side);        // (hoisted media as the render loop takes them)
    t.node = media_rest<F>(S, t.node);
    bool walking = true;
    walk_until<F>(S, t, walking, tmin, stk, RT_BLOCK, joint != 0, 0, 0, cnt, g, side);
    media_after<F>(S, t, tmin, cnt, g, side);
    if (t.tie || (kRefMixed<F> && t.lite)) {
      trav_redo<F>(t, S.world_ref, tmax);
      while (trav_step<F>(S, t, tmin, stk, RT_BLOCK, joint != 0, cnt, g, side)) {
      }
    }
    got = trav_finish<F>(S, t, r, tmin, h, side);
  }
  if (got) {
    o[0] = 1; o[1] = h.t;
    o[2] = h.p.x; o[3] = h.p.y; o[4] = h.p.z;
    o[5] = h.n.x; o[6] = h.n.y; o[7] = h.n.z;
    o[8] = h.u; o[9] = h.v; o[10] = h.ff; o[11] = h.mat;
  } else {
    for (int k = 0; k < 12; ++k) o[k] = 0;
  }
}

// ---------------------------------------------------------------- debug: per-function probes
// The hot-path functions one at a time on device inputs (rt_debug_probe; layouts in rt.h and
// oracle/oracle.c oracle_probe): record i draws from its own tier-B Philox stream (key = seed, pid = i,
// sample 0), so the oracle's golden vectors consume the same numbers.
constexpr int kProbeIn[6] = {18, 3, 6, 6, 2, 14}, kProbeOut[6] = {14, 4, 2, 3, 8, 3};
template <unsigned F>
__global__ void __launch_bounds__(RT_BLOCK) fn_probe(Scene S, rt_camera cam, int op, const double* in, int n,
                                                    uint64_t seed, double* out) {
  const int i = blockIdx.x * RT_BLOCK + threadIdx.x;
  if (i >= n) return;
  const double* q = in + (long long)kProbeIn[op] * i;
  double* o = out + (long long)kProbeOut[op] * i;
  for (int k = 0; k < kProbeOut[op]; ++k) o[k] = 0.0;
  RngPhilox g;
  g.init(seed, (uint32_t)i, 0);
  if (op == 0) {  // scatter (or emitted for DiffuseLight), as shade_hit runs it
    const Ray r{v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), q[6]};
    Hit h;
    h.t = q[7];
    h.p = v3(q[8], q[9], q[10]);
    h.n = v3(q[11], q[12], q[13]);
    h.u = q[14];
    h.v = q[15];
    h.ff = (int)q[16];
    h.mat = (int)q[17];
    const DMat m = S.mats[h.mat];
    const V3 tx = hit_texture<F>(S, m, h);
    if (m.type == RT_MAT_DIFFUSE_LIGHT) {
      const V3 e = h.ff ? v3(0, 0, 0) : mat_texture<F>(S, m, h, tx);
      o[8] = e.x, o[9] = e.y, o[10] = e.z;
    } else {
      Scatter sc;
      scatter<F>(S, m, r, h, g, sc, tx);
      o[0] = 1;
      o[1] = sc.ray.o.x, o[2] = sc.ray.o.y, o[3] = sc.ray.o.z;
      o[4] = sc.ray.d.x, o[5] = sc.ray.d.y, o[6] = sc.ray.d.z, o[7] = sc.ray.tm;
      o[8] = sc.att.x, o[9] = sc.att.y, o[10] = sc.att.z;
      o[11] = sc.pdf;
      o[12] = sc.specular;
    }
    o[13] = g.consumed();
  } else if (op == 1) {  // htblRandom on the lights tree
    const V3 d = htbl_random(S, S.lights, v3(q[0], q[1], q[2]), g);
    o[0] = d.x, o[1] = d.y, o[2] = d.z;
    o[3] = g.consumed();
  } else if (op == 2) {  // htblPdfValue on the lights tree
    const V3 org = v3(q[0], q[1], q[2]), v = v3(q[3], q[4], q[5]);
    o[0] = S.lights < 0 ? 0.0 : htbl_pdf_value<F, RT_LIGHT_DEPTH>(S, S.lights, org, v, prep(Ray{org, v, 0.0}));
    o[1] = g.consumed();
  } else if (op == 3) {  // textureValue
    const V3 a = texture_value<F>(S, (int)q[0], q[1], q[2], v3(q[3], q[4], q[5]));
    o[0] = a.x, o[1] = a.y, o[2] = a.z;
  } else if (op == 5) {  // the box test: division-free (the walks'), with divisions, the reference's per-axis
    const RayX r = prep(Ray{v3(q[6], q[7], q[8]), v3(q[9], q[10], q[11]), 0.0});
    o[0] = box_hit(q, r, q[12], q[13], true);
    o[1] = box_hit_exact(q, r, q[12], q[13], true);
    o[2] = box_hit_exact(q, r, q[12], q[13], false);
  } else {  // getRay
    const Ray r = get_ray(cam, q[0], q[1], g);
    o[0] = r.o.x, o[1] = r.o.y, o[2] = r.o.z;
    o[3] = r.d.x, o[4] = r.d.y, o[5] = r.d.z, o[6] = r.tm;
    o[7] = g.consumed();
  }
}

// ---------------------------------------------------------------- debug: numerics probe
__global__ void math_probe(int op, const double* x, const double* y, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = x[i], b = y[i];
  double r;
  switch (op) {
    case 0: r = a / b; break;
    case 1: r = div_exact(a, b, 1.0 / b); break;
    case 2: r = sqrt(a); break;
    case 3: r = sin(a); break;
    case 4: r = cos(a); break;
    case 5: r = atan(a); break;
    case 6: r = asin(a); break;
    case 7: r = log(a); break;
    case 8: r = pow(a, b); break;
    case 9: r = ghc_atan2(a, b); break;
    case 11: r = pow5(a); break;
    // the shared portable functions (include/rt_libm.h; RT_FLAG_SHARED_LIBM)
    case 12: r = rtlm_sin(a); break;
    case 13: r = rtlm_cos(a); break;
    case 14: r = rtlm_atan(a); break;
    case 15: r = rtlm_asin(a); break;
    case 16: r = rtlm_log(a); break;
    case 17: r = ghc_atan2<true>(a, b); break;
    default: r = tan(a); break;
  }
  out[i] = r;
}



// Kernel pointer for (variant, loop, LDS-staged?, waves per SIMD, counting build?); loop 0 = one
// sample per lane walk, 1 = ray replacement over the binary tree, 2 = replacement over the
// 4-wide tree.
template <unsigned V>
const void* pick_w(bool lds, int w, bool leaf_lds = false, bool q = false, bool w8 = false) {
  if constexpr (V == (kVarSpheres | F_WIDE)) {
    if (!lds && w8) {  // (the 8-wide tree as record pairs, from global memory: A/B)
      if (w == 2) return (const void*)render_philox2<V | F_W8, 2>;
      if (w == 4) return (const void*)render_philox2<V | F_W8, 4>;
      return (const void*)render_philox2<V | F_W8, 3>;
    }
  }
  if constexpr (V == (kVarSpheres | F_WIDE)) {
    if (!lds && q) {  // (the quantised tree and sphere quadruples from global memory)
      if (w == 2) return (const void*)render_philox2<V | F_QNODE, 2>;
      if (w == 3) return (const void*)render_philox2<V | F_QNODE, 3>;
      if (w == 4) return (const void*)render_philox2<V | F_QNODE, 4>;
      return (const void*)render_philox2<V | F_QNODE, 1>;
    }
  }
  if constexpr (V == (kVarSpheres | F_WIDE)) {
    if (lds && leaf_lds && q) {  // the compact LDS form: sphere quadruples, 16-bit stacks, state in LDS
      if (w == 4) return (const void*)render_philox2_lds<V | F_SLEAF, 4, true>;
      if (w == 3) return (const void*)render_philox2_lds<V | F_SLEAF, 3, true>;
    }
  }
  if constexpr ((V & F_WIDE) != 0) {
    if (lds && leaf_lds) {
      if (w == 4) return (const void*)render_philox2_lds<V, 4, true>;
      if (w == 2) return (const void*)render_philox2_lds<V, 2, true>;
      if (w == 3) return (const void*)render_philox2_lds<V, 3, true>;
    }  // (1 wave: the leaves are read from global memory)
  }
  if (lds) {
    if (w == 2) return (const void*)render_philox2_lds<V, 2>;
    if (w == 4) return (const void*)render_philox2_lds<V, 4>;
    if (w == 1) return (const void*)render_philox2_lds<V, 1>;
    return (const void*)render_philox2_lds<V, 3>;
  }
  if (w == 2) return (const void*)render_philox2<V, 2>;
  if (w == 3) return (const void*)render_philox2<V, 3>;
  if (w == 4) return (const void*)render_philox2<V, 4>;
  return (const void*)render_philox2<V, 1>;
}
template <unsigned V>
const void* pick(int loop, bool lds, int w, bool count, bool leaf_lds, bool q = false, bool w8 = false) {
  if (count) {
    if constexpr (V == kVarSpheres) {
      if (loop == 2 && w8) return (const void*)render_philox2<V | F_WIDE | F_COUNT | F_W8, 1>;
      if (loop == 2 && q) return (const void*)render_philox2<V | F_WIDE | F_COUNT | F_QNODE, 1>;
    }
    if (loop == 2) return (const void*)render_philox2<V | F_WIDE | F_COUNT, 1>;
    return loop ? (const void*)render_philox2<V | F_COUNT, 1> : (const void*)render_philox<V | F_COUNT, 1>;
  }
  if (loop == 2) return pick_w<V | F_WIDE>(lds, w, leaf_lds, q, w8);
  if (loop == 1) return pick_w<V>(lds, w);
  if (lds) {
    if (w == 2) return (const void*)render_philox_lds<V, 2>;
    if (w == 4) return (const void*)render_philox_lds<V, 4>;
    if (w == 1) return (const void*)render_philox_lds<V, 1>;
    return (const void*)render_philox_lds<V, 3>;
  }
  if (w == 2) return (const void*)render_philox<V, 2>;
  if (w == 3) return (const void*)render_philox<V, 3>;
  if (w == 4) return (const void*)render_philox<V, 4>;
  return (const void*)render_philox<V, 1>;
}
// full variants (media, frames, textures, motion): ray replacement over the caller's tree in the
// reference's order (loop 1), or the per-sample loop (loop 0)
template <unsigned V>
const void* pick_full(int loop, bool lds, int w, bool count) {
  if (count) return loop ? (const void*)render_philox2<V | F_COUNT, 1> : (const void*)render_philox<V | F_COUNT, 1>;
  if (loop) {
    if (lds) return w >= 3 ? (const void*)render_philox2_lds<V, 3> : (const void*)render_philox2_lds<V, 2>;
    if (w >= 4) return (const void*)render_philox2<V, 4>;  // (RTAMD_WAVES=4: A/B only)
    return w >= 3 ? (const void*)render_philox2<V, 3> : (const void*)render_philox2<V, 2>;
  }
  return w >= 2 ? (const void*)render_philox<V, 2> : (const void*)render_philox<V, 1>;
}

}  // namespace

// Render-kernel tables, one per kernel translation unit: the kernel for (loop, LDS-staged?, waves per
// SIMD, counting build?, leaf table in LDS?) of that unit's variant(s).
namespace rt {
const void* philox_kernel_spheres(int loop, bool lds, int w, bool count, bool leaf_lds, bool q, bool w8);
const void* philox_kernel_spheres_global(int w);  // rt_k_spheres_global.hip
const void* philox_kernel_cornell(int loop, bool lds, int w, bool count, bool leaf_lds);
const void* philox_kernel_full(int loop, bool lds, int w, bool count);
const void* philox_kernel_full_dark(int loop, bool lds, int w, bool count);
}  // namespace rt
