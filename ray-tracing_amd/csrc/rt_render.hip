// rt_render.hip — render kernels for gfx950 and the device half of the C ABI (include/rt.h).
//
// Kernel design:
//  * tier B work-items are (pixel, chunk of up to 32 samples): a lane sums its chunk in sample
//    order and stores the sum; `combine_chunks` adds a pixel's chunk sums in chunk order (rt.h);
//  * persistent waves with ray replacement (`philox_loop2`): the closest-hit walk is resumable;
//    each iteration shades the lanes whose walk ended and starts their next segment, sample or
//    work-item (one wave-aggregated atomicAdd on a work counter), then steps the walking lanes
//    until few still walk — a wave never waits for its slowest walk;
//  * the 4-wide fp32-box walk postpones leaves so wide-node steps and fp64 leaf tests do not
//    share a divergent step; worlds with media or instance frames walk the caller's tree in the
//    reference's own order (media draws);
//  * forward throughput (thr *= att * (spdf / pdf)) instead of the reference's continuation;
//    colour never feeds control flow or the RNG, so this changes rounding only;
//  * traversal stacks live in LDS, [entry][lane] so consecutive lanes hit consecutive banks;
//  * tier B (Philox per (pixel, sample)) shards by tiles with no data-path collective; tier A
//    (the reference's per-column SplitMix stream) runs one lane per column.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt.h"
#include "rt_device.h"
#include "rt_internal.h"
#include "rt_trace.h"

namespace rt {
int rebuild_world_bvh(std::vector<rt_node>& nodes, int root);
int rebuild_for_device(std::vector<rt_node>& nodes, int root);
bool build_wide_bvh(const std::vector<rt_node>& nodes, int root, std::vector<rt_wnode>& out, int* stack_need);
}

using namespace rtd;

namespace {

// Wave-level timestamp for the counting build's phase split (MI355X_MICROARCH.md / HIP guide
// "In-kernel stamps": one asm statement with its own lgkmcnt wait, fenced by sched barriers).
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

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
  long long work_total;  // work-items of this shard: slab pixels x sample chunks (< 2^32)
  long long slab;        // slab pixels of this shard
  int chunk, chunks;     // tier B: samples per chunk (rt_sample_chunk) and chunks per pixel
  UDiv div_tp, div_tile, div_tiles_x, div_bpr;  // by tile*tile, tile*tile*chunks, tiles_x, tile/8
  double* partial;       // tier B: chunk sums, [chunk][slab pixel][3]
  uint64_t seed;
  unsigned long long* counter;
  unsigned long long* work;  // counting build: [segments, box, prim, other, light, blocks, samples]
  int trav_stop;             // replacement loop: keep stepping while > trav_stop/64 of live lanes walk
  int batch;                 // replacement loop: most work-items a wave claims per atomic
  float batch_per_item;      // ...tapering to rem * batch_per_item as `rem` items remain (>= need)
  int leaf_stop;             // 4-wide walk: leaf step once <= leaf_stop/64 of live lanes seek a leaf
  int box_first;             // binary walk: box-only steps while > box_first/64 of live lanes are at BVH
                             // nodes (64: never)
  uint8_t* out_rgb;  // tier B: slab; tier A: image
  double* out_lin;
  uint64_t* gens;  // tier A: per-column (seed, gamma), updated in place
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
  const uint32_t lt = udiv(wi, A.div_tile);  // by tp * chunks
  const uint32_t rem = wi - lt * tp * (uint32_t)A.chunks;
  const uint32_t k = udiv(rem, A.div_tp);
  const uint32_t idx = lt * tp + (rem - k * tp);
  if (!work_pixel(A, idx, px, row)) return false;
  s0 = (int)k * A.chunk;
  s1 = min(A.spp, s0 + A.chunk);
  slot = (long long)k * A.slab + idx;
  return s0 < s1;
}
__device__ __forceinline__ void store_partial(const RenderArgs& A, long long slot, V3 sum) {
  double* q = A.partial + slot * 3;
  q[0] = sum.x;
  q[1] = sum.y;
  q[2] = sum.z;
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
  if (!got) {
    contrib = vmul(thr, v3(S.bg[0], S.bg[1], S.bg[2]));
    return true;
  }
  const DMat m = S.mats[h.mat];
  if (m.type == RT_MAT_DIFFUSE_LIGHT) {  // scatter -> Nothing: emitted (Lib.hs:880-885)
    const V3 e = h.ff ? v3(0, 0, 0) : texture_value<F>(S, m.tex, h.u, h.v, h.p);
    contrib = vmul(thr, e);
    return true;
  }
  Scatter s;
  if constexpr ((F & F_COUNT) != 0) cnt.light += (m.type == RT_MAT_LAMBERTIAN && S.lights >= 0);
  scatter<F>(S, m, ray, h, g, s);
  if (s.specular) {
    thr = vmul(thr, s.att);
  } else {
    const double c = dot(h.n, s.ray.d);  // scatteringPdf (Lib.hs:874-878)
    const double spdf = c < 0 ? 0 : c / kPi;
    const double k = spdf / s.pdf;
    thr = vmul(thr, scale(k, s.att));
  }
  ray = s.ray;
  --depth;
  return false;
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
  if (m.type == RT_MAT_DIFFUSE_LIGHT) {
    const V3 e = h.ff ? v3(0, 0, 0) : texture_value<F>(S, m.tex, h.u, h.v, h.p);
    contrib = vmul(thr, e);
    return true;
  }
  Scatter s;
  if constexpr ((F & F_COUNT) != 0) cnt.light += (m.type == RT_MAT_LAMBERTIAN && S.lights >= 0);
  scatter<F>(S, m, ray, h, g, s);
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
template <unsigned F>
__device__ __forceinline__ void philox_loop2(const RenderArgs& A, const Scene& S, int* stk, int stride, int* side_p,
                                             volatile uint32_t* wq) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lanes_below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const bool joint = !(A.flags & RT_FLAG_REFERENCE_CULL);

  long long w = -1;  // the current chunk's slot in A.partial
  bool done = false, walking = false, ready = false;
  // (worlds walked in the reference's order) the stream position at the start of the walk: a walk
  // redone for an exact tie repeats its media draws
  uint32_t walk_mark = 0;
  // wq[0..1]: the wave's claimed, not yet handed out work-items [next, end), in LDS (lanes that
  // are walking skip the acquisition code, so a per-lane copy would go stale); indices are < 2^32
  // (launch_philox checks)
  if (lane == 0) {
    wq[0] = 0u;
    wq[1] = 0u;
  }
  int px = 0, row = 0, s = 0, s_end = 0, depth = 0;
  V3 thr = v3(0, 0, 0), sum = v3(0, 0, 0);
  RngPhilox g;
  g.init(A.seed, 0, 0);
  Trav t;  // the segment's ray lives only here between segments (no second copy is carried)
  Side side{side_p, stride};
  Cnt cnt{};
  unsigned long long segs = 0, blocks = 0, samples = 0, ph_setup = 0, ph_trav = 0, ph_shade = 0;

  // sample s is over: add its colour; the chunk is done after its last sample
  auto end_sample = [&](V3 contrib) __attribute__((always_inline)) {
    if constexpr ((F & F_COUNT) != 0) {
      blocks += g.pair;
      ++samples;
    }
    if (A.flags & RT_FLAG_NAN_ZERO) contrib = nan_zero(contrib);
    sum = sum + contrib;
    ++s;
    const bool all_nan = (A.flags & RT_FLAG_NAN_CULL) && sum.x != sum.x && sum.y != sum.y && sum.z != sum.z;
    if (s == s_end || all_nan) {
      store_partial(A, w, sum);
      w = -1;
    }
  };

  for (;;) {
    unsigned long long s0 = 0;
    if constexpr ((F & F_COUNT) != 0) {
      s0 = stamp();
      ++cnt.oslot;
    }
    // ---- shade finished walks, then set up the next walk for every lane that is not walking
    if (ready && t.tie && !t.redo) {  // exact tie: redo this walk as the reference does (once)
      ready = false;
      if constexpr ((F & F_COUNT) != 0) ++cnt.ties;
      if constexpr (kRefMixed<F>) g.rewind(walk_mark);  // (the walk's media draws repeat)
      trav_restart_ref(t, S.world_ref, INFINITY, true);
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
      if (shade_hit<F>(S, got, h, ray, thr, depth, g, contrib, cnt)) {
        end_sample(contrib);
      } else if (depth <= 0) {  // rayColor's d <= 0 -> black (thr * 0 keeps a NaN throughput NaN)
        end_sample(vmul(thr, v3(0.0, 0.0, 0.0)));
      } else {  // next segment of the same path
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
            const uint32_t b = rem <= 0 ? 0u : (uint32_t)fminf((float)A.batch, (float)rem * A.batch_per_item);
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
          } else if (work_item(A, (uint32_t)wi, px, row, s, s_end, w)) {
            sum = v3(0, 0, 0);
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
      thr = v3(1.0, 1.0, 1.0);
      depth = A.max_depth;
      if (depth <= 0) {
        end_sample(vmul(thr, v3(0.0, 0.0, 0.0)));
        continue;
      }
      start = true;
      if constexpr ((F & F_COUNT) != 0) ++segs;
    }
    if (start) {
      trav_begin<F>(t, plain(t.ray), S.world, kEps, INFINITY);
      // worlds with media or frames: the reference's order over the re-bounded skeleton
      if (S.ref_walk) trav_restart_ref(t, S.world, INFINITY);
      if constexpr (kRefMixed<F>) walk_mark = g.consumed();
      // (media draw inside the walk: top the FIFO up here, where the starting lanes run together,
      // so that a medium's draw does not evaluate Philox inside a divergent walk step; the words and
      // their order are the stream's, and consumed() is unchanged)
      if constexpr ((F & F_MEDIA) != 0) g.reserve(2);
      walking = true;
    }
    if (!walking) break;  // this lane is finished; the rest of the wave carries on without it
    unsigned long long s1 = 0;
    if constexpr ((F & F_COUNT) != 0) s1 = stamp();
    // ---- walk until few lanes are still walking
    const int live = __popcll(__ballot(true));
    const int stop = (live * A.trav_stop) >> 6;
    const int ls = (F & F_WIDE) ? A.leaf_stop : A.box_first;
    walk_until<F>(S, t, walking, kEps, stk, stride, joint, stop, (live * ls) >> 6, cnt, g, side);
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
  return ((F & F_WIDE) ? RT_WSTACK : RT_STACK) + ((F & F_FRAMES) ? kSideInts : 0);
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
  {
    const uint4* src = (F & F_WIDE) ? reinterpret_cast<const uint4*>(A.S.wnodes)
                                    : reinterpret_cast<const uint4*>(A.S.nodes);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    const int n16 = n_nodes * (rec / 16);
    for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
    // F_WIDE: the leaf table too, when it fits (n_leaves > 0)
    const uint4* lsrc = reinterpret_cast<const uint4*>(A.S.leaves);
    uint4* ldst = reinterpret_cast<uint4*>(lds + (size_t)n_nodes * rec);
    const int l16 = n_leaves * (int)(sizeof(rt_node) / 16);
    for (int i = threadIdx.x; i < l16; i += blockDim.x) ldst[i] = lsrc[i];
  }
  __syncthreads();
  Scene S = A.S;
  if constexpr ((F & F_WIDE) != 0) S.wnodes = reinterpret_cast<const rt_wnode*>(lds);
  else S.nodes = reinterpret_cast<const rt_node*>(lds);
  if constexpr (LEAF_LDS) S.leaves = reinterpret_cast<const rt_node*>(lds + (size_t)n_nodes * rec);
  else n_leaves = 0;
  int* stk = reinterpret_cast<int*>(lds + (size_t)n_nodes * rec + (size_t)n_leaves * sizeof(rt_node)) + threadIdx.x;
  // (the host sizes the dynamic LDS for stack_entries stack ints + kSideInts Side ints per lane
  // when F has F_FRAMES)
  philox_loop2<F>(A, S, stk, WAVES * 256, stk + stack_entries * WAVES * 256,
                  wave_q[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)]);
}

// Tier B: a slab pixel's chunk sums added in chunk order, then averaged and stored (rt.h).
__global__ void __launch_bounds__(256) combine_chunks(RenderArgs A) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= A.slab) return;
  int px, row;
  if (!work_pixel(A, (uint32_t)idx, px, row)) return;  // outside the image: never assembled
  V3 acc = v3(0, 0, 0);
  for (int k = 0; k < A.chunks; ++k) {
    const double* q = A.partial + ((long long)k * A.slab + idx) * 3;
    acc = acc + v3(q[0], q[1], q[2]);
  }
  store_pixel(A, idx, divide(acc, (double)A.spp));
}

// ---------------------------------------------------------------- tier A: the reference's stream
// One lane per image column; rows top to bottom; each pixel draws its 2*ns UVs first and uses
// them in reverse draw order (uniformRandomUVs' foldr, Lib.hs:1358-1371) — the UV pairs are
// recomputed from the pixel's starting state (SplitMix is seed + k*gamma), no list is stored.
template <unsigned F>
__global__ void __launch_bounds__(RT_BLOCK) render_exact(RenderArgs A) {
  __shared__ int stk_mem[RT_STACK * RT_BLOCK];
  int* stk = &stk_mem[threadIdx.x];
  // Tier A reproduces the reference's stream exactly, exact ties included: walk the caller's tree.
  Scene S = A.S;
  S.world = S.world_ref;
  const int x = blockIdx.x * RT_BLOCK + threadIdx.x;
  if (x >= A.W) return;
  RngExact g{A.gens[2 * x], A.gens[2 * x + 1]};
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
      while (!segment<F>(A, S, ray, thr, depth, g, stk, contrib, cnt)) {
      }
      sum = sum + contrib;
    }
    store_pixel(A, (long long)row * A.W + x, divide(sum, (double)ns));
  }
  A.gens[2 * x] = g.seed;
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
  __shared__ int stk_mem[lane_ints<F>() * RT_BLOCK];
  int* stk = &stk_mem[threadIdx.x];
  Side side{&stk_mem[((F & F_WIDE) ? RT_WSTACK : RT_STACK) * RT_BLOCK + threadIdx.x], RT_BLOCK};
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
    bool walking = true;
    walk_until<F>(S, t, walking, tmin, stk, RT_BLOCK, joint != 0, 0, 0, cnt, g, side);
    if (t.tie) {
      if (S.ref_walk) g.rewind(0);  // media draws repeat on the caller's tree
      trav_restart_ref(t, S.world_ref, tmax, true);
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
constexpr int kProbeIn[5] = {18, 3, 6, 6, 2}, kProbeOut[5] = {14, 4, 2, 3, 8};
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
    if (m.type == RT_MAT_DIFFUSE_LIGHT) {
      const V3 e = h.ff ? v3(0, 0, 0) : texture_value<F>(S, m.tex, h.u, h.v, h.p);
      o[8] = e.x, o[9] = e.y, o[10] = e.z;
    } else {
      Scatter sc;
      scatter<F>(S, m, r, h, g, sc);
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
    default: r = tan(a); break;
  }
  out[i] = r;
}

}  // namespace

// =================================================================== host side
struct rt_ctx {
  int device = 0;
  int cu_count = 0;
  int blocks_per_cu = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // Recorded after every tier-B launch: the next launch (on any stream) waits on it before it
  // resets the shared work counter and reuses the chunk-sum buffer.
  hipEvent_t ev_done = nullptr;
  hipStream_t last_stream = nullptr;  // the stream of the last tier-B launch (ev_done's)
  // device scene
  rt_node* d_nodes = nullptr;
  DMat* d_mats = nullptr;
  rt_texture* d_texs = nullptr;
  rt_perlin* d_perlins = nullptr;
  rt_image* d_images = nullptr;
  uint8_t* d_pool = nullptr;
  Scene scene{};
  unsigned features = 0;
  int n_nodes = 0;
  int stack_need = 0;  // deepest traversal stack the world tree needs (entries)
  rt_wnode* d_wnodes = nullptr;  // 4-wide world tree (replace_ok worlds with a BVH root)
  rt_node* d_leaves = nullptr;   // its leaf table (Scene::leaves)
  int n_leaves = 0;
  int n_wnodes = 0;
  int wide_stack_need = 0;
  bool rebuilt_bvh = false;
  bool replace_ok = false;  // frames nest <= RT_MAX_FRAMES deep: the replacement loop applies
  bool has_scene = false;
  unsigned long long* d_counter = nullptr;
  double* d_partial = nullptr;  // tier-B chunk sums (grown on demand)
  size_t partial_bytes = 0;
  double last_ms = 0.0;
  rt_launch_info last_launch{};  // rt_last_launch
};

namespace {

int hip_fail(hipError_t e, const char* what) {
  rt::set_error(std::string(what) + ": " + hipGetErrorString(e));
  return RT_E_HIP;
}
#define HIPCHK(x)                                  \
  do {                                             \
    hipError_t _e = (x);                           \
    if (_e != hipSuccess) return hip_fail(_e, #x); \
  } while (0)

// Device allocation released when it goes out of scope (every return path of the blocking calls).
struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

// Selects a ctx's device for the duration of a C-ABI call and restores the caller's current device
// on every return path (a process driving several GPUs from one thread keeps its own selection).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define DEVICE_SCOPE(dev)                                  \
  DeviceGuard _dg(dev);                                    \
  if (_dg.err != hipSuccess) return hip_fail(_dg.err, "hipSetDevice")

int invalid(const std::string& s) {
  rt::set_error(s);
  return RT_E_INVALID;
}
int unsupported(const std::string& s) {
  rt::set_error(s);
  return RT_E_UNSUPPORTED;
}

void free_scene(rt_ctx* c) {
  (void)hipFree(c->d_nodes);
  (void)hipFree(c->d_mats);
  (void)hipFree(c->d_texs);
  (void)hipFree(c->d_perlins);
  (void)hipFree(c->d_images);
  (void)hipFree(c->d_pool);
  (void)hipFree(c->d_wnodes);
  (void)hipFree(c->d_leaves);
  c->d_wnodes = nullptr;
  c->d_leaves = nullptr;
  c->n_leaves = 0;
  c->n_wnodes = 0;
  c->d_nodes = nullptr;
  c->d_mats = nullptr;
  c->d_texs = nullptr;
  c->d_perlins = nullptr;
  c->d_images = nullptr;
  c->d_pool = nullptr;
  c->has_scene = false;
}

bool is_leaf_prim(int type) {
  return type == RT_NODE_SPHERE || type == RT_NODE_MOVING_SPHERE || type == RT_NODE_CUBOID ||
         (type >= RT_NODE_RECT_XY && type <= RT_NODE_RECT_YZ);
}

struct Validator {
  const rt_scene_desc* d;
  std::vector<rt_node> nodes;  // device copy (type flags added)
  std::vector<int> stack_need, chain_prim, frame_depth;  // frame_depth: nesting of instance frames
  std::string err;

  bool child_ok(int parent, int child) { return child >= 0 && child < parent; }

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
          break;
        case RT_NODE_UNHITTABLE:
        case RT_NODE_EXT:
          break;
        default:
          return fail("unknown node type");
      }
    }
    if (d->world_root < 0 || d->world_root >= n) return fail("world root out of range");
    if (stack_need[d->world_root] > RT_STACK - 2) return unsup("scene BVH too deep for the LDS traversal stack");
    if (d->lights_root >= n) return fail("lights root out of range");
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

template <class T>
int upload(T** dst, const T* src, size_t count) {
  if (count == 0 || !src) return RT_OK;
  HIPCHK(hipMalloc((void**)dst, sizeof(T) * count));
  HIPCHK(hipMemcpy(*dst, src, sizeof(T) * count, hipMemcpyHostToDevice));
  return RT_OK;
}

int check_params(const rt_render_params* p) {
  if (!p) return invalid("null params");
  if (p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->max_depth < 0)
    return invalid("width/height/spp must be positive and max_depth >= 0");
  if (p->rng_mode != RT_RNG_EXACT && p->rng_mode != RT_RNG_PHILOX) return invalid("unknown rng_mode");
  const int tile = p->tile ? p->tile : 16;
  if (tile <= 0 || tile % 8 || tile > 256) return invalid("tile must be a multiple of 8 in [8, 256]");
  if (p->shard_count < 0 || (p->shard_count > 0 && (p->shard_rank < 0 || p->shard_rank >= p->shard_count)) ||
      (p->shard_count <= 1 && p->shard_rank != 0))
    return invalid("bad shard_rank/shard_count");
  if ((long long)p->width * p->height >= (1ll << 32)) return invalid("image too large for 32-bit pixel ids");
  return RT_OK;
}

void geometry(const rt_render_params* p, int& tile, int& tiles_x, long long& tiles_total, long long& per_shard,
              long long& slab_pixels) {
  tile = p->tile ? p->tile : 16;
  const int shards = p->shard_count > 0 ? p->shard_count : 1;
  tiles_x = (p->width + tile - 1) / tile;
  const int tiles_y = (p->height + tile - 1) / tile;
  tiles_total = (long long)tiles_x * tiles_y;
  per_shard = (tiles_total + shards - 1) / shards;
  slab_pixels = per_shard * tile * tile;
}

// Dynamic LDS a CU's workgroup may take: 160 KiB less the replacement loop's static per-wave work
// queues (16 waves x 8 B).
constexpr size_t kLdsBudget = 160 * 1024 - 16 * 8;

// Kernel variants: spheres-only (configs 1, 2, 5), Cornell-like (rects, instances, lights), full.
constexpr unsigned kVarSpheres = 0u;
constexpr unsigned kVarCornell = F_RECT | F_INST | F_LIGHTS;
// the full variant without light sampling (lights Unhittable: next_week_final, the textured
// scenes), whose Lambertian scatter needs no lights-tree code
constexpr unsigned kVarFullDark = F_ALL & ~F_LIGHTS;
unsigned variant_for(unsigned f) {
  if ((f & ~kVarSpheres) == 0) return kVarSpheres;
  if ((f & ~kVarCornell) == 0) return kVarCornell;
  return (f & F_LIGHTS) ? F_ALL : kVarFullDark;
}
bool is_full(unsigned var) { return (var & F_FRAMES) != 0; }
// Occupancy target (waves per SIMD) of the render kernel; RTAMD_WAVES overrides (1..4) for A/B
// measurements. The defaults (launch_philox) are measured.
int waves_target(int dflt) {
  const char* e = std::getenv("RTAMD_WAVES");
  const int w = e ? std::atoi(e) : dflt;
  return (w >= 1 && w <= 4) ? w : dflt;
}
// Kernel pointer for (variant, loop, LDS-staged?, waves per SIMD, counting build?); loop 0 = one
// sample per lane walk, 1 = ray replacement over the binary tree, 2 = replacement over the
// 4-wide tree.
template <unsigned V>
const void* pick_w(bool lds, int w, bool leaf_lds = false) {
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
const void* pick(int loop, bool lds, int w, bool count, bool leaf_lds) {
  if (count) {
    if (loop == 2) return (const void*)render_philox2<V | F_WIDE | F_COUNT, 1>;
    return loop ? (const void*)render_philox2<V | F_COUNT, 1> : (const void*)render_philox<V | F_COUNT, 1>;
  }
  if (loop == 2) return pick_w<V | F_WIDE>(lds, w, leaf_lds);
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
    return w >= 3 ? (const void*)render_philox2<V, 3> : (const void*)render_philox2<V, 2>;
  }
  return w >= 2 ? (const void*)render_philox<V, 2> : (const void*)render_philox<V, 1>;
}
const void* philox_kernel(unsigned var, int loop, bool lds, int w, bool count, bool leaf_lds = false) {
  if (var == kVarSpheres) return pick<kVarSpheres>(loop, lds, w, count, leaf_lds);
  if (var == kVarCornell) return pick<kVarCornell>(loop, lds, w, count, leaf_lds);
  if (var == kVarFullDark) return pick_full<kVarFullDark>(loop, lds, w, count);
  return pick_full<F_ALL>(loop, lds, w, count);
}
bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}
const void* exact_variant(unsigned f) {
  switch (variant_for(f)) {
    case kVarSpheres: return (const void*)render_exact<kVarSpheres>;
    case kVarCornell: return (const void*)render_exact<kVarCornell>;
    default: return (const void*)render_exact<F_ALL>;
  }
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

int launch_combine(rt_ctx* c, const RenderArgs& A, hipStream_t st) {
  RenderArgs B = A;
  void* args[] = {&B};
  HIPCHK(hipLaunchKernel((const void*)combine_chunks, dim3((unsigned)((A.slab + 255) / 256)), dim3(256), args, 0,
                         st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev_done, st));
  return RT_OK;
}

int launch_philox(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int rank, int shards, uint8_t* d_rgb,
                  double* d_lin, hipStream_t st, unsigned long long* d_work = nullptr) {
  RenderArgs A{};
  A.S = c->scene;
  A.cam = *cam;
  A.W = p->width;
  A.H = p->height;
  A.spp = p->spp;
  A.max_depth = p->max_depth;
  A.flags = p->flags;
  long long tiles_total, per_shard, slab;
  geometry(p, A.tile, A.tiles_x, tiles_total, per_shard, slab);
  A.tiles_total = (int)tiles_total;
  A.shard_rank = rank;
  A.shard_count = shards;
  A.slab = slab;
  A.chunk = rt_sample_chunk((int64_t)p->width * p->height, p->spp);
  // RTAMD_CHUNK: another chunk size, for timing experiments only (it changes the summation order,
  // so the image no longer follows rt.h's tier-B definition)
  if (const char* ce = std::getenv("RTAMD_CHUNK")) A.chunk = std::max(1, std::min(p->spp, std::atoi(ce)));
  A.chunks = (p->spp + A.chunk - 1) / A.chunk;
  A.work_total = slab * A.chunks;
  // (work-item indices are 32-bit on the device, and wave claims may run up to one batch per wave
  // past the end: keep 2^24 of headroom)
  if (A.work_total >= (1ll << 32) - (1ll << 24))
    return invalid("image too large: more than 2^32 - 2^24 work-items per shard");
  A.div_tp = make_udiv((uint32_t)(A.tile * A.tile));
  A.div_tile = make_udiv((uint32_t)(A.tile * A.tile * A.chunks));
  A.div_tiles_x = make_udiv((uint32_t)A.tiles_x);
  A.div_bpr = make_udiv((uint32_t)(A.tile >> 3));
  A.seed = p->seed;
  A.counter = c->d_counter;
  A.work = d_work;
  A.out_rgb = d_rgb;
  A.out_lin = d_lin;
  // The work counter and the chunk-sum buffer are the ctx's: order this launch after the previous
  // one, whichever stream that was on (on the same stream, stream order already does).
  if (st != c->last_stream) HIPCHK(hipStreamWaitEvent(st, c->ev_done, 0));
  c->last_stream = st;
  {  // chunk sums: [chunk][slab pixel][3] doubles, kept on the ctx and grown on demand
    const size_t need = (size_t)A.chunks * (size_t)slab * 3 * sizeof(double);
    if (need > c->partial_bytes) {
      HIPCHK(hipEventSynchronize(c->ev_done));
      (void)hipFree(c->d_partial);
      c->d_partial = nullptr;
      c->partial_bytes = 0;
      HIPCHK(hipMalloc((void**)&c->d_partial, need));
      c->partial_bytes = need;
    }
    A.partial = c->d_partial;
  }
  HIPCHK(hipMemsetAsync(c->d_counter, 0, sizeof(unsigned long long), st));
  const char* stop_env = std::getenv("RTAMD_TRAV_STOP");
  // refill when at most trav_stop/64 of a wave's live lanes still walk (measured: C2 flat at 2-8,
  // -4 % at 16; the 100k-sphere C5 tree, walks ~3x longer, best at 16)
  // (the full variant's walks over the caller's tree: 16, C4 1496 vs 1567 ms at 200 spp)
  // Work-items a wave claims per atomic: one claim per batch instead of one per acquisition round
  // (RTAMD_BATCH; 1 = the lanes' exact need every time). The batch tapers as the frame runs out: a
  // wave claims at most rem / (16 * waves) items when about `rem` remain, so the waves' unstarted
  // claims together never exceed 1/16 of what is left.
  {
    const char* be = std::getenv("RTAMD_BATCH");
    A.batch = be ? std::max(1, std::min(4096, std::atoi(be))) : 1024;
    const double waves = (double)c->cu_count * 4 * 4;  // at most 4 waves per SIMD
    A.batch_per_item = (float)(1.0 / (16.0 * waves));
  }
  A.trav_stop = stop_env ? std::max(0, std::min(63, std::atoi(stop_env)))
                         : (c->n_nodes > 20000 || is_full(variant_for(c->features)) ? 16 : 8);
  const char* leaf_env = std::getenv("RTAMD_LEAF_STOP");
  // leaf steps once <= that many lanes still seek their first leaf (measured: C2 212.6 ms at 6-8/64
  // vs 219.7 at 0 and 232 without postponement; C5 (16 spp) 219.9 ms at 16/64 vs 326 at 0)
  A.leaf_stop = leaf_env ? std::max(0, std::min(64, std::atoi(leaf_env))) : A.trav_stop;
  // binary walks of the full variant (media / frame worlds, C4): box-only steps while more than
  // box_first/64 of the live lanes are at BVH nodes (measured on C4 at 100 spp: 64 (never) 430 ms,
  // 48 416, 32 406, 16 398, 8 413; C3's Cornell kernel does not take it)
  const char* box_env = std::getenv("RTAMD_BOX_FIRST");
  A.box_first = box_env ? std::max(0, std::min(64, std::atoi(box_env))) : 16;
  const unsigned var = variant_for(c->features);
  const bool count = d_work != nullptr;
  // Replacement loop (RTAMD_REPLACE=0 disables) for every world whose instance frames nest at most
  // RT_MAX_FRAMES deep; worlds with media or frames walk the caller's tree in the reference's order.
  // Over the 4-wide tree when one was built (RTAMD_WIDE=0 disables; the reference-cull flag asks
  // for the binary tree's exact box test).
  const bool replace = c->replace_ok && !env_off("RTAMD_REPLACE");
  // The wide tree pays off on rebuilt (>= 16-leaf) worlds; small worlds keep the binary walk
  // (Cornell: 409 vs 262-399 Msamples/s measured), RTAMD_WIDE=1 forces it.
  const char* wenv = std::getenv("RTAMD_WIDE");
  const bool want_wide = wenv ? wenv[0] != '0' : c->rebuilt_bvh;
  // (the full variant has no 4-wide instantiation: its media-free worlds walk the binary tree)
  const bool wide = replace && c->d_wnodes && !(p->flags & RT_FLAG_REFERENCE_CULL) && want_wide && !is_full(var);
  const int loop = wide ? 2 : (replace ? 1 : 0);
  // waves per SIMD (measured): spheres 4 when the LDS-staged kernel fits at 4 (C2 158.4 ms vs
  // 166.6 at 3, 203.2 at 2), else 3 (C5 186.7 ms vs 228.5 at 4, -15 % at 2); Cornell-like on the
  // replacement loop 3 (C3 359.6 ms vs 374.3 at 4, 453.3 at 2), 1 on the per-sample loop; full
  // variant on the replacement loop 3 (C4 at 100 spp: 90.9 vs 87.5 Msamples/s at 2), on the
  // per-sample loop 2 despite 784 B/lane of scratch (C4 35.2 vs 23.4 at 1 wave, 9.1 at 3)
  int waves = (var == kVarSpheres || loop) ? waves_target(3) : waves_target(is_full(var) ? 2 : 1);
  const int side_ints = (var & F_FRAMES) && loop == 1 ? kSideInts : 0;  // Side slots after the stacks
  // LDS-staged kernel when the traversal's node array plus the stacks fit one CU's 160 KiB
  // (RTAMD_LDS=0 disables it for A/B runs).
  if (!count && !env_off("RTAMD_LDS") && (!is_full(var) || loop)) {
    const int entries = wide ? c->wide_stack_need + 3 : c->stack_need + 2;  // (wide_node writes 3 slots)
    const int items = wide ? c->n_wnodes : c->n_nodes;
    const size_t rec = wide ? sizeof(rt_wnode) : sizeof(rt_node);
    const bool leaf_lds = wide && !env_off("RTAMD_LEAF_LDS");  // RTAMD_LEAF_LDS=0: leaves never in LDS
    // LDS bytes at `w` waves per SIMD: the nodes, the lane stacks, and the wide walk's leaf table
    // when it fits as well
    auto lds_bytes = [&](int w, int& n_leaves) {
      size_t b = (size_t)items * rec + (size_t)(entries + side_ints) * (w * 256) * sizeof(int);
      n_leaves = leaf_lds && b + (size_t)c->n_leaves * sizeof(rt_node) <= kLdsBudget ? c->n_leaves : 0;
      return b + (size_t)n_leaves * sizeof(rt_node);
    };
    int n_leaves = 0;
    // (and only when there is work for the 4th wave: C1's 20 000 items fill less than 3 waves)
    if (var == kVarSpheres && !std::getenv("RTAMD_WAVES") && lds_bytes(4, n_leaves) <= kLdsBudget &&
        (!leaf_lds || n_leaves > 0) && A.work_total >= (long long)c->cu_count * 1024)
      waves = 4;
    const int block = waves * 256;
    const size_t bytes = lds_bytes(waves, n_leaves);
    if (bytes <= kLdsBudget) {
      const void* fn = philox_kernel(var, loop, true, waves, false, n_leaves > 0);
      HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
      int n_items = items;
      void* args[] = {&A, &n_items, (void*)&entries, &n_leaves};
      c->last_launch = rt_launch_info{var | (loop == 2 ? F_WIDE : 0u), loop, 1, n_leaves > 0, waves, c->cu_count,
                                      block, (int)bytes, A.work_total, A.chunk, 0};
      HIPCHK(hipEventRecord(c->ev0, st));
      HIPCHK(hipLaunchKernel(fn, dim3(c->cu_count), dim3(block), args, bytes, st));
      HIPCHK(hipEventRecord(c->ev1, st));
      return launch_combine(c, A, st);
    }
  }
  const void* fn = philox_kernel(var, loop, false, count ? 1 : waves, count);
  // replacement loops: lane stacks (+ Side slots) in dynamic LDS, sized for this world's stack bound
  int entries = wide ? c->wide_stack_need + 3 : c->stack_need + 2;  // (wide_node writes 3 slots)
  const size_t dyn = loop ? (size_t)(entries + side_ints) * RT_BLOCK * sizeof(int) : 0;
  if (loop) HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
  int bpc = 1;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, fn, RT_BLOCK, dyn));
  const long long want = (A.work_total + RT_BLOCK - 1) / RT_BLOCK;
  const long long resident = (long long)c->cu_count * std::max(1, bpc);
  const int grid = (int)std::max(1ll, std::min(want, resident));
  c->last_launch = rt_launch_info{var | (loop == 2 ? F_WIDE : 0u) | (count ? F_COUNT : 0u), loop, 0, 0,
                                  count ? 1 : waves, grid, RT_BLOCK, (int)dyn, A.work_total, A.chunk, 0};
  HIPCHK(hipEventRecord(c->ev0, st));
  void* args[] = {&A, &entries};
  HIPCHK(hipLaunchKernel(fn, dim3(grid), dim3(RT_BLOCK), args, dyn, st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev1, st));
  return launch_combine(c, A, st);
}

}  // namespace

extern "C" {

int rt_device_count(int* out) {
  if (!out) return invalid("null out");
  HIPCHK(hipGetDeviceCount(out));
  return RT_OK;
}

int rt_create(int device, rt_ctx** out) {
  if (!out) return invalid("null out");
  *out = nullptr;
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return invalid("device index out of range");
  DEVICE_SCOPE(device);
  rt_ctx* c = new rt_ctx();
  c->device = device;
  auto init = [c]() -> int {
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, c->device));
    c->cu_count = prop.multiProcessorCount;
    int bpc = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void*)render_philox<F_ALL, 1>, RT_BLOCK, 0));
    c->blocks_per_cu = bpc;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev0));
    HIPCHK(hipEventCreate(&c->ev1));
    HIPCHK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
    HIPCHK(hipMalloc((void**)&c->d_counter, 256));
    return RT_OK;
  };
  const int rc = init();
  if (rc) {
    rt_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

void rt_destroy(rt_ctx* c) {
  if (!c) return;
  DeviceGuard _dg(c->device);
  free_scene(c);
  (void)hipFree(c->d_counter);
  (void)hipFree(c->d_partial);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int rt_upload_scene(rt_ctx* c, const rt_scene_desc* d) { return rt_upload_scene_ex(c, d, 0u); }

int rt_upload_scene_ex(rt_ctx* c, const rt_scene_desc* din, uint32_t flags) {
  if (!c || !din) return invalid("null argument");
  if (din->n_nodes <= 0 || !din->nodes || din->world_root < 0 || din->world_root >= din->n_nodes)
    return invalid("rt_upload_scene: bad node array or world root");
  DEVICE_SCOPE(c->device);
  // World-tree rebuild (rt_bvh.cpp) unless the caller or RTAMD_REFERENCE_BVH=1 asks for the
  // reference's own makeBVH tree; never for trees holding media.
  std::vector<rt_node> nodes(din->nodes, din->nodes + din->n_nodes);
  rt_scene_desc dd = *din;
  const char* env = std::getenv("RTAMD_REFERENCE_BVH");
  const bool keep = (flags & RT_UPLOAD_REFERENCE_BVH) || (env && env[0] == '1');
  if (!keep) {
    // validate the original first so the rebuild only ever sees well-formed DAGs
    Validator v0{din};
    if (!v0.run()) {
      rt::set_error("rt_upload_scene: " + v0.err);
      return v0.code;
    }
    // Worlds without media or instance frames: a whole new tree over the same leaves (exact ties are
    // redone on the caller's tree). Worlds walked in the reference's order (media draws, frames):
    // the skeleton above the media stays, the media-free subtrees below it (and the trees inside
    // frames) are re-bounded; RTAMD_SKELETON=0 keeps the caller's tree as is.
    dd.world_root = rt::rebuild_for_device(nodes, din->world_root);
  }
  if ((int)nodes.size() >= RT_SUB) return invalid("rt_upload_scene: too many nodes (ids must stay below 2^29)");
  dd.nodes = nodes.data();
  dd.n_nodes = (int)nodes.size();
  const rt_scene_desc* d = &dd;
  Validator v{d};
  if (!v.run()) {
    rt::set_error("rt_upload_scene: " + v.err);
    return v.code;
  }
  for (int i = 0; i < d->n_textures; ++i) {
    const rt_texture& t = d->textures[i];
    if (t.type == RT_TEX_CHECKER && (t.a < 0 || t.a >= i || t.b < 0 || t.b >= i))
      return invalid("rt_upload_scene: checker children must precede the checker");
    if (t.type == RT_TEX_PERLIN && (t.a < 0 || t.a >= d->n_perlins)) return invalid("rt_upload_scene: bad perlin id");
    if (t.type == RT_TEX_IMAGE && t.a >= 0) {
      if (t.a >= d->n_images) return invalid("rt_upload_scene: bad image id");
      const rt_image& im = d->images[t.a];
      if (im.width != t.b || im.height != t.c || im.offset < 0 ||
          im.offset + (int64_t)im.width * im.height * 3 > d->image_pool_bytes)
        return invalid("rt_upload_scene: image raster out of the pool");
    }
  }
  std::vector<DMat> mats(d->n_materials);
  for (int i = 0; i < d->n_materials; ++i) {
    const rt_material& m = d->materials[i];
    if (m.type < RT_MAT_LAMBERTIAN || m.type > RT_MAT_ISOTROPIC) return invalid("rt_upload_scene: bad material");
    if (m.type != RT_MAT_DIELECTRIC && (m.texture < 0 || m.texture >= d->n_textures))
      return invalid("rt_upload_scene: material texture out of range");
    mats[i] = DMat{m.type, m.texture, m.param, m.type != RT_MAT_DIELECTRIC && tex_needs_uv(d, m.texture), 0};
  }
  if (d->image_pool_bytes < 0 || (d->image_pool_bytes > 0 && !d->image_pool))
    return invalid("rt_upload_scene: image_pool is null but image_pool_bytes > 0");
  free_scene(c);
  c->rebuilt_bvh = dd.world_root != din->world_root;
  int rc;
  if ((rc = upload(&c->d_nodes, v.nodes.data(), v.nodes.size())) ||
      (rc = upload(&c->d_mats, mats.data(), mats.size())) ||
      (rc = upload(&c->d_texs, d->textures, (size_t)d->n_textures)) ||
      (rc = upload(&c->d_perlins, d->perlins, (size_t)d->n_perlins)) ||
      (rc = upload(&c->d_images, d->images, (size_t)d->n_images)) ||
      (rc = upload(&c->d_pool, d->image_pool, (size_t)d->image_pool_bytes))) {
    free_scene(c);
    return rc;
  }
  Scene& S = c->scene;
  S.nodes = c->d_nodes;
  S.mats = c->d_mats;
  S.texs = c->d_texs;
  S.perlins = c->d_perlins;
  S.images = c->d_images;
  S.pool = c->d_pool;
  S.world = d->world_root;
  S.world_ref = din->world_root;
  S.lights = d->lights_root;
  for (int i = 0; i < 3; ++i) S.bg[i] = d->background[i];
  c->features = scene_features(d);
  c->n_nodes = d->n_nodes;
  // (tie redo walks the caller's tree: size the stacks for both)
  c->stack_need = std::max(v.stack_need[d->world_root], v.stack_need[din->world_root]);
  // The replacement loop takes every world whose frames nest at most RT_MAX_FRAMES deep (its Side
  // slots); worlds with media or frames walk the caller's tree in the reference's order.
  const bool frames = v.frame_depth[d->world_root] > 0;
  c->replace_ok = v.frame_depth[d->world_root] <= RT_MAX_FRAMES;
  S.ref_walk = (c->features & F_MEDIA) || frames;
  if (frames) c->features |= F_FRAMES;
  if (c->replace_ok && !S.ref_walk) {  // 4-wide fp32-box tree over the same world tree (unflagged node copy)
    std::vector<rt_wnode> wide;
    int need = 0;
    if (rt::build_wide_bvh(nodes, d->world_root, wide, &need) && need + 3 <= RT_WSTACK &&
        (size_t)wide.size() < (size_t)INT32_MAX / 2) {
      // The walk's leaf table: the leaves the wide tree references, each copied once (a moving
      // sphere with its EXT record), with `c` = the flat node id; leaf references ~id become ~slot.
      std::vector<rt_node> leaves;
      std::vector<int> slot(v.nodes.size(), -1);
      for (rt_wnode& w : wide)
        for (int k = 0; k < RT_WIDE; ++k) {
          if (w.child[k] >= 0) continue;
          const int id = ~w.child[k];
          if (slot[id] < 0) {
            slot[id] = (int)leaves.size();
            leaves.push_back(v.nodes[id]);
            leaves.back().c = id;
            if ((v.nodes[id].type & RT_TYPE_MASK) == RT_NODE_MOVING_SPHERE) leaves.push_back(v.nodes[id + 1]);
          }
          w.child[k] = ~slot[id];
        }
      if ((rc = upload(&c->d_wnodes, wide.data(), wide.size())) ||
          (rc = upload(&c->d_leaves, leaves.data(), leaves.size()))) {
        free_scene(c);
        return rc;
      }
      c->n_leaves = (int)leaves.size();
      S.leaves = c->d_leaves;
      c->n_wnodes = (int)wide.size();
      c->wide_stack_need = std::max(need, v.stack_need[din->world_root]);
      S.wnodes = c->d_wnodes;
    }
  }
  if (!c->d_wnodes) S.wnodes = nullptr, S.leaves = nullptr;
  c->has_scene = true;
  return RT_OK;
}

int rt_shard_geometry(const rt_render_params* p, int64_t* tiles_total, int64_t* tiles_per_shard,
                      int64_t* slab_pixels) {
  int rc = check_params(p);
  if (rc) return rc;
  int tile, tiles_x;
  long long tt, ps, sp;
  geometry(p, tile, tiles_x, tt, ps, sp);
  if (tiles_total) *tiles_total = tt;
  if (tiles_per_shard) *tiles_per_shard = ps;
  if (slab_pixels) *slab_pixels = sp;
  return RT_OK;
}

int rt_render_shard_async(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, uint8_t* d_rgb, double* d_lin,
                          void* stream) {
  if (!c || !cam || !d_rgb) return invalid("null argument");
  int rc = check_params(p);
  if (rc) return rc;
  if (!c->has_scene) {
    rt::set_error("rt_render_shard_async: no scene uploaded");
    return RT_E_STATE;
  }
  if (p->rng_mode != RT_RNG_PHILOX) return invalid("sharded rendering needs RT_RNG_PHILOX (tier B)");
  DEVICE_SCOPE(c->device);
  const int shards = p->shard_count > 0 ? p->shard_count : 1;
  return launch_philox(c, cam, p, p->shard_rank, shards, d_rgb, d_lin, (hipStream_t)stream);
}

int rt_assemble_async(rt_ctx* c, const rt_render_params* p, const uint8_t* d_slabs, uint8_t* d_image, void* stream) {
  if (!c || !d_slabs || !d_image) return invalid("null argument");
  int rc = check_params(p);
  if (rc) return rc;
  int tile, tiles_x;
  long long tt, ps, sp;
  geometry(p, tile, tiles_x, tt, ps, sp);
  const long long n = (long long)p->width * p->height;
  DEVICE_SCOPE(c->device);  // (the caller's current device may be another ctx's)
  hipLaunchKernelGGL(assemble<uint8_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_slabs,
                     d_image, p->width, p->height, tile, tiles_x, p->shard_count > 0 ? p->shard_count : 1, sp);
  HIPCHK(hipGetLastError());
  return RT_OK;
}

int rt_assemble_linear_async(rt_ctx* c, const rt_render_params* p, const double* d_slabs, double* d_image,
                             void* stream) {
  if (!c || !d_slabs || !d_image) return invalid("null argument");
  int rc = check_params(p);
  if (rc) return rc;
  int tile, tiles_x;
  long long tt, ps, sp;
  geometry(p, tile, tiles_x, tt, ps, sp);
  const long long n = (long long)p->width * p->height;
  DEVICE_SCOPE(c->device);
  hipLaunchKernelGGL(assemble<double>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_slabs,
                     d_image, p->width, p->height, tile, tiles_x, p->shard_count > 0 ? p->shard_count : 1, sp);
  HIPCHK(hipGetLastError());
  return RT_OK;
}

int rt_render(rt_ctx* c, const rt_camera* cam, const rt_render_params* pin, const uint64_t* col_gens, uint8_t* out_rgb,
              double* out_lin, uint64_t* out_gens) {
  if (!c || !cam || !pin || !out_rgb) return invalid("null argument");
  rt_render_params p = *pin;  // whole image: the shard fields are ignored
  p.shard_rank = 0;
  p.shard_count = 1;
  int rc = check_params(&p);
  if (rc) return rc;
  if (!c->has_scene) {
    rt::set_error("rt_render: no scene uploaded");
    return RT_E_STATE;
  }
  if (p.rng_mode == RT_RNG_EXACT && !col_gens) return invalid("rt_render: tier A needs col_gens (2*width words)");
  DEVICE_SCOPE(c->device);
  const long long npx = (long long)p.width * p.height;
  hipStream_t st = c->stream;
  DevBuf img, img_lin, slab_buf, slab_lin, gens;  // freed on every return path
  HIPCHK(hipMalloc(&img.p, (size_t)npx * 3));
  if (out_lin) HIPCHK(hipMalloc(&img_lin.p, sizeof(double) * (size_t)npx * 3));
  uint8_t* d_img = (uint8_t*)img.p;
  double* d_img_lin = (double*)img_lin.p;
  if (p.rng_mode == RT_RNG_PHILOX) {
    int tile, tiles_x;
    long long tt, ps, slab;
    geometry(&p, tile, tiles_x, tt, ps, slab);
    HIPCHK(hipMalloc(&slab_buf.p, (size_t)slab * 3));
    if (out_lin) HIPCHK(hipMalloc(&slab_lin.p, sizeof(double) * (size_t)slab * 3));
    rc = launch_philox(c, cam, &p, 0, 1, (uint8_t*)slab_buf.p, (double*)slab_lin.p, st);
    if (!rc) rc = rt_assemble_async(c, &p, (const uint8_t*)slab_buf.p, d_img, st);
    if (!rc && out_lin) rc = rt_assemble_linear_async(c, &p, (const double*)slab_lin.p, d_img_lin, st);
    HIPCHK(hipStreamSynchronize(st));
    if (rc) return rc;
  } else {
    HIPCHK(hipMalloc(&gens.p, sizeof(uint64_t) * 2 * (size_t)p.width));
    uint64_t* d_gens = (uint64_t*)gens.p;
    HIPCHK(hipMemcpyAsync(d_gens, col_gens, sizeof(uint64_t) * 2 * (size_t)p.width, hipMemcpyHostToDevice, st));
    RenderArgs A{};
    A.S = c->scene;
    A.cam = *cam;
    A.W = p.width;
    A.H = p.height;
    A.spp = p.spp;
    A.max_depth = p.max_depth;
    A.gens = d_gens;
    A.out_rgb = d_img;
    A.out_lin = d_img_lin;
    HIPCHK(hipEventRecord(c->ev0, st));
    void* args[] = {&A};
    HIPCHK(hipLaunchKernel(exact_variant(c->features), dim3((p.width + RT_BLOCK - 1) / RT_BLOCK), dim3(RT_BLOCK),
                           args, 0, st));
    HIPCHK(hipEventRecord(c->ev1, st));
    if (out_gens)
      HIPCHK(hipMemcpyAsync(out_gens, d_gens, sizeof(uint64_t) * 2 * (size_t)p.width, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  HIPCHK(hipMemcpy(out_rgb, d_img, (size_t)npx * 3, hipMemcpyDeviceToHost));
  if (out_lin) HIPCHK(hipMemcpy(out_lin, d_img_lin, sizeof(double) * (size_t)npx * 3, hipMemcpyDeviceToHost));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->last_ms = ms;
  return RT_OK;
}

int rt_render_work(rt_ctx* c, const rt_camera* cam, const rt_render_params* pin, uint64_t out_work[16]) {
  if (!c || !cam || !pin || !out_work) return invalid("null argument");
  int rc = check_params(pin);
  if (rc) return rc;
  if (!c->has_scene) {
    rt::set_error("rt_render_work: no scene uploaded");
    return RT_E_STATE;
  }
  if (pin->rng_mode != RT_RNG_PHILOX) return invalid("rt_render_work: tier B only");
  DEVICE_SCOPE(c->device);
  rt_render_params p = *pin;
  const int shards = p.shard_count > 0 ? p.shard_count : 1;
  int tile, tiles_x;
  long long tt, ps, slab;
  geometry(&p, tile, tiles_x, tt, ps, slab);
  DevBuf slab_buf, work;
  HIPCHK(hipMalloc(&slab_buf.p, (size_t)slab * 3));
  HIPCHK(hipMalloc(&work.p, sizeof(unsigned long long) * 16));
  unsigned long long* d_work = (unsigned long long*)work.p;
  HIPCHK(hipMemsetAsync(d_work, 0, sizeof(unsigned long long) * 16, c->stream));
  rc = launch_philox(c, cam, &p, p.shard_rank, shards, (uint8_t*)slab_buf.p, nullptr, c->stream, d_work);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (rc) return rc;
  unsigned long long w[16];
  HIPCHK(hipMemcpy(w, d_work, sizeof w, hipMemcpyDeviceToHost));
  for (int i = 0; i < 16; ++i) out_work[i] = w[i];
  return RT_OK;
}

int rt_last_kernel_ms(rt_ctx* c, double* out_ms) {
  if (!c || !out_ms) return invalid("null argument");
  float ms = 0;
  HIPCHK(hipEventSynchronize(c->ev1));
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->last_ms = ms;
  *out_ms = ms;
  return RT_OK;
}

int rt_last_launch(rt_ctx* c, rt_launch_info* out) {
  if (!c || !out) return invalid("null argument");
  *out = c->last_launch;
  return RT_OK;
}

int rt_debug_closest_hits(rt_ctx* c, const double* rays, int n, double tmin, double tmax, uint64_t seed,
                          uint32_t flags, double* out) {
  if (!c || !rays || !out || n < 0) return invalid("null argument");
  if (!c->has_scene) {
    rt::set_error("rt_debug_closest_hits: no scene uploaded");
    return RT_E_STATE;
  }
  if ((flags & (RT_DEBUG_RESUMABLE | RT_DEBUG_WIDE)) && !c->replace_ok)
    return unsupported("rt_debug_closest_hits: the resumable walks need a world without media and frames");
  if ((flags & RT_DEBUG_WIDE) && !c->d_wnodes)
    return unsupported("rt_debug_closest_hits: no 4-wide tree for this world");
  if (n == 0) return RT_OK;
  DEVICE_SCOPE(c->device);
  DevBuf rays_buf, out_buf;
  HIPCHK(hipMalloc(&rays_buf.p, sizeof(double) * 7 * (size_t)n));
  HIPCHK(hipMalloc(&out_buf.p, sizeof(double) * 12 * (size_t)n));
  double* d_rays = (double*)rays_buf.p;
  double* d_out = (double*)out_buf.p;
  HIPCHK(hipMemcpy(d_rays, rays, sizeof(double) * 7 * (size_t)n, hipMemcpyHostToDevice));
  const int joint = !(flags & RT_FLAG_REFERENCE_CULL);
  const dim3 grid((n + RT_BLOCK - 1) / RT_BLOCK);
  if (flags & RT_DEBUG_WIDE)
    hipLaunchKernelGGL(closest_hits<F_ALL | F_UV | F_WIDE>, grid, dim3(RT_BLOCK), 0, c->stream, c->scene, d_rays, n,
                       tmin, tmax, seed, joint, 1, d_out);
  else
    hipLaunchKernelGGL(closest_hits<F_ALL | F_UV>, grid, dim3(RT_BLOCK), 0, c->stream, c->scene, d_rays, n, tmin,
                       tmax, seed, joint, (flags & RT_DEBUG_RESUMABLE) ? 1 : 0, d_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, d_out, sizeof(double) * 12 * (size_t)n, hipMemcpyDeviceToHost));
  return RT_OK;
}

int rt_debug_probe(rt_ctx* c, const rt_camera* cam, int op, const double* in, int n, uint64_t seed, double* out) {
  if (!c || !in || !out || n < 0 || op < 0 || op > 4 || (op == 4 && !cam)) return invalid("rt_debug_probe: bad argument");
  if (!c->has_scene) {
    rt::set_error("rt_debug_probe: no scene uploaded");
    return RT_E_STATE;
  }
  if (n == 0) return RT_OK;
  DEVICE_SCOPE(c->device);
  DevBuf bin, bout;
  const size_t nin = sizeof(double) * kProbeIn[op] * (size_t)n, nout = sizeof(double) * kProbeOut[op] * (size_t)n;
  HIPCHK(hipMalloc(&bin.p, nin));
  HIPCHK(hipMalloc(&bout.p, nout));
  HIPCHK(hipMemcpy(bin.p, in, nin, hipMemcpyHostToDevice));
  rt_camera k{};
  if (cam) k = *cam;
  hipLaunchKernelGGL(fn_probe<F_ALL>, dim3((n + RT_BLOCK - 1) / RT_BLOCK), dim3(RT_BLOCK), 0, c->stream, c->scene, k, op,
                     (const double*)bin.p, n, seed, (double*)bout.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, bout.p, nout, hipMemcpyDeviceToHost));
  return RT_OK;
}

int rt_debug_math(rt_ctx* c, int op, const double* x, const double* y, int n, double* out) {
  if (!c || !x || !y || !out || n < 0 || op < 0 || op > 11) return invalid("rt_debug_math: bad argument");
  if (n == 0) return RT_OK;
  DEVICE_SCOPE(c->device);
  const size_t bytes = sizeof(double) * (size_t)n;
  DevBuf bx, by, bout;
  HIPCHK(hipMalloc(&bx.p, bytes));
  HIPCHK(hipMalloc(&by.p, bytes));
  HIPCHK(hipMalloc(&bout.p, bytes));
  double *dx = (double*)bx.p, *dy = (double*)by.p, *dout = (double*)bout.p;
  HIPCHK(hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy, y, bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(math_probe, dim3((n + 255) / 256), dim3(256), 0, c->stream, op, dx, dy, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
  return RT_OK;
}

}  // extern "C"
