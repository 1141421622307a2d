// rt_render.hip — the device half of the C ABI (include/rt.h): scene upload, launches, assembly,
// debug probes. The render kernels are templates in rt_kernels.h, instantiated per scene variant in
// rt_k_spheres.hip / rt_k_cornell.hip / rt_k_full.hip / rt_k_full_dark.hip.
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
//  * tier B (Philox per (pixel, sample)) shards by tiles with no data-path collective before the
//    final framebuffer gather; tier A (the reference's per-column SplitMix stream) runs one lane per
//    column;
//  * a multi-device ctx (rt_create_multi) renders one tile shard per GPU from one host thread and
//    gathers the RGB8 slabs to its first device with RCCL (grouped ncclGather), which assembles.
#include <rccl/rccl.h>

#include <numeric>
#include <vector>

#include "rt_kernels.h"
#include "rt_prepare.h"


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
  int n_materials = 0, n_textures = 0;  // (rt_debug_probe checks record ids against them)
  int stack_need = 0;  // deepest traversal stack the world tree needs (entries)
  rt_wnode* d_wnodes = nullptr;  // 4-wide world tree (replace_ok worlds with a BVH root)
  rt_node* d_leaves = nullptr;   // its leaf table (Scene::leaves)
  rt_qnode* d_qnodes = nullptr;  // spheres-only worlds: the 4-wide tree quantised (Scene::qnodes)
  double* d_sleaves = nullptr;   // and the leaf table's spheres (Scene::sleaves)
  int n_leaves = 0;
  int n_wnodes = 0;
  int wide_stack_need = 0;
  bool w8 = false;           // the 4-wide arrays hold the 8-wide tree as record pairs (F_W8 kernels, A/B)
  bool rebuilt_bvh = false;
  bool far_boxes = false;    // a BVH box coordinate beyond 2^100: the walks take the per-axis box test (cull())
  bool mixed_wide = false;   // media / frame world with 4-wide trees over its re-bounded subtrees (F_MIXW)
  bool replace_ok = false;  // frames nest <= RT_MAX_FRAMES deep: the replacement loop applies
  bool has_scene = false;
  unsigned long long* d_counter = nullptr;
  double* d_partial = nullptr;  // tier-B chunk sums (grown on demand, at most kPartialCap)
  size_t partial_bytes = 0;
  double* d_tail = nullptr;     // tier-B tail units' sample colours (RenderArgs::tail_buf), grown on demand
  size_t tail_bytes = 0;
  double* d_acc = nullptr;      // running per-pixel sums of a frame rendered in chunk batches
  size_t acc_bytes = 0;
  double last_ms = 0.0;
  rt_launch_info last_launch{};  // rt_last_launch
  // rt_render's frame events: after the render launches (gather start), after the gather, after assembly
  hipEvent_t ev_gather = nullptr, ev_gathered = nullptr, ev_asm = nullptr;
  rt_frame_timing last_frame{};  // rt_last_frame_timing
  // Multi-device ctx (rt_create_multi): this ctx is the first device's (RCCL rank 0, the gather root);
  // peers[r - 1] is device r's, comms[r] its communicator (ncclCommInitAll, ranks in list order).
  std::vector<rt_ctx*> peers;
  std::vector<ncclComm_t> comms;
  // rt_render's own device buffers, kept between calls and grown on demand (every rt_render returns after
  // its stream is drained, so the next call may reuse them): the slab (RGB8, fp64) this device renders
  // into, and on a multi-device ctx's first device the gathered slabs and the assembled image; tier A's
  // column generators. Repeated frames of one size allocate nothing.
  struct FrameBuf {
    void* p = nullptr;
    size_t bytes = 0;
  };
  FrameBuf fb_slab, fb_slab_lin, fb_gather, fb_gather_lin, fb_img, fb_img_lin, fb_gens;
  int allocs = 0;  // hipMalloc calls made on this device by the current rt_render (rt_frame_timing)
};

namespace {

int hip_fail(hipError_t e, const char* what) {
  rt::set_error(std::string(what) + ": " + hipGetErrorString(e));
  return RT_E_HIP;
}
int hip_ok(hipError_t e, const char* what) { return e == hipSuccess ? RT_OK : hip_fail(e, what); }
#define HIPCHK(x)                                  \
  do {                                             \
    hipError_t _e = (x);                           \
    if (_e != hipSuccess) return hip_fail(_e, #x); \
  } while (0)

int nccl_fail(ncclResult_t r, const char* what) {
  rt::set_error(std::string(what) + ": " + ncclGetErrorString(r));
  return RT_E_COMM;
}
#define NCCLCHK(x)                                    \
  do {                                                \
    ncclResult_t _r = (x);                            \
    if (_r != ncclSuccess) return nccl_fail(_r, #x);  \
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

// A frame buffer of the ctx with at least `need` bytes on the current device (the caller selects the
// ctx's device): reused as is when large enough, else freed and allocated again (counted in c->allocs).
int grow(rt_ctx* c, rt_ctx::FrameBuf& b, size_t need) {
  if (need <= b.bytes) return RT_OK;
  (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  ++c->allocs;
  HIPCHK(hipMalloc(&b.p, need));
  b.bytes = need;
  return RT_OK;
}
void free_frame_bufs(rt_ctx* c) {
  for (rt_ctx::FrameBuf* b : {&c->fb_slab, &c->fb_slab_lin, &c->fb_gather, &c->fb_gather_lin, &c->fb_img,
                              &c->fb_img_lin, &c->fb_gens}) {
    (void)hipFree(b->p);
    b->p = nullptr;
    b->bytes = 0;
  }
}

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
  (void)hipFree(c->d_qnodes);
  (void)hipFree(c->d_sleaves);
  c->d_wnodes = nullptr;
  c->d_leaves = nullptr;
  c->d_qnodes = nullptr;
  c->d_sleaves = nullptr;
  c->mixed_wide = false;
  c->w8 = false;
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

template <class T>
int upload(T** dst, const T* src, size_t count) {
  if (count == 0 || !src) return RT_OK;
  HIPCHK(hipMalloc((void**)dst, sizeof(T) * count));
  HIPCHK(hipMemcpy(*dst, src, sizeof(T) * count, hipMemcpyHostToDevice));
  return RT_OK;
}

// Tile edge when the caller leaves it 0 (round 5: 8, was 16; work order and shard dealing only, the
// image does not depend on it: C2 136.0-136.2 -> 135.5 ms, its 8-shard probe 19.1 -> 18.9 ms slowest
// shard, C3 320.0 -> 318.7, C4 at 100 spp 153.3 -> 148.6, C5 at 64 spp 653.0 -> 651.8)
constexpr int kDefaultTile = 8;
int check_params(const rt_render_params* p) {
  if (!p) return invalid("null params");
  if (p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->max_depth < 0)
    return invalid("width/height/spp must be positive and max_depth >= 0");
  if (p->rng_mode != RT_RNG_EXACT && p->rng_mode != RT_RNG_PHILOX) return invalid("unknown rng_mode");
  if ((p->flags & RT_FLAG_SHARED_LIBM) && p->rng_mode != RT_RNG_EXACT)
    return invalid("RT_FLAG_SHARED_LIBM is a tier-A (RT_RNG_EXACT) flag");
  const int tile = p->tile ? p->tile : kDefaultTile;
  if (tile <= 0 || tile % 8 || tile > 256) return invalid("tile must be a multiple of 8 in [8, 256]");
  if (p->shard_count < 0 || (p->shard_count > 0 && (p->shard_rank < 0 || p->shard_rank >= p->shard_count)) ||
      (p->shard_count <= 1 && p->shard_rank != 0))
    return invalid("bad shard_rank/shard_count");
  if ((long long)p->width * p->height >= (1ll << 32)) return invalid("image too large for 32-bit pixel ids");
  return RT_OK;
}

void geometry(const rt_render_params* p, int& tile, int& tiles_x, long long& tiles_total, long long& per_shard,
              long long& slab_pixels) {
  tile = p->tile ? p->tile : kDefaultTile;
  const int shards = p->shard_count > 0 ? p->shard_count : 1;
  tiles_x = (p->width + tile - 1) / tile;
  const int tiles_y = (p->height + tile - 1) / tile;
  tiles_total = (long long)tiles_x * tiles_y;
  per_shard = (tiles_total + shards - 1) / shards;
  slab_pixels = per_shard * tile * tile;
}

// Most bytes of chunk sums one launch writes (2 GiB; C5 at 2000 spp: 24.9 GB of chunk sums in 13 batches)
constexpr size_t kPartialCap = 2ull << 30;

// Dynamic LDS a CU's workgroup may take: 160 KiB less the replacement loop's static per-wave work
// queues (16 waves x 8 B).
constexpr size_t kLdsBudget = 160 * 1024 - 16 * 8;

// Occupancy target (waves per SIMD) of the render kernel; RTAMD_WAVES overrides (1..4) for A/B
// measurements. The defaults (launch_philox) are measured.
int waves_target(int dflt) {
  const char* e = std::getenv("RTAMD_WAVES");
  const int w = e ? std::atoi(e) : dflt;
  return (w >= 1 && w <= 4) ? w : dflt;
}
// (the render kernels live in one translation unit per variant: rt_k_*.hip)
const void* philox_kernel(unsigned var, int loop, bool lds, int w, bool count, bool leaf_lds = false, bool q = false,
                          bool w8 = false) {
  if (var == kVarSpheres) {
    // (the 4-wide tree from global memory, 128-byte nodes: its own unit, rt_k_spheres_global.hip)
    if (loop == 2 && !lds && !count && !q && !w8 && !std::getenv("RTAMD_NO_COLD")) return rt::philox_kernel_spheres_global(w);
    return rt::philox_kernel_spheres(loop, lds, w, count, leaf_lds, q, w8);
  }
  if (var == kVarCornell) return rt::philox_kernel_cornell(loop, lds, w, count, leaf_lds);
  if (var == kVarFullDark) return rt::philox_kernel_full_dark(loop, lds, w, count);
  return rt::philox_kernel_full(loop, lds, w, count);
}
bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}
template <bool LDS>
const void* exact_variant_l(unsigned f, bool shared_libm) {
  switch (variant_for(f)) {
    case kVarSpheres:
      return shared_libm ? (const void*)render_exact<kVarSpheres | F_SLIBM, LDS> : (const void*)render_exact<kVarSpheres, LDS>;
    case kVarCornell:
      return shared_libm ? (const void*)render_exact<kVarCornell | F_SLIBM, LDS> : (const void*)render_exact<kVarCornell, LDS>;
    default: return shared_libm ? (const void*)render_exact<F_ALL | F_SLIBM, LDS> : (const void*)render_exact<F_ALL, LDS>;
  }
}
// Blocks of the tier-A kernel: kExactColsPerWave columns per wave, RT_BLOCK / 64 waves per block.
unsigned exact_blocks(int width) {
  const int per_block = (RT_BLOCK / 64) * kExactColsPerWave;
  return (unsigned)((width + per_block - 1) / per_block);
}
// The tier-A kernel for the ctx's scene and its dynamic LDS bytes: the node array staged in LDS when it
// fits beside the static lane stacks (RTAMD_EXACT_LDS=0: never).
int exact_launch(rt_ctx* c, bool shared_libm, const void** fn, size_t* bytes) {
  const size_t need = (size_t)c->n_nodes * sizeof(rt_node);
  const size_t budget = 160 * 1024 - (size_t)RT_STACK * RT_BLOCK * sizeof(int);
  const char* e = std::getenv("RTAMD_EXACT_LDS");
  if (need <= budget && !(e && e[0] == '0')) {
    *fn = exact_variant_l<true>(c->features, shared_libm);
    *bytes = need;
    HIPCHK(hipFuncSetAttribute(*fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need));
  } else {
    *fn = exact_variant_l<false>(c->features, shared_libm);
    *bytes = 0;
  }
  return RT_OK;
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

// The launch's culling flags: the caller's, with the per-axis test alone for far-box worlds (rt_ctx::far_boxes).
uint32_t cull(const rt_ctx* c, uint32_t flags) { return flags | (c->far_boxes ? RT_FLAG_REFERENCE_CULL : 0u); }

int launch_philox(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int rank, int shards, uint8_t* d_rgb,
                  double* d_lin, hipStream_t st, unsigned long long* d_work = nullptr,
                  unsigned long long* d_prof = nullptr) {
  RenderArgs A{};
  A.S = c->scene;
  A.cam = *cam;
  A.W = p->width;
  A.H = p->height;
  A.spp = p->spp;
  A.max_depth = p->max_depth;
  A.flags = cull(c, p->flags);
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
  A.work_total = slab * A.chunks;  // (the whole frame's; each chunk batch's launch sets its own)
  A.items_total = A.work_total;
  A.tail_start = A.work_total;
  A.div_tp = make_udiv((uint32_t)(A.tile * A.tile));
  A.div_tiles_x = make_udiv((uint32_t)A.tiles_x);
  A.div_bpr = make_udiv((uint32_t)(A.tile >> 3));
  A.seed = p->seed;
  A.counter = c->d_counter;
  A.work = d_work;
  A.prof = d_prof;
  A.out_rgb = d_rgb;
  A.out_lin = d_lin;
  // The work counter and the chunk-sum buffer are the ctx's: order this launch after the previous
  // one, whichever stream that was on (on the same stream, stream order already does).
  if (st != c->last_stream) HIPCHK(hipStreamWaitEvent(st, c->ev_done, 0));
  c->last_stream = st;
  // Chunk sums: [chunk][slab pixel][3] doubles, kept on the ctx and grown on demand, at most
  // kPartialCap bytes (RTAMD_PARTIAL_CAP overrides, for tests): a frame with more chunks renders them
  // in batches of consecutive chunks, one launch each, and combine_chunks folds each batch into a
  // running per-pixel sum in chunk order — the sum rt.h defines, whatever the batching.
  const int chunks_total = A.chunks;
  const size_t per_chunk = (size_t)slab * 3 * sizeof(double);
  size_t cap = kPartialCap;
  if (const char* pc = std::getenv("RTAMD_PARTIAL_CAP")) cap = (size_t)std::max(1ll, std::atoll(pc));
  const int per_batch = (int)std::max<size_t>(1, std::min<size_t>((size_t)chunks_total, cap / per_chunk));
  const int batches = (chunks_total + per_batch - 1) / per_batch;
  {
    const size_t need = (size_t)per_batch * per_chunk;
    const size_t need_acc = batches > 1 ? per_chunk : 0;
    if (need > c->partial_bytes || need_acc > c->acc_bytes) {
      HIPCHK(hipEventSynchronize(c->ev_done));
      if (need > c->partial_bytes) {
        (void)hipFree(c->d_partial);
        c->d_partial = nullptr;
        c->partial_bytes = 0;
        ++c->allocs;
        HIPCHK(hipMalloc((void**)&c->d_partial, need));
        c->partial_bytes = need;
      }
      if (need_acc > c->acc_bytes) {
        (void)hipFree(c->d_acc);
        c->d_acc = nullptr;
        c->acc_bytes = 0;
        ++c->allocs;
        HIPCHK(hipMalloc((void**)&c->d_acc, need_acc));
        c->acc_bytes = need_acc;
      }
    }
    A.partial = c->d_partial;
    A.acc = c->d_acc;
  }
  // The frame's tail (the full variants' replacement loop, kTail in rt_kernels.h; set below with the
  // loop): the last `tail_items` work-items of each launch are dealt one sample per unit, their colours
  // summed in sample order afterwards (tail_combine): the sums rt.h defines, whatever the dealing.
  // RTAMD_TAIL: tail items per CU (default 768, one per lane of 12 waves; 0: no tail).
  long long tail_items = 0;
  A.div_chunk = make_udiv((uint32_t)A.chunk);
  auto units_of = [&](long long items) { return items + std::min(items, tail_items) * (A.chunk - 1); };
  // one launch per chunk batch (stream-ordered; the events span all of them)
  auto run = [&](const void* fn, dim3 grid, dim3 block, size_t bytes, void** args) -> int {
    // (work-unit indices are 32-bit on the device, and wave claims may run up to one batch per wave
    // past the end: keep 2^24 of headroom)
    if (units_of(slab * per_batch) >= (1ll << 32) - (1ll << 24))
      return invalid("image too large: more than 2^32 - 2^24 work units per shard and launch");
    const size_t need_tail = (size_t)std::min(slab * per_batch, tail_items) * (size_t)A.chunk * 3 * sizeof(double);
    if (need_tail > c->tail_bytes) {
      HIPCHK(hipEventSynchronize(c->ev_done));
      (void)hipFree(c->d_tail);
      c->d_tail = nullptr;
      c->tail_bytes = 0;
      ++c->allocs;
      HIPCHK(hipMalloc((void**)&c->d_tail, need_tail));
      c->tail_bytes = need_tail;
    }
    A.tail_buf = c->d_tail;
    for (int k0 = 0; k0 < chunks_total; k0 += per_batch) {
      const int nk = std::min(per_batch, chunks_total - k0);
      A.chunk_base = k0;
      A.chunks = nk;
      A.items_total = slab * nk;
      A.tail_start = A.items_total - std::min(A.items_total, tail_items);
      A.work_total = units_of(A.items_total);
      A.div_tile = make_udiv((uint32_t)(A.tile * A.tile * nk));
      A.combine = (k0 > 0 ? 1 : 0) | (k0 + nk == chunks_total ? 2 : 0);
      HIPCHK(hipMemsetAsync(c->d_counter, 0, sizeof(unsigned long long), st));
      if (k0 == 0) HIPCHK(hipEventRecord(c->ev0, st));
      HIPCHK(hipLaunchKernel(fn, grid, block, args, bytes, st));  // (arguments are copied at launch)
      HIPCHK(hipGetLastError());
      if (A.tail_start < A.items_total) {
        RenderArgs B = A;
        void* targs[] = {&B};
        HIPCHK(hipLaunchKernel((const void*)tail_combine, dim3((unsigned)((A.items_total - A.tail_start + 255) / 256)),
                               dim3(256), targs, 0, st));
        HIPCHK(hipGetLastError());
      }
      if (A.combine & 2) HIPCHK(hipEventRecord(c->ev1, st));
      const int rc = launch_combine(c, A, st);
      if (rc) return rc;
    }
    return RT_OK;
  };
  const char* stop_env = std::getenv("RTAMD_TRAV_STOP");
  // refill when at most trav_stop/64 of a wave's live lanes still walk (measured: C2 flat at 2-8,
  // -4 % at 16; the 100k-sphere C5 tree, walks ~3x longer, best at 16)
  // (the full variant's walks over the caller's tree: 16 in round 2, C4 1496 vs 1567 ms at 200 spp; with
  // the mixed walk (round 3) 8: C4 at 100 spp 323.7 vs 326.0 ms, 24: 334.0)
  // Work-items a wave claims per atomic: one claim per batch instead of one per acquisition round
  // (RTAMD_BATCH; 1 = the lanes' exact need every time). The batch tapers as the frame runs out: a
  // wave claims at most rem / (16 * waves) items when about `rem` remain, so the waves' unstarted
  // claims together never exceed 1/16 of what is left.
  {
    const char* be = std::getenv("RTAMD_BATCH");
    A.batch = be ? std::max(1, std::min(4096, std::atoi(be))) : 1024;
    const double waves = (double)c->cu_count * 4 * 4;  // at most 4 waves per SIMD
    A.batch_per_item = (float)(1.0 / (16.0 * waves));
    // ... but never below one item per lane of the claiming wave (RTAMD_BATCH_FLOOR): near the end of
    // a frame the taper otherwise shrinks claims to the lanes' exact need, one contended atomic per
    // few items; 64 items are consumed by the wave's lanes in parallel, so they hoard nothing (C2
    // per shard at N = 8: 21.05 -> 19.95 ms, 0.83 -> 0.88 of ideal; N = 1 140.7 -> 139.3 ms; 256:
    // 21.2 ms, 512: 26 ms). Not for the full variant, whose items are long and uneven (C4 at 100
    // spp with 128: 286 -> 293 ms): 0 there.
    const char* bf = std::getenv("RTAMD_BATCH_FLOOR");
    A.batch_floor = bf ? std::max(0, std::min(1024, std::atoi(bf))) : (is_full(variant_for(c->features)) ? 0 : 64);
  }
  A.trav_stop = stop_env ? std::max(0, std::min(63, std::atoi(stop_env)))
                         : (c->n_nodes > 20000 ? 16 : 8);
  const char* leaf_env = std::getenv("RTAMD_LEAF_STOP");
  // leaf steps once <= that many lanes still seek their first leaf (measured: C2 212.6 ms at 6-8/64
  // vs 219.7 at 0 and 232 without postponement; C5 (16 spp) 219.9 ms at 16/64 vs 326 at 0)
  A.leaf_stop = leaf_env ? std::max(0, std::min(64, std::atoi(leaf_env))) : A.trav_stop;
  // binary walks of the full variant (media / frame worlds, C4): box-only steps while more than
  // box_first/64 of the live lanes are at BVH nodes (4-wide nodes count; measured on C4 at 100 spp, round
  // 2: 64 (never) 430 ms, 48 416, 32 406, 16 398, 8 413; round 5, hoisted media and one 4-wide tree, with
  // trav_stop 8: 0 189.6, 2 178.6, 4 174.6, 8 176.3, 16 182.3, 32 185.3; C3's Cornell kernel does not
  // take it)
  const char* box_env = std::getenv("RTAMD_BOX_FIRST");
  A.box_first = box_env ? std::max(0, std::min(64, std::atoi(box_env))) : 4;
  const char* med_env = std::getenv("RTAMD_MED_BATCH");
  // lanes at a medium wait for med_batch of them (round 4, C4 at 100 spp: 0 249.0 ms, 4 245.3, 8 245.9,
  // 16 295). Since round 5 a world's own media are hoisted (RT_BVH_MEDIA_FIRST, taken where walks start):
  // only media inside instance frames still wait here, none in C4 (0 174.6 ms vs 4 176.3): off by default
  A.med_batch = med_env ? std::max(0, std::min(64, std::atoi(med_env))) : 0;
  // work order only (the chunk sums do not depend on it): the slab's tiles last to first
  A.rev_tiles = env_off("RTAMD_TILE_REV") || !std::getenv("RTAMD_TILE_REV") ? 0u : (uint32_t)per_shard;
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
  const bool wide = replace && c->d_wnodes && !(A.flags & RT_FLAG_REFERENCE_CULL) && want_wide && !is_full(var);
  const int loop = wide ? 2 : (replace ? 1 : 0);
  if (loop && is_full(var)) {  // (kTail kernels; the per-sample loop claims whole work-items)
    const char* te = std::getenv("RTAMD_TAIL");
    tail_items = (long long)c->cu_count * (te ? std::max(0, std::min(1 << 16, std::atoi(te))) : 768);
  }
  // waves per SIMD (measured): spheres 4 when the LDS-staged kernel fits at 4 (C2 158.4 ms vs
  // 166.6 at 3, 203.2 at 2), else 3 (C5 186.7 ms vs 228.5 at 4, -15 % at 2); Cornell-like on the
  // replacement loop 3 (C3 359.6 ms vs 374.3 at 4, 453.3 at 2), 1 on the per-sample loop; full
  // variant on the replacement loop 3 (C4 at 100 spp: 90.9 vs 87.5 Msamples/s at 2), on the
  // per-sample loop 2 despite 784 B/lane of scratch (C4 35.2 vs 23.4 at 1 wave, 9.1 at 3)
  int waves = (var == kVarSpheres || loop) ? waves_target(3) : waves_target(is_full(var) ? 2 : 1);
  // the mixed walk's leaf postponement (kMixPostpone, rt_trace.h) keeps a lane's next node on the stack
  // while its parked leaf is tested (or its frame opened): one stack entry more
  const int postpone = (loop == 1 && (var & F_MIXW) && RT_MIXW_POSTPONE) ? 1 : 0;
  // Side slots after the stacks, then the 4 lane ints philox_loop2 keeps in LDS (RT_LANE_LDS)
  const int side_ints = side_ints_of(var, c->scene.frames, loop) + (lane_lds_of(var, loop) ? 4 : 0);
  // LDS-staged kernel when the traversal's node array plus the stacks fit one CU's 160 KiB
  // (RTAMD_LDS=0 disables it for A/B runs).
  if (!count && !env_off("RTAMD_LDS") && (!is_full(var) || loop) && !(wide && c->w8)) {  // (F_W8: global only)
    const int entries = wide ? c->wide_stack_need + 3 + (RT_LEAF_Q ? 1 : 0) : c->stack_need + 2 + postpone;  // (wide_node writes 3 slots; + the leaf queue word)
    const int items = wide ? c->n_wnodes : c->n_nodes;
    const size_t rec = wide ? sizeof(rt_wnode) : sizeof(rt_node);
    const bool leaf_lds = wide && !env_off("RTAMD_LEAF_LDS");  // RTAMD_LEAF_LDS=0: leaves never in LDS
    // The compact form of a spheres-only world's 4-wide kernel (F_SLEAF, rt_kernels.h render_philox2_lds):
    // 32-byte sphere leaves, 16-bit lane stacks (ids below 2^15), the lanes' throughput and chunk sums in
    // LDS. Opt-in (RTAMD_COMPACT=1): measured slower on C2
    const char* ce = std::getenv("RTAMD_COMPACT");
    const bool compact = var == kVarSpheres && wide && leaf_lds && waves >= 3 && c->d_sleaves && c->n_nodes < 32768 &&
                         c->n_wnodes < 32768 && c->n_leaves <= 32768 && ce && ce[0] == '1';
    constexpr size_t kStateBytes = kStateLdsBytes;
    constexpr size_t kStackBytes = RT_COMPACT_STACK16 ? sizeof(short) : sizeof(int);
    constexpr size_t kLeafBytes = RT_COMPACT_SLEAF ? 32 : sizeof(rt_node);
    // LDS bytes at `w` waves per SIMD: the nodes, the lane stacks, and the wide walk's leaf table
    // when it fits as well
    auto lds_bytes = [&](int w, int& n_leaves) {
      if (compact) {
        const size_t b = (size_t)items * rec + ((size_t)entries * kStackBytes + (size_t)side_ints * sizeof(int) +
                                                kStateBytes) * (w * 256);
        n_leaves = c->n_leaves;
        return b + (size_t)n_leaves * kLeafBytes;
      }
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
      const void* fn = philox_kernel(var, loop, true, waves, false, n_leaves > 0, compact);
      HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
      int n_items = items;
      void* args[] = {&A, &n_items, (void*)&entries, &n_leaves};
      c->last_launch = rt_launch_info{var | (loop == 2 ? F_WIDE : 0u), loop, 1, n_leaves > 0, waves, c->cu_count,
                                      block, (int)bytes, A.work_total, A.chunk,
                                      (loop == 2 || (loop == 1 && c->mixed_wide)) ? c->n_wnodes : 0, batches, 0};
      return run(fn, dim3(c->cu_count), dim3(block), bytes, args);
    }
  }
  // (spheres-only worlds uploaded with RTAMD_QNODE=1 read the 4-wide tree from global memory in its
  // 64-byte quantised form: A/B only, measured slower)
  const void* fn = philox_kernel(var, loop, false, count ? 1 : waves, count, false, loop == 2 && c->d_qnodes,
                                 loop == 2 && c->w8);
  // replacement loops: lane stacks (+ Side slots) in dynamic LDS, sized for this world's stack bound
  // (wide_node writes 3 slots, F_W8's farther half 4; + the leaf queue word)
  int entries = wide ? c->wide_stack_need + (c->w8 ? 4 : 3) + (RT_LEAF_Q ? 1 : 0) : c->stack_need + 2 + postpone;
  const size_t dyn = loop ? (size_t)(entries + side_ints) * RT_BLOCK * sizeof(int) : 0;
  if (loop) HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
  int bpc = 1;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, fn, RT_BLOCK, dyn));
  const long long want = (A.work_total + RT_BLOCK - 1) / RT_BLOCK;
  const long long resident = (long long)c->cu_count * std::max(1, bpc);
  const int grid = (int)std::max(1ll, std::min(want, resident));
  c->last_launch = rt_launch_info{var | (loop == 2 ? F_WIDE : 0u) | (count ? F_COUNT : 0u) | (loop == 2 && c->w8 ? F_W8 : 0u), loop, 0, 0,
                                  count ? 1 : waves, grid, RT_BLOCK, (int)dyn, A.work_total, A.chunk,
                                  (loop == 2 || (loop == 1 && c->mixed_wide)) ? c->n_wnodes : 0, batches, 0};
  void* args[] = {&A, &entries};
  return run(fn, dim3(grid), dim3(RT_BLOCK), dyn, args);
}

// rt_render, tier B, on a multi-device ctx (rt_create_multi): shard r of N = the ctx's r-th device. Every
// device renders its tiles into a slab on its own stream (the launches are queued from this thread and
// run concurrently); the slabs are gathered to device 0 by RCCL (one ncclGather per communicator, grouped,
// each on its device's stream after that device's render), which assembles the image.
// Not in place: device 0 renders into its own slab too, so the gather moves bytes even at N = 1.
int render_multi(rt_ctx* c, const rt_camera* cam, rt_render_params p, uint8_t* out_rgb, double* out_lin) {
  const int n = 1 + (int)c->peers.size();
  p.shard_count = n;
  int tile, tiles_x;
  long long tt, ps, slab;
  geometry(&p, tile, tiles_x, tt, ps, slab);
  auto dev_ctx = [&](int r) { return r == 0 ? c : c->peers[r - 1]; };
  const long long npx = (long long)p.width * p.height;
  // the send slabs on every device, the gathered slabs and the image on device 0: the ctx's frame buffers,
  // grown on demand (rt_ctx::FrameBuf), so that repeated frames allocate nothing
  int rc = RT_OK;
  for (int r = 0; r < n && !rc; ++r) {
    rt_ctx* d = dev_ctx(r);
    DEVICE_SCOPE(d->device);
    if ((rc = grow(d, d->fb_slab, (size_t)slab * 3))) break;
    if (out_lin && (rc = grow(d, d->fb_slab_lin, sizeof(double) * (size_t)slab * 3))) break;
  }
  {
    DEVICE_SCOPE(c->device);
    if (!rc) rc = grow(c, c->fb_gather, (size_t)n * slab * 3);
    if (!rc && out_lin) rc = grow(c, c->fb_gather_lin, sizeof(double) * (size_t)n * slab * 3);
    if (!rc) rc = grow(c, c->fb_img, (size_t)npx * 3);
    if (!rc && out_lin) rc = grow(c, c->fb_img_lin, sizeof(double) * (size_t)npx * 3);
  }
  if (rc) return rc;
  void* gathered = c->fb_gather.p;
  void* gathered_lin = c->fb_gather_lin.p;
  void* img = c->fb_img.p;
  void* img_lin = c->fb_img_lin.p;
  // the shards' renders, one per device, queued back to back
  for (int r = 0; r < n; ++r) {
    rt_ctx* d = dev_ctx(r);
    DEVICE_SCOPE(d->device);
    rt_render_params pr = p;
    pr.shard_rank = r;
    if ((rc = launch_philox(d, cam, &pr, r, n, (uint8_t*)d->fb_slab.p, out_lin ? (double*)d->fb_slab_lin.p : nullptr,
                            d->stream)))
      return rc;
    if (r == 0) HIPCHK(hipEventRecord(c->ev_gather, c->stream));
  }
  // the RCCL gather of the slabs to device 0 (rank 0), in the ranks' stream order after their renders
  {
    DeviceGuard _dg(c->device);
    NCCLCHK(ncclGroupStart());
    for (int r = 0; r < n; ++r) {
      rt_ctx* d = dev_ctx(r);
      const ncclResult_t g = ncclGather(d->fb_slab.p, r == 0 ? gathered : nullptr, (size_t)slab * 3, ncclUint8, 0,
                                        c->comms[r], d->stream);
      const ncclResult_t gl = g == ncclSuccess && out_lin
                                  ? ncclGather(d->fb_slab_lin.p, r == 0 ? gathered_lin : nullptr, (size_t)slab * 3,
                                               ncclFloat64, 0, c->comms[r], d->stream)
                                  : g;
      if (gl != ncclSuccess) {
        (void)ncclGroupEnd();
        return nccl_fail(gl, "ncclGather");
      }
    }
    NCCLCHK(ncclGroupEnd());
  }
  {
    DEVICE_SCOPE(c->device);
    HIPCHK(hipEventRecord(c->ev_gathered, c->stream));
    if ((rc = rt_assemble_async(c, &p, (const uint8_t*)gathered, (uint8_t*)img, c->stream))) return rc;
    if (out_lin && (rc = rt_assemble_linear_async(c, &p, (const double*)gathered_lin, (double*)img_lin, c->stream)))
      return rc;
    HIPCHK(hipEventRecord(c->ev_asm, c->stream));
  }
  for (int r = 0; r < n; ++r) {  // (the peers' streams too: the next frame reuses their slabs)
    rt_ctx* d = dev_ctx(r);
    DEVICE_SCOPE(d->device);
    HIPCHK(hipStreamSynchronize(d->stream));
  }
  DEVICE_SCOPE(c->device);
  HIPCHK(hipMemcpy(out_rgb, img, (size_t)npx * 3, hipMemcpyDeviceToHost));
  if (out_lin) HIPCHK(hipMemcpy(out_lin, img_lin, sizeof(double) * (size_t)npx * 3, hipMemcpyDeviceToHost));
  rt_frame_timing ft{};
  ft.n_devices = n;
  for (int r = 0; r < n; ++r) ft.device_allocs += dev_ctx(r)->allocs;
  float ms = 0;
  for (int r = 0; r < n; ++r) {
    rt_ctx* d = dev_ctx(r);
    HIPCHK(hipEventElapsedTime(&ms, d->ev0, d->ev1));
    d->last_ms = ms;
    ft.kernel_ms[r] = ms;
  }
  HIPCHK(hipEventElapsedTime(&ms, c->ev_gather, c->ev_gathered));
  ft.gather_ms = ms;
  HIPCHK(hipEventElapsedTime(&ms, c->ev_gathered, c->ev_asm));
  ft.assemble_ms = ms;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev_asm));
  ft.frame_ms = ms;
  c->last_frame = ft;
  return RT_OK;
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
    HIPCHK(hipEventCreate(&c->ev_gather));
    HIPCHK(hipEventCreate(&c->ev_gathered));
    HIPCHK(hipEventCreate(&c->ev_asm));
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

int rt_create_multi(int n, const int* devices, rt_ctx** out) {
  if (!out) return invalid("null out");
  *out = nullptr;
  if (n < 1 || n > RT_MAX_DEVICES) return invalid("n_devices must be in [1, RT_MAX_DEVICES]");
  int avail = 0;
  HIPCHK(hipGetDeviceCount(&avail));
  std::vector<int> list(n);
  if (devices) std::copy(devices, devices + n, list.begin());
  else std::iota(list.begin(), list.end(), 0);
  for (int i = 0; i < n; ++i) {
    if (list[i] < 0 || list[i] >= avail) return invalid("device index out of range");
    for (int j = 0; j < i; ++j)
      if (list[j] == list[i]) return invalid("device listed twice (one RCCL rank per GPU)");
  }
  rt_ctx* c = nullptr;
  int rc = rt_create(list[0], &c);
  if (rc) return rc;
  for (int i = 1; i < n && !rc; ++i) {
    rt_ctx* p = nullptr;
    rc = rt_create(list[i], &p);
    if (!rc) c->peers.push_back(p);
  }
  if (!rc) {
    DeviceGuard _dg(list[0]);  // (ncclCommInitAll selects each device in turn; the caller's is restored)
    c->comms.assign(n, nullptr);
    const ncclResult_t r = ncclCommInitAll(c->comms.data(), n, list.data());
    if (r != ncclSuccess) {
      c->comms.clear();
      rc = nccl_fail(r, "ncclCommInitAll");
    }
  }
  if (rc) {
    rt_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

int rt_ctx_devices(const rt_ctx* c, int* out_n, int* out_devices, int cap) {
  if (!c || !out_n || cap < 0) return invalid("null argument");
  *out_n = 1 + (int)c->peers.size();
  for (int r = 0; out_devices && r < *out_n && r < cap; ++r)
    out_devices[r] = r == 0 ? c->device : c->peers[r - 1]->device;
  return RT_OK;
}

int rt_last_frame_timing(rt_ctx* c, rt_frame_timing* out) {
  if (!c || !out) return invalid("null argument");
  *out = c->last_frame;
  return RT_OK;
}

void rt_destroy(rt_ctx* c) {
  if (!c) return;
  for (size_t r = 0; r < c->comms.size(); ++r) {
    if (!c->comms[r]) continue;
    DeviceGuard _dr(r == 0 ? c->device : c->peers[r - 1]->device);
    (void)ncclCommDestroy(c->comms[r]);
  }
  c->comms.clear();
  for (rt_ctx* p : c->peers) rt_destroy(p);
  c->peers.clear();
  DeviceGuard _dg(c->device);
  free_scene(c);
  free_frame_bufs(c);
  (void)hipFree(c->d_counter);
  (void)hipFree(c->d_partial);
  (void)hipFree(c->d_tail);
  (void)hipFree(c->d_acc);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  if (c->ev_gather) (void)hipEventDestroy(c->ev_gather);
  if (c->ev_gathered) (void)hipEventDestroy(c->ev_gathered);
  if (c->ev_asm) (void)hipEventDestroy(c->ev_asm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}


int rt_upload_scene(rt_ctx* c, const rt_scene_desc* d) { return rt_upload_scene_ex(c, d, 0u); }

}  // extern "C"

namespace {
// Copies a prepared scene to c's device (replacing its scene).
int upload_prepared(rt_ctx* c, const rt::PreparedScene& P, const rt_scene_desc* din) {
  int rc = RT_OK;
  DEVICE_SCOPE(c->device);
  free_scene(c);
  if ((rc = upload(&c->d_nodes, P.nodes.data(), P.nodes.size())) ||
      (rc = upload(&c->d_mats, P.mats.data(), P.mats.size())) ||
      (rc = upload(&c->d_texs, din->textures, (size_t)din->n_textures)) ||
      (rc = upload(&c->d_perlins, din->perlins, (size_t)din->n_perlins)) ||
      (rc = upload(&c->d_images, din->images, (size_t)din->n_images)) ||
      (rc = upload(&c->d_pool, din->image_pool, (size_t)din->image_pool_bytes)) ||
      (rc = upload(&c->d_wnodes, P.wnodes.data(), P.wnodes.size())) ||
      (rc = upload(&c->d_leaves, P.leaves.data(), P.leaves.size())) ||
      (rc = upload(&c->d_qnodes, P.qnodes.data(), P.qnodes.size())) ||
      (rc = upload(&c->d_sleaves, P.sleaves.data(), P.sleaves.size()))) {
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
  S.wnodes = c->d_wnodes;
  S.leaves = c->d_leaves;
  S.qnodes = c->d_qnodes;
  S.sleaves = c->d_sleaves;
  S.world = P.world;
  S.world_ref = P.world_ref;
  S.lights = P.lights;
  S.ref_walk = P.ref_walk;
  S.frames = std::max(1, std::min(RT_MAX_FRAMES, P.frame_depth));
  for (int i = 0; i < 3; ++i) S.bg[i] = din->background[i];
  c->features = P.features;
  c->n_nodes = (int)P.nodes.size();
  c->n_materials = din->n_materials;
  c->n_textures = din->n_textures;
  c->n_wnodes = (int)P.wnodes.size();
  c->n_leaves = (int)P.leaves.size();
  c->stack_need = P.stack_need;
  c->wide_stack_need = P.wide_stack_need;
  c->w8 = P.w8;
  c->rebuilt_bvh = P.rebuilt_bvh;
  // The division-free box test (rt_trace.h box_hit) reads an infinite slab product as the quotient; with
  // |origin| <= 2^100 (ray_safe) and |d| >= 2^-900 that holds while every finite box coordinate is within
  // 2^100 (no finite quotient overflows as a product). Worlds beyond it are walked with the reference's
  // per-axis test alone (RT_FLAG_REFERENCE_CULL), which divides.
  c->far_boxes = false;
  for (const rt_node& x : P.nodes)
    if ((x.type & RT_TYPE_MASK) == RT_NODE_BVH)
      for (int k = 0; k < 6; ++k) c->far_boxes |= std::isfinite(x.f[k]) && std::fabs(x.f[k]) > 0x1p100;
  c->mixed_wide = P.mixed_wide;
  c->replace_ok = P.replace_ok;
  c->has_scene = true;
  return RT_OK;
}
}  // namespace

extern "C" {

int rt_upload_scene_ex(rt_ctx* c, const rt_scene_desc* din, uint32_t flags) {
  if (!c || !din) return invalid("null argument");
  // the host half (rt_prepare.cpp): validation, the walk's trees, the tagged device copy — once, then
  // the copy goes to every device of the ctx (a malformed descriptor leaves every device's scene as it was)
  rt::PreparedScene P;
  int rc = rt::prepare_scene(din, flags, P);
  if (rc) return rc;
  rc = upload_prepared(c, P, din);
  for (size_t r = 0; r < c->peers.size() && !rc; ++r) rc = upload_prepared(c->peers[r], P, din);
  if (rc) {  // (a device failed: no device keeps a scene, so a multi-device render cannot mix two)
    for (rt_ctx* p : c->peers) {
      DeviceGuard _dg(p->device);
      free_scene(p);
    }
    DeviceGuard _dg(c->device);
    free_scene(c);
  }
  return rc;
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
  for (rt_ctx* q : c->peers)
    if (!q->has_scene) {
      rt::set_error("rt_render: no scene uploaded on every device");
      return RT_E_STATE;
    }
  c->allocs = 0;
  for (rt_ctx* q : c->peers) q->allocs = 0;
  if (p.rng_mode == RT_RNG_PHILOX && !c->comms.empty()) return render_multi(c, cam, p, out_rgb, out_lin);
  DEVICE_SCOPE(c->device);
  const long long npx = (long long)p.width * p.height;
  hipStream_t st = c->stream;
  // (the ctx's frame buffers, grown on demand: repeated frames allocate nothing)
  if ((rc = grow(c, c->fb_img, (size_t)npx * 3))) return rc;
  if (out_lin && (rc = grow(c, c->fb_img_lin, sizeof(double) * (size_t)npx * 3))) return rc;
  uint8_t* d_img = (uint8_t*)c->fb_img.p;
  double* d_img_lin = out_lin ? (double*)c->fb_img_lin.p : nullptr;
  rt_frame_timing ft{};
  ft.n_devices = 1;
  if (p.rng_mode == RT_RNG_PHILOX) {
    int tile, tiles_x;
    long long tt, ps, slab;
    geometry(&p, tile, tiles_x, tt, ps, slab);
    if ((rc = grow(c, c->fb_slab, (size_t)slab * 3))) return rc;
    if (out_lin && (rc = grow(c, c->fb_slab_lin, sizeof(double) * (size_t)slab * 3))) return rc;
    const uint8_t* slab_rgb = (const uint8_t*)c->fb_slab.p;
    const double* slab_lin = out_lin ? (const double*)c->fb_slab_lin.p : nullptr;
    rc = launch_philox(c, cam, &p, 0, 1, (uint8_t*)slab_rgb, (double*)slab_lin, st);
    if (!rc) rc = hip_ok(hipEventRecord(c->ev_gather, st), "hipEventRecord");
    if (!rc) rc = rt_assemble_async(c, &p, slab_rgb, d_img, st);
    if (!rc && out_lin) rc = rt_assemble_linear_async(c, &p, slab_lin, d_img_lin, st);
    if (!rc) rc = hip_ok(hipEventRecord(c->ev_asm, st), "hipEventRecord");
    HIPCHK(hipStreamSynchronize(st));
    if (rc) return rc;
    float a = 0, f = 0;
    HIPCHK(hipEventElapsedTime(&a, c->ev_gather, c->ev_asm));
    HIPCHK(hipEventElapsedTime(&f, c->ev0, c->ev_asm));
    ft.assemble_ms = a;
    ft.frame_ms = f;
  } else {
    if ((rc = grow(c, c->fb_gens, sizeof(uint64_t) * 2 * (size_t)p.width))) return rc;
    uint64_t* d_gens = (uint64_t*)c->fb_gens.p;
    HIPCHK(hipMemcpyAsync(d_gens, col_gens, sizeof(uint64_t) * 2 * (size_t)p.width, hipMemcpyHostToDevice, st));
    RenderArgs A{};
    A.S = c->scene;
    A.cam = *cam;
    A.W = p.width;
    A.H = p.height;
    A.spp = p.spp;
    A.max_depth = p.max_depth;
    A.flags = cull(c, p.flags);  // (RT_FLAG_REFERENCE_CULL)
    A.gens = d_gens;
    A.out_rgb = d_img;
    A.out_lin = d_img_lin;
    const void* fn = nullptr;
    size_t lds = 0;
    if (int rc = exact_launch(c, (p.flags & RT_FLAG_SHARED_LIBM) != 0, &fn, &lds)) return rc;
    int n_nodes = c->n_nodes;
    HIPCHK(hipEventRecord(c->ev0, st));
    void* args[] = {&A, &n_nodes};
    HIPCHK(hipLaunchKernel(fn, dim3(exact_blocks(p.width)), dim3(RT_BLOCK), args, lds, st));
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
  ft.kernel_ms[0] = ms;
  if (p.rng_mode == RT_RNG_EXACT) ft.frame_ms = ms;
  ft.device_allocs = c->allocs;
  c->last_frame = ft;
  return RT_OK;
}

namespace {
int render_counting(rt_ctx* c, const rt_camera* cam, const rt_render_params* pin, uint64_t* out_work, uint64_t* out_prof) {
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
  HIPCHK(hipMalloc(&work.p, sizeof(unsigned long long) * (16 + 64)));
  unsigned long long* d_work = (unsigned long long*)work.p;
  HIPCHK(hipMemsetAsync(d_work, 0, sizeof(unsigned long long) * (16 + 64), c->stream));
  rc = launch_philox(c, cam, &p, p.shard_rank, shards, (uint8_t*)slab_buf.p, nullptr, c->stream, d_work,
                     out_prof ? d_work + 16 : nullptr);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (rc) return rc;
  unsigned long long w[16 + 64];
  HIPCHK(hipMemcpy(w, d_work, sizeof w, hipMemcpyDeviceToHost));
  for (int i = 0; i < 16; ++i) out_work[i] = w[i];
  if (out_prof)
    for (int i = 0; i < 64; ++i) out_prof[i] = w[16 + i];
  return RT_OK;
}
}  // namespace

int rt_render_work(rt_ctx* c, const rt_camera* cam, const rt_render_params* pin, uint64_t out_work[16]) {
  return render_counting(c, cam, pin, out_work, nullptr);
}

int rt_render_step_profile(rt_ctx* c, const rt_camera* cam, const rt_render_params* pin, uint64_t out_work[16],
                           uint64_t out_prof[64]) {
  if (!out_prof) return invalid("null argument");
  return render_counting(c, cam, pin, out_work, out_prof);
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
  if ((flags & (RT_DEBUG_RESUMABLE | RT_DEBUG_WIDE | RT_DEBUG_QNODE)) && !c->replace_ok)
    return unsupported("rt_debug_closest_hits: the resumable walks need a world without media and frames");
  if ((flags & (RT_DEBUG_WIDE | RT_DEBUG_QNODE)) && !c->d_wnodes)
    return unsupported("rt_debug_closest_hits: no 4-wide tree for this world");
  if (n == 0) return RT_OK;
  DEVICE_SCOPE(c->device);
  DevBuf rays_buf, out_buf;
  HIPCHK(hipMalloc(&rays_buf.p, sizeof(double) * 7 * (size_t)n));
  HIPCHK(hipMalloc(&out_buf.p, sizeof(double) * 12 * (size_t)n));
  double* d_rays = (double*)rays_buf.p;
  double* d_out = (double*)out_buf.p;
  HIPCHK(hipMemcpy(d_rays, rays, sizeof(double) * 7 * (size_t)n, hipMemcpyHostToDevice));
  const int joint = !(cull(c, flags) & RT_FLAG_REFERENCE_CULL);
  const dim3 grid((n + RT_BLOCK - 1) / RT_BLOCK);
  if ((flags & RT_DEBUG_QNODE) && !c->d_qnodes)
    return unsupported("rt_debug_closest_hits: no quantised 4-wide tree for this world (spheres-only worlds)");
  if ((flags & RT_DEBUG_WIDE) && c->w8)  // (the 8-wide pairs: spheres-only worlds)
    hipLaunchKernelGGL(closest_hits<F_UV | F_WIDE | F_W8>, grid, dim3(RT_BLOCK), 0, c->stream, c->scene, d_rays, n,
                       tmin, tmax, seed, joint, 1, d_out);
  else if (flags & RT_DEBUG_QNODE)
    hipLaunchKernelGGL(closest_hits<F_UV | F_WIDE | F_QNODE>, grid, dim3(RT_BLOCK), 0, c->stream, c->scene, d_rays, n,
                       tmin, tmax, seed, joint, 1, d_out);
  else if (flags & RT_DEBUG_WIDE)
    hipLaunchKernelGGL(closest_hits<F_ALL | F_UV | F_WIDE>, grid, dim3(RT_BLOCK), 0, c->stream, c->scene, d_rays, n,
                       tmin, tmax, seed, joint, 1, d_out);
  else
    hipLaunchKernelGGL(closest_hits<F_ALL | F_UV | F_MIXW>, grid, dim3(RT_BLOCK), 0, c->stream, c->scene, d_rays, n,
                       tmin, tmax, seed, joint, (flags & RT_DEBUG_RESUMABLE) ? 1 : 0, d_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, d_out, sizeof(double) * 12 * (size_t)n, hipMemcpyDeviceToHost));
  return RT_OK;
}

int rt_debug_exact_trace(rt_ctx* c, const rt_camera* cam, const rt_render_params* pin, const uint64_t* col_gens,
                         int col, double* out, int cap, int* out_n) {
  if (!c || !cam || !pin || !col_gens || !out || !out_n || cap < 0) return invalid("rt_debug_exact_trace: null argument");
  rt_render_params p = *pin;
  p.shard_rank = 0;
  p.shard_count = 1;
  int rc = check_params(&p);
  if (rc) return rc;
  if (p.rng_mode != RT_RNG_EXACT) return invalid("rt_debug_exact_trace: tier A only");
  if (col < 0 || col >= p.width) return invalid("rt_debug_exact_trace: column out of range");
  if (!c->has_scene) {
    rt::set_error("rt_debug_exact_trace: no scene uploaded");
    return RT_E_STATE;
  }
  DEVICE_SCOPE(c->device);
  const long long npx = (long long)p.width * p.height;
  DevBuf img, gens, tr, trn;
  HIPCHK(hipMalloc(&img.p, (size_t)npx * 3));
  HIPCHK(hipMalloc(&gens.p, sizeof(uint64_t) * 2 * (size_t)p.width));
  HIPCHK(hipMalloc(&tr.p, sizeof(double) * 10 * (size_t)std::max(1, cap)));
  HIPCHK(hipMalloc(&trn.p, sizeof(int)));
  HIPCHK(hipMemcpy(gens.p, col_gens, sizeof(uint64_t) * 2 * (size_t)p.width, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(trn.p, 0, sizeof(int)));
  RenderArgs A{};
  A.S = c->scene;
  A.cam = *cam;
  A.W = p.width;
  A.H = p.height;
  A.spp = p.spp;
  A.max_depth = p.max_depth;
  A.flags = cull(c, p.flags);
  A.gens = (uint64_t*)gens.p;
  A.out_rgb = (uint8_t*)img.p;
  A.trace = (double*)tr.p;
  A.trace_n = (int*)trn.p;
  A.trace_col = col;
  A.trace_cap = cap;
  const void* fn = nullptr;
  size_t lds = 0;
  if (int rc = exact_launch(c, (p.flags & RT_FLAG_SHARED_LIBM) != 0, &fn, &lds)) return rc;
  int n_nodes = c->n_nodes;
  void* args[] = {&A, &n_nodes};
  HIPCHK(hipLaunchKernel(fn, dim3(exact_blocks(p.width)), dim3(RT_BLOCK), args, lds, c->stream));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out_n, trn.p, sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(out, tr.p, sizeof(double) * 10 * (size_t)std::min(*out_n, cap), hipMemcpyDeviceToHost));
  return RT_OK;
}

int rt_debug_probe(rt_ctx* c, const rt_camera* cam, int op, const double* in, int n, uint64_t seed, double* out) {
  if (!c || !in || !out || n < 0 || op < 0 || op > RT_PROBE_BOX || (op == 4 && !cam)) return invalid("rt_debug_probe: bad argument");
  if (!c->has_scene) {
    rt::set_error("rt_debug_probe: no scene uploaded");
    return RT_E_STATE;
  }
  if (n == 0) return RT_OK;
  // ids the device indexes with come from the caller: check them here (an out-of-range id would be
  // an out-of-bounds device read, not an error)
  auto id_ok = [](double x, int count) { return std::isfinite(x) && x >= 0 && x < count && x == std::floor(x); };
  for (int i = 0; i < n; ++i) {
    const double* q = in + (size_t)kProbeIn[op] * i;
    if (op == RT_PROBE_SCATTER && !id_ok(q[17], c->n_materials))
      return invalid("rt_debug_probe: scatter record " + std::to_string(i) + " has a material id out of range");
    if (op == RT_PROBE_TEXTURE && !id_ok(q[0], c->n_textures))
      return invalid("rt_debug_probe: texture record " + std::to_string(i) + " has a texture id out of range");
  }
  if (op == RT_PROBE_HTBL_RANDOM && c->scene.lights < 0)
    return invalid("rt_debug_probe: the scene has no lights tree");
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
  if (!c || !x || !y || !out || n < 0 || op < 0 || op > 17) return invalid("rt_debug_math: bad argument");
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
