// rt_k_full_dark.hip — render kernels of the full variant without light sampling (lights Unhittable:
// next_week_final (config 4) and the textured scenes): one translation unit per variant (rt_kernels.h).
// The Philox key opaque per block (RT_PHILOX_OPAQUE_KEY, rt_device.h; with the cold-branch hints, on everywhere): C4 at 100 spp 141.6-149.2 -> 141.2-145.9 ms (noisy), same images (round 6).
#define RT_PHILOX_OPAQUE_KEY 1
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_full_dark(int loop, bool lds, int w, bool count) {
  return pick_full<kVarFullDark>(loop, lds, w, count);
}
}  // namespace rt
