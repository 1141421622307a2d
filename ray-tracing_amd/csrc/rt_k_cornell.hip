// rt_k_cornell.hip — render kernels of the Cornell-like variant (rects, instance chains, lights; config 3): one translation unit per variant, so
// that the variants compile in parallel (rt_kernels.h).
// The Philox key opaque per block (RT_PHILOX_OPAQUE_KEY, rt_device.h; with the cold-branch hints, on everywhere): C3 at 300 spp 98.3-98.7 -> 97.2-97.6 ms, same images (round 6).
#define RT_PHILOX_OPAQUE_KEY 1
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_cornell(int loop, bool lds, int w, bool count, bool leaf_lds) {
  return pick<kVarCornell>(loop, lds, w, count, leaf_lds);
}
}  // namespace rt
