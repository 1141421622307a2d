// rt_k_spheres.hip — render kernels of the spheres-only variant (configs 1, 2, 5): one translation unit per variant, so
// that the variants compile in parallel (rt_kernels.h).
// The Philox key made opaque per block (RT_PHILOX_OPAQUE_KEY, rt_device.h): the LDS-staged 4-wave kernel (C2)
// 108 -> 100 B/lane of scratch, SGPR spills 211 -> 145, C2 135.9-136.2 -> 135.3-135.7 ms (and with the cold-branch
// hints 134.7-134.9); C5's kernel is 0.5 % slower with it, so it has a unit of its own (rt_k_spheres_global.hip).
#define RT_PHILOX_OPAQUE_KEY 1
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_spheres(int loop, bool lds, int w, bool count, bool leaf_lds, bool q, bool w8) {
  return pick<kVarSpheres>(loop, lds, w, count, leaf_lds, q, w8);
}
}  // namespace rt
