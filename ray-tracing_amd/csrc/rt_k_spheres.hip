// rt_k_spheres.hip — render kernels of the spheres-only variant (configs 1, 2, 5): one translation unit per variant, so
// that the variants compile in parallel (rt_kernels.h).
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_spheres(int loop, bool lds, int w, bool count, bool leaf_lds, bool q, bool w8) {
  return pick<kVarSpheres>(loop, lds, w, count, leaf_lds, q, w8);
}
}  // namespace rt
