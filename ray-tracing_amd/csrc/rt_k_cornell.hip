// rt_k_cornell.hip — render kernels of the Cornell-like variant (rects, instance chains, lights; config 3): one translation unit per variant, so
// that the variants compile in parallel (rt_kernels.h).
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_cornell(int loop, bool lds, int w, bool count, bool leaf_lds) {
  return pick<kVarCornell>(loop, lds, w, count, leaf_lds);
}
}  // namespace rt
