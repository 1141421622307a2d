// rt_k_full_dark.hip — render kernels of the full variant without light sampling (lights Unhittable:
// next_week_final (config 4) and the textured scenes): one translation unit per variant (rt_kernels.h).
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_full_dark(int loop, bool lds, int w, bool count) {
  return pick_full<kVarFullDark>(loop, lds, w, count);
}
}  // namespace rt
