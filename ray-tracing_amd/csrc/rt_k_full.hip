// rt_k_full.hip — render kernels of the full variant (media, instance frames, textures, motion) with
// light sampling: one translation unit per variant, so that the variants compile in parallel
// (rt_kernels.h).
#include "rt_kernels.h"

namespace rt {
const void* philox_kernel_full(int loop, bool lds, int w, bool count) { return pick_full<kVarFull>(loop, lds, w, count); }
}  // namespace rt
